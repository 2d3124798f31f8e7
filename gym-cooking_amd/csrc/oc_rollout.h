// oc_rollout.h -- one navigation-planner rollout row, scalar per lane.
//
// A row is (state, planner configuration, action).  Everything here follows the reference
// planner as restated in include/oc_engine.h's rollout section:
//   level0()        E2E_BRTDP._configure_planner_level, LEVEL0   e2e_brtdp.py:389-406
//   interact()      utils/interact.py:4-89 (the same rules as ocsw::step4, one env)
//   action_legal()  get_actions / get_single_actions      e2e_brtdp.py:151-206, nav utils.py:55-90
//   is_goal()       _define_goal_state                   e2e_brtdp.py:435-566
//   lower_bound()   get_lower_bound_for_subtask_given_objs  overcooked_environment.py:480-664,
//                   World.get_lower_bound_between(_helper), check_bound  world.py:115-283
// The reachability graph of the static level (world.py:67-108) is precomputed by
// build_roll_level() as a compact all-pairs distance table (u8, 0xFF = no path; u16, 0xFFFF = no
// path, when some BFS distance reaches 255: a maze kitchen's long corridors, round 6).  The static
// tables of a level (tile classes, graph node ids, Cutboard / Delivery lists, distances) form
// one byte blob, sized per level (the tables + nnodes^2 distance bytes).  A narrow level's
// kernels stage all of it in LDS when its graph has at most kMaxNodes nodes: a 7x7 kitchen's blob
// is ~7 KB, the largest ~134 KB, which they get as dynamic LDS past the default 64 KB (gfx950 has
// 160 KB per CU).  A larger graph (round 5: a narrow level of more than kMaxNodes nodes, e.g. a
// 255-cell kitchen dense with counter islands) and every wide level (more than 255 cells) stage
// the tables in front of the distances only and read the distance table from device memory (L2;
// RollLevel.dist_global, the planner kernels' GD instantiation), so a narrow graph may have every
// node its cells can make (5 x 255) and a wide one up to kMaxNodesWide (a 1,024-cell kitchen's
// 5,120 approach nodes at most, 26 MB).  Distances and bounds are exact in fp32 (integers and
// halves < 2^9).  (Round 5 also measured a table of the distances between Floor squares only --
// an approach node is a leaf one edge from its Floor -- with no node limit: 10-20 % slower C5
// kernels at the same outputs, profiles/r05/ab/; not kept.)
//
// The includer defines __host__ / __device__ (HIP, or empty for the host test harness).
#pragma once

#include <stdint.h>

#include <vector>

// Every row function is force-inlined: a GPU call spills the caller's live registers to
// scratch (the bound walk was being emitted as s_swappc calls with ~100 B of scratch per lane).
#define OC_RH __host__ __device__ inline __attribute__((always_inline))
#define OC_RL __attribute__((always_inline))

namespace ocro {

template <bool B, class T, class F>
struct ConditionalT {
    using type = T;
};
template <class T, class F>
struct ConditionalT<false, T, F> {
    using type = F;
};

constexpr int kMaxCells = 255;      // narrow levels: cell ids are bytes, 0xFF = dead / none
constexpr int kMaxCellsWide = 1024;  // wide levels (more than 255 cells): u16 cell ids, 0xFFFF dead
// compact reachability-graph node ids are u16 (kNoNode = none); at most kMaxNodes nodes keep a
// block's LDS (blob + 64 configurations + the kernels' own) within the 160 KB of a gfx950 CU,
// a larger graph's distances stay in device memory; distances are bytes (0xFF = no path), or
// u16 (0xFFFF = no path) in device memory when some BFS distance reaches 255 (RollLevel.dist16;
// round 5 refused such a graph)
constexpr int kMaxNodes = 360;  // 360^2 + the other tables + the compacted likelihood's 18 KB < 160 KB
constexpr int kMaxSqBytes = 8192;  // the node-to-square table is built when nnodes x cells fits this
constexpr size_t kMaxPairBytes = (size_t)4 << 20;  // the agent-pair table: nnodes^2 x cells x 4 bytes
constexpr int kMaxNodesNarrow = 5 * kMaxCells;    // narrow levels: every node 255 cells can make
constexpr int kMaxNodesWide = 5 * kMaxCellsWide;  // wide levels: the distances stay in device memory
constexpr uint8_t kNone = 0xFF;
constexpr uint16_t kNoNode = 0xFFFF;
constexpr int kFloor = 0, kCounter = 1, kCutboard = 2, kDelivery = 3;  // OC_TILE_*
constexpr int kNoop = 4;
constexpr int kDX[5] = {0, 0, -1, 1, 0}, kDY[5] = {1, -1, 0, 0, 0};  // World.NAV_ACTIONS + (0, 0)

// Static level tables, one byte blob (offsets in RollLevel, set by build_roll_level):
//   tile_off   [TC] tile class per cell (TC = 256 for a narrow level: cell ids >= W*H, the dead
//              slot 0xFF among them, read Counter; the cell count rounded up to 4 for a wide one)
//   xy_off     u16 [C] x | y << 8 of each cell (C = the cell count rounded up to 4; the bound's
//              Manhattan terms read it instead of dividing by W: round 5)
//   node_off   u16 [C * 5] graph node of (cell, approach), approach 4 = (0, 0)
//   cut_off    Cutboard cells in scan order (L.ncut; u8 narrow, u16 wide; padded to 4 bytes)
//   deliv_off  Delivery cells in scan order (L.ndeliv; likewise)
//   man_off    u16 [2][C] Manhattan distance from a cell to the nearest Cutboard (row 0) /
//              Delivery (row 1) square (the two-agent static bound's B term; round 6)
//   dmin_off   [2][nnodes] the distance from a node to the nearest Cutboard (row 0) / Delivery
//              (row 1) approach node, 0xFF = none reachable (u16 and 0xFFFF with dist16)
//   dist_off   [nnodes][nnodes] BFS distances (a wide level stages the blob up to here; u16
//              entries with dist16)
//   sq_off     [nnodes][cells] node-to-square distances: min over the square's approach nodes
//              (its own node for a Floor square), 0xFF = none reachable; only on a small narrow
//              level whose blob stays in LDS (kMaxSqBytes), where the single-agent Merge bound
//              reads it once per (A approach, B square) instead of walking B's approaches
//   pair_off   u32 [nnodes][nnodes][cells] after everything the kernels stage (device memory
//              only, never in LDS): for agent nodes (u0, u1) and a square, the two-agent bound's
//              per-type minima over the square's approach nodes (byte 0: u0 strictly nearer, byte
//              1: u1 strictly nearer, byte 2: a tie; 0xFF = no such approach), an unreachable
//              distance counted as the perimeter as the walk does; only on a narrow level with LDS
//              distances, a perimeter below 255 and at most kMaxPairBytes of entries (round 6)
// Only the tile table's size is fixed (256 entries on a narrow level); the others follow the
// level's cell count (round 6; before, every per-cell table had 256 entries on a narrow level).

struct RollLevel {  // scalars (kernel argument); the tables are in the blob
    int32_t W, H, perimeter, nnodes;
    int32_t ncut, ndeliv;
    int32_t enc;       // item mask encoding (OC_ENC_*)
    int32_t dmin_off;  // blob offset of the nearest-Cutboard / nearest-Delivery distance rows
    int32_t tile_off, node_off, cut_off, deliv_off, dist_off;
    int32_t xy_off;    // u16 x | y << 8 per cell
    int32_t man_off;   // u16 [2][man_stride]: Manhattan distance from a cell to the nearest Cutboard
                       // (row 0) / Delivery (row 1) square
    int32_t man_stride;
    int32_t wide;     // u16 cell ids (W * H > 255)
    int32_t blob_bytes;  // the blob's size (a multiple of 4)
    int32_t lds_bytes;   // what the kernels stage in LDS: all of it, or up to dist_off (dist_global)
    int32_t dist_global; // the distance table is read from device memory: a wide level, or a narrow
                         // one of more than kMaxNodes nodes (the planner kernels' GD instantiation)
    int32_t dist16;      // the distance and nearest-side tables are u16 (some BFS distance >= 255);
                         // implies dist_global (round 6)
    int32_t sq_off;      // blob offset of the node-to-square table ([nnodes][cells] u8, the distance
                         // from a node to the nearest approach node of a square), 0 = none (round 6)
    int32_t sq_cells;    // its row length (the level's cell count)
    int32_t pair_off;    // blob offset of the agent-pair table (device memory only), 0 = none
};

// A wide level's reset template (oc_reset_wide_kernel).
struct StepLevel {
    int32_t done_cell;  // first Delivery in scan order (done() reads only it, overcooked_environment.py:349)
    int32_t max_T;      // 0 = no limit
    int32_t ngoals;
    uint8_t goal[4];    // Deliver goal masks
    uint8_t spawn_x[4], spawn_y[4];
    uint16_t item_cell[16];  // the template's item slots (dead past the level's items)
    uint8_t item_mask[16];
};

struct Sub {  // oc_subtask, device copy
    int32_t kind, n;
    uint8_t agent[2], start[2], goal, count, level, pad;
};

// One row's state, packed so that run-time slot / agent indices are shifts, not memory:
// agent a in byte a of x, y, h (h = held slot or kNone); slot j's mask in byte j % 8 of word
// j / 8 of mask, its cell in byte j % 8 of word j / 8 of loc (narrow) or in the 16-bit field
// j % 4 of word j / 4 (WIDE); a run-time j picks the word with selects on register values.
template <int K, bool WIDE = false>
struct RowT {
    static constexpr int NW = (K + 7) / 8;          // mask words
    static constexpr int LPW = WIDE ? 4 : 8;        // cells per location word
    static constexpr int NL = (K + LPW - 1) / LPW;  // location words
    static constexpr int kLocBits = WIDE ? 16 : 8;
    static constexpr uint32_t kDead = WIDE ? 0xFFFFu : 0xFFu;  // OC_LOC_DEAD
    uint32_t x = 0, y = 0, h = 0;
    uint64_t loc[NL] = {}, mask[NW] = {};
    static OC_RH uint32_t b32(uint32_t w, int i) { return (w >> (8 * i)) & 0xFFu; }
    static OC_RH void s32(uint32_t& w, int i, uint32_t v) { w = (w & ~(0xFFu << (8 * i))) | (v << (8 * i)); }
    // word i of w[N], selected on register values: folded into a select of addresses the
    // compiler turns the words into a scratch array with a run-time offset
    template <int N>
    static OC_RH uint64_t wsel(const uint64_t (&w)[N], int i) {
        if constexpr (N == 1) {
            return w[0];
        } else {
            uint64_t r = w[0];
#pragma unroll
            for (int q = 1; q < N; ++q) {
                uint64_t v = w[q];
#if defined(__HIP_DEVICE_COMPILE__)
                asm("" : "+v"(r), "+v"(v));
#endif
                r = i == q ? v : r;
            }
            return r;
        }
    }
    template <int N>
    static OC_RH void wput(uint64_t (&w)[N], int i, int shift, uint64_t field, uint64_t v) {
#pragma unroll
        for (int q = 0; q < N; ++q)
            if (i == q) w[q] = (w[q] & ~(field << shift)) | (v << shift);
    }
    OC_RH int ax(int a) const { return (int)b32(x, a); }
    OC_RH int ay(int a) const { return (int)b32(y, a); }
    OC_RH int ah(int a) const { return (int)b32(h, a); }
    OC_RH int il(int j) const { return (int)((wsel(loc, j / LPW) >> (kLocBits * (j % LPW))) & kDead); }
    OC_RH int im(int j) const { return (int)((wsel(mask, j >> 3) >> (8 * (j & 7))) & 0xFFu); }
    OC_RH void set_loc(int j, uint32_t v) { wput(loc, j / LPW, kLocBits * (j % LPW), (uint64_t)kDead, (uint64_t)v); }
    OC_RH void set_mask(int j, uint32_t v) { wput(mask, j >> 3, 8 * (j & 7), 0xFFull, (uint64_t)v); }
};

// Some lane of the wave (the active ones) has p: a wave-uniform trip count for the bound walks
// (every lane of the host build is its own wave).
OC_RH bool wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ballot(p) != 0ull;
#else
    return p;
#endif
}

// a * b for operands and product below 2^24: v_mul_u32_u24 (full rate) on the device, where the
// plain 32-bit multiply is quarter rate
OC_RH uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul24(a, b);
#else
    return a * b;
#endif
}

// byte v occurs in one of the four bytes of w
OC_RH bool has_byte(uint32_t w, uint32_t v) {
    const uint32_t x = w ^ (v * 0x01010101u);
    return ((x - 0x01010101u) & ~x & 0x80808080u) != 0u;
}

// byte / u16 v occurs in one of the fields of w (the AgentCounter cells of a Level-0 view)
OC_RH bool has_u16(uint64_t w, uint32_t v) {
    const uint64_t x = w ^ ((uint64_t)v * 0x0001000100010001ull);
    return ((x - 0x0001000100010001ull) & ~x & 0x8000800080008000ull) != 0ull;
}

// ---- host: level tables ----------------------------------------------------------------------
// Builds the reachability graph of make_reachability_graph (world.py:67-108) and its BFS
// distances into `blob_v` (resized to the blob).  Returns the node count, or -1 when the level
// has more cells than its layout takes (255 narrow, kMaxCellsWide wide).  The distance table is
// u8 while every BFS distance is below 255, u16 otherwise (dist16).
inline int build_roll_level(RollLevel& L, std::vector<uint8_t>& blob_v, int W, int H, const uint8_t* tiles, int enc) {
    L.W = W;
    L.enc = enc;
    L.H = H;
    L.perimeter = 2 * (W + H);
    L.ncut = L.ndeliv = 0;
    L.nnodes = -1;
    L.dist16 = 0;
    L.sq_off = 0;
    L.sq_cells = 0;
    L.pair_off = 0;
    const int cells = W * H;
    L.wide = cells > kMaxCells ? 1 : 0;
    if (cells > kMaxCellsWide) return -1;
    // the tile table covers every cell id a row can hold (a narrow level's 0xFF dead slot
    // included: 256 entries); the other per-cell tables only the level's cells (round 6: a 7x7
    // kitchen's fixed tables shrink from 4.9 to 1.1 KB, and every block stages them)
    const int TC = L.wide ? (cells + 3) & ~3 : 256, C = (cells + 3) & ~3, lb = L.wide ? 2 : 1;
    const int max_nodes = L.wide ? kMaxNodesWide : kMaxNodesNarrow;
    int ncut = 0, ndeliv = 0;
    for (int c = 0; c < cells; ++c) {
        ncut += tiles[c] == kCutboard;
        ndeliv += tiles[c] == kDelivery;
    }
    L.tile_off = 0;
    L.xy_off = TC;
    L.node_off = L.xy_off + 2 * C;
    L.cut_off = L.node_off + 2 * C * 5;
    L.deliv_off = L.cut_off + ((lb * ncut + 3) & ~3);
    L.man_off = L.deliv_off + ((lb * ndeliv + 3) & ~3);
    L.man_stride = C;
    L.dmin_off = L.man_off + 2 * 2 * C;
    blob_v.assign((size_t)L.dmin_off, 0);  // grown below once the node count is known
    uint8_t* blob = blob_v.data();
    uint8_t* tile = blob + L.tile_off;
    uint16_t* node = (uint16_t*)(blob + L.node_off);
    auto put_list = [&](int off, int i, int c) {
        if (L.wide) ((uint16_t*)(blob + off))[i] = (uint16_t)c;
        else blob[off + i] = (uint8_t)c;
    };
    for (int c = 0; c < TC; ++c) {
        tile[c] = c < cells ? tiles[c] : (uint8_t)kCounter;
        if (c < cells && tiles[c] == kCutboard) put_list(L.cut_off, L.ncut++, c);
        if (c < cells && tiles[c] == kDelivery) put_list(L.deliv_off, L.ndeliv++, c);
    }
    for (int i = 0; i < C * 5; ++i) node[i] = kNoNode;
    for (int c = 0; c < C; ++c)
        ((uint16_t*)(blob + L.xy_off))[c] = c < cells ? (uint16_t)((c % W) | ((c / W) << 8)) : (uint16_t)0;
    // min over a static B side of manhattan(A, B) (world.py:215, 242-244: the two-agent bound's
    // B term), per A cell; 0x7FFF where the side is empty (the bound returns before reading it)
    for (int side = 0; side < 2; ++side) {
        const int off = side == 0 ? L.cut_off : L.deliv_off, nb = side == 0 ? L.ncut : L.ndeliv;
        uint16_t* man = (uint16_t*)(blob + L.man_off) + side * C;
        for (int c = 0; c < C; ++c) {
            int best = 0x7FFF;
            for (int i = 0; c < cells && i < nb; ++i) {
                const int b = L.wide ? ((const uint16_t*)(blob + off))[i] : blob[off + i];
                const int dx = c % W - b % W, dy = c / W - b / W;
                const int m = (dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy);
                best = m < best ? m : best;
            }
            man[c] = (uint16_t)best;
        }
    }
    int n = 0;
    auto clampx = [&](int v) { return v < 0 ? 0 : (v > W - 1 ? W - 1 : v); };
    auto clampy = [&](int v) { return v < 0 ? 0 : (v > H - 1 ? H - 1 : v); };
    for (int c = 0; c < cells; ++c) {
        const int x = c % W, y = c / W;
        const bool coll = tiles[c] != kFloor;
        if (!coll) {
            if (n >= max_nodes) return -1;
            node[c * 5 + 4] = (uint16_t)n++;
        }
        for (int d = 0; d < 4; ++d) {
            const int nc = clampy(y + kDY[d]) * W + clampx(x + kDX[d]);
            if (coll && tiles[nc] == kFloor) {
                if (n >= max_nodes) return -1;
                node[c * 5 + d] = (uint16_t)n++;
            }
        }
    }
    // adjacency (undirected): floor-floor, and a collidable square's approach node with the
    // floor it is approached from
    static const int opp[4] = {1, 0, 3, 2};
    std::vector<uint16_t> adj_v((size_t)n * 8);
    std::vector<int> deg((size_t)n, 0), q((size_t)n);
    auto adj = [&](int u, int k) -> uint16_t& { return adj_v[(size_t)u * 8 + k]; };
    auto link = [&](int u, int v) {
        if (u == kNoNode || v == kNoNode || u == v) return;
        for (int k = 0; k < deg[u]; ++k)
            if (adj(u, k) == v) return;
        adj(u, deg[u]++) = (uint16_t)v;
        adj(v, deg[v]++) = (uint16_t)u;
    };
    for (int c = 0; c < cells; ++c) {
        const int x = c % W, y = c / W;
        const bool coll = tiles[c] != kFloor;
        for (int d = 0; d < 4; ++d) {
            const int nc = clampy(y + kDY[d]) * W + clampx(x + kDX[d]);
            const bool ncoll = tiles[nc] != kFloor;
            if (coll && !ncoll) link(node[c * 5 + d], node[nc * 5 + 4]);
            else if (!coll && ncoll) link(node[c * 5 + 4], node[nc * 5 + opp[d]]);
            else if (!coll && !ncoll) link(node[c * 5 + 4], node[nc * 5 + 4]);
        }
    }
    // all-pairs BFS into u16 rows first: a distance of 255 or more makes the tables u16
    std::vector<uint16_t> d16((size_t)n * n, (uint16_t)0xFFFF);
    int dmax = 0;
    for (int s = 0; s < n; ++s) {
        uint16_t* row = d16.data() + (size_t)s * n;
        int qh = 0, qt = 0;
        row[s] = 0;
        q[qt++] = s;
        while (qh < qt) {
            const int u = q[qh++];
            for (int k = 0; k < deg[u]; ++k) {
                const int v = adj(u, k);
                if (row[v] == 0xFFFF) {
                    row[v] = (uint16_t)(row[u] + 1);
                    dmax = row[v] > dmax ? row[v] : dmax;
                    q[qt++] = v;
                }
            }
        }
    }
    L.dist16 = dmax >= (int)kNone ? 1 : 0;
    const int db = L.dist16 ? 2 : 1;  // bytes per distance entry
    const uint32_t none = L.dist16 ? 0xFFFFu : kNone;
    L.dist_off = (L.dmin_off + 2 * n * db + 3) & ~3;
    blob_v.resize((size_t)L.dist_off + (size_t)n * n * db + 4, 0);
    blob = blob_v.data();
    tile = blob + L.tile_off;
    node = (uint16_t*)(blob + L.node_off);
    auto put = [&](size_t off, size_t i, uint32_t v) {
        if (L.dist16) ((uint16_t*)(blob + off))[i] = (uint16_t)v;
        else blob[off + i] = (uint8_t)v;
    };
    for (size_t i = 0; i < (size_t)n * n; ++i) put((size_t)L.dist_off, i, d16[i] == 0xFFFF ? none : d16[i]);
    // Chop and Deliver have a static B side (every Cutboard / every Delivery square, from any
    // side it is approached from): the single-agent bound's min over B of dist(A node, B node)
    // is this per-node table (world.py:175-189 evaluated once per level)
    for (int side = 0; side < 2; ++side) {
        const int off = side == 0 ? L.cut_off : L.deliv_off;
        const int nc = side == 0 ? L.ncut : L.ndeliv;
        for (int v = 0; v < n; ++v) {
            uint32_t best = none;
            for (int i = 0; i < nc; ++i) {
                const int cell = L.wide ? ((const uint16_t*)(blob + off))[i] : blob[off + i];
                for (int d = 0; d < 4; ++d) {
                    const int b = node[cell * 5 + d];
                    if (b == kNoNode) continue;
                    const uint32_t dd = d16[(size_t)v * n + b];
                    if (dd != 0xFFFF && dd < best) best = dd;
                }
            }
            put((size_t)L.dmin_off, (size_t)side * n + v, best);
        }
    }
    L.nnodes = n;
    L.blob_bytes = (int32_t)((L.dist_off + (size_t)n * n * db + 3) & ~(size_t)3);
    L.dist_global = L.wide || n > kMaxNodes || L.dist16 ? 1 : 0;
    if (!L.dist_global && (size_t)n * cells <= (size_t)kMaxSqBytes) {
        // node-to-square distances (World.get_lower_bound_between_helper's min over B's approach
        // nodes, world.py:175-189, for every (node, square)); a collidable square's approaches are
        // its approach-0..3 nodes, a Floor square's its own node (the static graph; a square that
        // is an AgentCounter in a Level-0 view is caught at the lookup)
        L.sq_off = L.blob_bytes;
        L.sq_cells = cells;
        blob_v.resize((size_t)L.sq_off + (size_t)n * cells + 4, 0);
        blob = blob_v.data();
        node = (uint16_t*)(blob + L.node_off);
        uint8_t* sq = blob + L.sq_off;
        for (int v = 0; v < n; ++v)
            for (int c = 0; c < cells; ++c) {
                uint32_t best = kNone;
                for (int d = 0; d < 5; ++d) {
                    const int b = node[c * 5 + d];
                    if (b == kNoNode || (d == 4) != (tiles[c] == kFloor)) continue;
                    const uint32_t dd = d16[(size_t)v * n + b];
                    if (dd != 0xFFFF && dd < best) best = dd;
                }
                sq[(size_t)v * cells + c] = (uint8_t)best;
            }
        L.blob_bytes = (int32_t)((L.sq_off + (size_t)n * cells + 3) & ~(size_t)3);
    }
    L.lds_bytes = L.dist_global ? L.dist_off : L.blob_bytes;
    if (!L.dist_global && L.perimeter < 255 && (size_t)n * n * cells * 4 <= kMaxPairBytes) {
        // the agent-pair table (device memory): side()'s per-type minima of helper_n's two-agent
        // bound, for every (u0, u1, square), over the approach set approaches() walks on the
        // static graph (a Floor square's own node, else its four approach nodes)
        L.pair_off = L.blob_bytes;
        blob_v.resize((size_t)L.pair_off + (size_t)n * n * cells * 4, 0);
        blob = blob_v.data();
        node = (uint16_t*)(blob + L.node_off);
        uint32_t* pt = (uint32_t*)(blob + L.pair_off);
        const uint32_t per = (uint32_t)L.perimeter;
        for (int c = 0; c < cells; ++c) {
            int vs[4], nv = 0;
            if (node[c * 5 + 4] != kNoNode) vs[nv++] = node[c * 5 + 4];
            else
                for (int q = 0; q < 4; ++q) vs[nv++] = node[c * 5 + q];
            for (int u0 = 0; u0 < n; ++u0)
                for (int u1 = 0; u1 < n; ++u1) {
                    uint32_t M[3] = {0xFFu, 0xFFu, 0xFFu};
                    for (int i = 0; i < nv; ++i) {
                        const int v = vs[i];
                        const uint32_t d1 = v == kNoNode ? 0xFFFFu : d16[(size_t)u0 * n + v];
                        const uint32_t d2 = v == kNoNode ? 0xFFFFu : d16[(size_t)u1 * n + v];
                        const uint32_t b1 = d1 == 0xFFFFu ? per : d1, b2 = d2 == 0xFFFFu ? per : d2;
                        const uint32_t m = b1 < b2 ? b1 : b2, t = b1 < b2 ? 0 : (b2 < b1 ? 1 : 2);
                        if (m < M[t]) M[t] = m;
                    }
                    pt[((size_t)u0 * n + u1) * cells + c] = M[0] | M[1] << 8 | M[2] << 16;
                }
        }
        L.blob_bytes = (int32_t)(L.pair_off + (size_t)n * n * cells * 4);
    }
    blob_v.resize((size_t)L.blob_bytes, 0);
    return n;
}

// ---- row logic ----------------------------------------------------------------------------
// LEAN (the likelihood kernels, whose compacted form sits at 122 of the 128 VGPRs that keep 4
// waves per SIMD): the bound walk reads a square's tile before its approach nodes, as before
// round 6, instead of all five node reads at once (which keeps more values live).
// DG (the planner kernels' device-memory-distance instantiation, and the host builds): the level
// may have u16 distance tables (RollLevel.dist16, a wave-uniform branch at each read); without DG
// the tables are u8 (a dist16 level always takes the device-memory path).
template <int A, int K, bool WIDE = false, bool LEAN = false, bool DG = false>
struct RowOps {
    using Row = RowT<K, WIDE>;
    using AcT = typename ConditionalT<WIDE, uint64_t, uint32_t>::type;
    static constexpr int kDead = (int)Row::kDead;
    static constexpr AcT kNoAc = ~(AcT)0;
    const RollLevel& L;
    const uint8_t* T;       // the level's table blob (LDS on the device)
    const uint8_t* D;       // its distance table: in T (narrow), in device memory (wide)
    AcT ac = kNoAc;         // AgentCounter cells of this row's Level-0 view, one per byte (narrow) or
                            // u16 field (wide), all ones = none
    const uint32_t* PT = nullptr;  // the agent-pair table (device memory; L.pair_off), or none:
                                   // the kernel that reads it sets it (round 6)
    uint32_t active = 0;    // bit a: agent a is a subtask agent
    uint32_t blockers = 0;  // bit a: agent a's cell may not be moved into (get_single_actions)

    OC_RH RowOps(const RollLevel& l, const uint8_t* blob) : L(l), T(blob), D(blob + l.dist_off) {}
    OC_RH RowOps(const RollLevel& l, const uint8_t* blob, const uint8_t* dist) : L(l), T(blob), D(dist) {}

    OC_RH int static_tile(int cell) const { return T[L.tile_off + cell]; }
    OC_RH bool is_ac(int cell) const {
        if constexpr (WIDE) return has_u16(ac, (uint32_t)cell);
        else return has_byte(ac, (uint32_t)cell);
    }
    OC_RH void set_ac(int a, uint32_t cell) {
        if constexpr (WIDE) ac = (ac & ~(0xFFFFull << (16 * a))) | ((uint64_t)cell << (16 * a));
        else Row::s32(ac, a, cell);
    }
    OC_RH int tile(int cell) const { return is_ac(cell) ? kCounter : T[L.tile_off + cell]; }
    OC_RH int list_cell(int off, int i) const {  // Cutboard / Delivery list entry
        if constexpr (WIDE) return ((const uint16_t*)(T + off))[i];
        else return T[off + i];
    }
    OC_RH int cell(int x, int y) const { return (int)mul24((uint32_t)y, (uint32_t)L.W) + x; }
    OC_RH uint32_t xy(int c) const { return ((const uint16_t*)(T + L.xy_off))[c]; }  // x | y << 8
    OC_RH int agent_cell(const Row& r, int a) const { return cell(r.ax(a), r.ay(a)); }

    // level0: agents outside the subtask freeze into AgentCounters; their items leave.
    // Returns true where the reference raises: a second removed agent on an already replaced
    // Floor (World.remove asserts, world.py:307-315).
    OC_RH bool level0(Row& r, const Sub& s) {
        active = 0;
        bool raised = false;
        for (int i = 0; i < s.n; ++i) active |= 1u << s.agent[i];
        if (s.level != 0) {  // Level 1: every agent stays in sim_agents, nothing is removed
            blockers = (1u << A) - 1u;
            return false;
        }
        blockers = active;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            if ((active >> a) & 1u) continue;
            const int hh = r.ah(a);
            if (hh != kNone) {
                r.set_loc(hh, (uint32_t)kDead);
                r.set_mask(hh, 0);
                Row::s32(r.h, a, kNone);
            }
            const uint32_t c = (uint32_t)agent_cell(r, a);
            raised |= is_ac((int)c);
            set_ac(a, c);
        }
        return raised;
    }

    // the un-held item on a non-Floor square (at most one off Delivery), or -1
    OC_RH int item_at(const Row& r, int c) const {
        int o = -1;
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (r.il(j) == c) o = j;
        return o;
    }

    // Object predicates (core.py:176-241) in the level's mask encoding.  OC_ENC_COUNTS: 2-bit
    // T/L/O counts, 0x40 Plate, 0x80 Fresh (a single fresh food; merged objects are all-Chopped).
    OC_RH int ncontents(int m) const {
        return L.enc ? (m & 3) + ((m >> 2) & 3) + ((m >> 4) & 3) + ((m >> 6) & 1)
                     : __builtin_popcount((unsigned)m & 0x0Fu);
    }
    OC_RH bool deliverable(int m) const {
        return L.enc ? ncontents(m) >= 2 : ncontents(m) >= 2 && ((m & 7) & ~(m >> 4)) == 0;
    }
    OC_RH bool mergeable(int a, int b) const {
        const int u = a | b;
        return L.enc ? !(a & b & 0x40) && !(u & 0x80) : !(a & b & 8) && ((u & 7) & ~(u >> 4)) == 0;
    }
    OC_RH bool needs_chopped(int m) const {
        return L.enc ? (m & 0x80) != 0 : ncontents(m) == 1 && (m & 0x78) == 0;
    }
    OC_RH int merged(int a, int b) const { return L.enc ? a + b : a | b; }        // Object.merge
    OC_RH int chopped(int m) const { return L.enc ? m & 0x7F : m | ((m << 4) & 0x70); }  // Object.chop

    // The square agent a's action points at, clamped to the grid (interact's and get_single_
    // actions' World.inbounds), and its tile in the Level-0 view.  single_legal and interact
    // read the same square (interact moves no other agent and the AgentCounters are fixed), so
    // a row reads each subtask agent's tile once, all agents' reads together (round 6).
    struct Target {
        int x, y, c, t;
    };
    OC_RH Target target(const Row& r, int a, int code) const {
        Target g;
        const int k = code > kNoop ? kNoop : code;
        g.x = r.ax(a) + kDX[k];
        g.y = r.ay(a) + kDY[k];
        g.x = g.x < 0 ? 0 : (g.x > L.W - 1 ? L.W - 1 : g.x);
        g.y = g.y < 0 ? 0 : (g.y > L.H - 1 ? L.H - 1 : g.y);
        g.c = cell(g.x, g.y);
        g.t = tile(g.c);
        return g;
    }

    // interact(agent, world), play = False (utils/interact.py:4-89)
    OC_RH void interact(Row& r, int a, int code) const {
        if (code == kNoop) return;  // before the target's read, as the reference returns first
        interact(r, a, code, target(r, a, code));
    }
    OC_RH void interact(Row& r, int a, int code, const Target& g) const {
        if (code == kNoop) return;
        const int tx = g.x, ty = g.y, tc = g.c, t = g.t, h = r.ah(a);
        if (t == kFloor) {  // move_to: the held item follows
            Row::s32(r.x, a, (uint32_t)tx);
            Row::s32(r.y, a, (uint32_t)ty);
            if (h != kNone) r.set_loc(h, (uint32_t)tc);
        } else if (h != kNone) {
            const int hm = r.im(h);
            if (t == kDelivery) {
                if (deliverable(hm)) {
                    r.set_loc(h, (uint32_t)tc);
                    Row::s32(r.h, a, kNone);
                }
            } else {
                const int o = item_at(r, tc);
                if (o >= 0) {
                    if (mergeable(hm, r.im(o))) {  // the holder's item absorbs o
                        r.set_mask(h, (uint32_t)merged(hm, r.im(o)));
                        r.set_loc(o, (uint32_t)kDead);
                        r.set_mask(o, 0);
                    }
                } else if (t == kCutboard && needs_chopped(hm)) {
                    r.set_mask(h, (uint32_t)chopped(hm));
                } else {  // put down
                    r.set_loc(h, (uint32_t)tc);
                    Row::s32(r.h, a, kNone);
                }
            }
        } else if (t != kDelivery) {
            const int o = item_at(r, tc);
            if (o >= 0) {  // pick up: the item moves onto the agent
                Row::s32(r.h, a, (uint32_t)o);
                r.set_loc(o, (uint32_t)agent_cell(r, a));
            }
        }
    }

    // OvercookedEnvironment.is_collision (overcooked_environment.py:671-722): both execute
    OC_RH bool no_collision(const Row& r, int i, int j, int ci, int cj) const {
        const int lix = r.ax(i), liy = r.ay(i), ljx = r.ax(j), ljy = r.ay(j);
        int nix = lix + kDX[ci], niy = liy + kDY[ci], njx = ljx + kDX[cj], njy = ljy + kDY[cj];
        if (tile(cell(nix, niy)) != kFloor) { nix = lix; niy = liy; }
        if (tile(cell(njx, njy)) != kFloor) { njx = ljx; njy = ljy; }
        if (nix == njx && niy == njy) return false;  // every same-target branch blocks someone
        return !(lix == njx && liy == njy && ljx == nix && ljy == niy);
    }

    // nav_utils.get_single_actions membership
    OC_RH bool single_legal(const Row& r, int a, int code) const {
        if (code == kNoop) return true;
        return single_legal(r, a, code, target(r, a, code));
    }
    OC_RH bool single_legal(const Row& r, int a, int code, const Target& g) const {
        if (code == kNoop) return true;
        const int nx = g.x, ny = g.y;
#pragma unroll
        for (int b = 0; b < A; ++b)
            if (((blockers >> b) & 1u) && r.ax(b) == nx && r.ay(b) == ny) return false;
        const int c = g.c, t = g.t;
        if (t == kFloor || t == kDelivery) return true;
        const int o = item_at(r, c);
        const int h = r.ah(a);
        if (o < 0) return h != kNone;
        return h == kNone || mergeable(r.im(h), r.im(o));
    }

    // The same test without branches (the rollout row: the blocker scan, the square's class and
    // its item are all evaluated and combined with selects)
    OC_RH bool single_legal_flat(const Row& r, int a, int code, const Target& g) const {
        uint32_t on = 0;  // agents on the target square
#pragma unroll
        for (int b = 0; b < A; ++b) on |= r.ax(b) == g.x && r.ay(b) == g.y ? 1u << b : 0u;
        const int o = item_at(r, g.c), h = r.ah(a);
        const int hm = r.im(h == kNone ? 0 : h), om = r.im(o < 0 ? 0 : o);
        const bool open = g.t == kFloor || g.t == kDelivery;
        const bool item_ok = o < 0 ? h != kNone : (h == kNone || mergeable(hm, om));
        return code == kNoop || ((on & blockers) == 0u && (open || item_ok));
    }

    // The short-cut form (the likelihood kernels: fewer registers live across the checks)
    OC_RH bool action_legal(const Row& r, const Sub& s, int c0, int c1) const {
        if (s.kind == 0) return c0 == kNoop && (s.n < 2 || c1 == kNoop);
        if (!single_legal(r, s.agent[0], c0)) return false;
        if (s.n < 2) return true;
        return single_legal(r, s.agent[1], c1) && no_collision(r, s.agent[0], s.agent[1], c0, c1);
    }
    // The rollout row's form: g0, g1 the subtask agents' targets (g1 unused with one agent),
    // read once for the legality and interact; the checks are all evaluated (no short cut), so
    // their table reads issue together
    OC_RH bool action_legal(const Row& r, const Sub& s, int c0, int c1, const Target& g0, const Target& g1) const {
        if (s.kind == 0) return c0 == kNoop && (s.n < 2 || c1 == kNoop);
        const bool l0 = single_legal_flat(r, s.agent[0], c0, g0);
        if (s.n < 2) return l0;
        return ((int)l0 & (int)single_legal_flat(r, s.agent[1], c1, g1) & (int)no_collision(r, s.agent[0], s.agent[1], c0, c1)) != 0;
    }

    OC_RH bool is_goal(const Row& r, const Sub& s) const {
        if (s.kind == 0) return true;
        int count = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int c = r.il(j);
            if (c == kDead || r.im(j) != s.goal) continue;
            if (s.kind == 3) {  // un-held goal items on a Delivery square
                count += static_tile(c) == kDelivery ? 1 : 0;
            } else {  // distinct locations of goal items, held or not: count a slot's cell once
                bool dup = false;
#pragma unroll
                for (int i = 0; i < j; ++i) dup |= r.il(i) == c && r.im(i) == s.goal;
                count += dup ? 0 : 1;
            }
        }
        return count > s.count;
    }

    OC_RH int nid(int c, int d) const {  // graph node of (cell, approach)
        return ((const uint16_t*)(T + L.node_off))[mul24((uint32_t)c, 5u) + d];
    }
    OC_RH int dn(int u, int v) const {  // nx.shortest_path_length between node ids, or -1
        // branch-free: a missing node reads entry (0, 0) and is masked, so every lane of a
        // wave issues the same table reads
        const bool none = u == kNoNode || v == kNoNode;
        // narrow: u * nnodes < 1275^2 < 2^24, the full-rate 24-bit multiply; wide: up to 5,120^2
        const uint32_t i = WIDE ? (uint32_t)u * (uint32_t)L.nnodes + (uint32_t)v : mul24((uint32_t)u, (uint32_t)L.nnodes) + (uint32_t)v;
        if constexpr (DG) {
            if (L.dist16) {
                const int d = ((const uint16_t*)D)[none ? 0u : i];
                return none || d == 0xFFFF ? -1 : d;
            }
        }
        const int d = D[none ? 0u : i];
        return none || d == kNone ? -1 : d;
    }
    // the distance from node v to the nearest approach node of square c (the node-to-square table,
    // when the level has one), or -1: none reachable, v missing, or c an AgentCounter of the
    // Level-0 view (collidable there, and its approach nodes are not in the static graph)
    OC_RH int dsq(int v, int c) const {
        const int m = T[L.sq_off + (int)mul24((uint32_t)(v == kNoNode ? 0 : v), (uint32_t)L.sq_cells) + c];
        return v == kNoNode || m == kNone || is_ac(c) ? -1 : m;
    }
    // the nearest-Cutboard / nearest-Delivery distance of node v (dmin row `side`), or -1
    OC_RH int dmin(int side, int v) const {
        const uint32_t i = (uint32_t)(side * L.nnodes + (v == kNoNode ? 0 : v));
        if constexpr (DG) {
            if (L.dist16) {
                const int m = ((const uint16_t*)(T + L.dmin_off))[i];
                return m == 0xFFFF ? -1 : m;
            }
        }
        const int m = T[L.dmin_off + i];
        return m == kNone ? -1 : m;
    }

    // A square's graph nodes as the bound walks them: its four approach nodes when it is
    // collidable in the Level-0 view, else its own node (approach 4) four times; returns the
    // collidability.  A square is statically collidable exactly when it has no approach-4 node
    // (only Floor squares get one, world.py:67-108), so the five node reads issue together and
    // no tile read comes first (round 6).
    OC_RH bool approaches(int c, int (&v)[4]) const {
        if constexpr (LEAN) {
            const bool coll = tile(c) != kFloor;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = nid(c, coll ? q : 4);
            return coll;
        }
        const int n4 = nid(c, 4);
        const bool coll = n4 == kNoNode || is_ac(c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int nq = nid(c, q);
            v[q] = coll ? nq : n4;
        }
        return coll;
    }

    // World.get_lower_bound_between_helper (world.py:148-264) with check_bound (:266-283).  The
    // agents' node ids are looked up once, the A-side distances once per A approach and (two
    // agents) the B-side distances once per B approach, out of the pair loop; the arithmetic
    // is the reference's.  Only Merge comes here: Chop and Deliver have a static B side
    // (helper_static).
    // Uniform across lanes: the approach loops run 1 or 4 times for the whole wave (4 when some
    // lane's square is collidable, wave_any), never a per-lane trip count.  A Floor square has
    // one node (its own, approach 4), looked up for every approach index; repeated pairs give
    // the same bound, which the min takes once.  The reference's (ia, ib) order does not
    // matter: the result is a min.  (Per-lane trip counts of 1 or 4 per side left 0.56 of the
    // lanes active per VALU instruction in oc_bounds_kernel, with more SALU than VALU
    // instructions, profiles/r03/c5_static_b2/pmc_c5.json.)
    OC_RH float helper(const Sub& s, int u0, int u1, int Ac, int Bc) const {
        const int B1[1] = {Bc};
        return helper_n<1>(s, u0, u1, Ac, B1);
    }
    // min over NB B squares of helper(s, u0, u1, Ac, Bc[j]) (a repeated square is harmless):
    // the B squares' node and distance reads issue together (round 6, two at a time for the
    // rollout and bounds rows; two Plates make two B squares on the Salad kitchens)
    template <int NB>
    OC_RH float helper_n(const Sub& s, int u0, int u1, int Ac, const int (&Bc)[NB]) const {
        const float per = (float)L.perimeter;
        float lower = per + 1.0f;
        if (PT != nullptr && s.n == 2) {  // wave-uniform: the per-type minima from the agent-pair table
            bool ok = u0 != kNoNode && u1 != kNoNode && !is_ac(Ac);
#pragma unroll
            for (int j = 0; j < NB; ++j) ok = ok && !is_ac(Bc[j]);
            if (!wave_any(!ok)) return pair_bound(u0, u1, Ac, Bc);
        }
        int vA[4], vB[NB][4];
        const bool Acoll = approaches(Ac, vA);
        if (L.sq_off != 0 && s.n == 1) {  // wave-uniform: min over B's approaches from the table
            const int nA = wave_any(Acoll) ? 4 : 1;
#pragma unroll
            for (int ia = 0; ia < 4; ++ia) {
                if (ia >= nA) continue;  // wave-uniform
                const int a1 = dn(u0, vA[ia]);
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    const int b2 = dsq(vA[ia], Bc[j]);
                    const float bound = (float)(a1 + b2 - 1);
                    lower = a1 >= 0 && b2 >= 0 && bound < lower ? bound : lower;
                }
            }
            return lower > 1.0f ? lower : 1.0f;
        }
        bool Bcoll = false;
#pragma unroll
        for (int j = 0; j < NB; ++j) Bcoll |= approaches(Bc[j], vB[j]);
        const int nA = wave_any(Acoll) ? 4 : 1, nB = wave_any(Bcoll) ? 4 : 1;
        const uint32_t pa = xy(Ac);
        if (s.n == 1) {
#pragma unroll
            for (int ia = 0; ia < 4; ++ia) {
                if (ia >= nA) continue;  // wave-uniform
                const int a1 = dn(u0, vA[ia]);
#pragma unroll
                for (int j = 0; j < NB; ++j)
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib) {
                        if (ib >= nB) continue;
                        const int b2 = dn(vA[ia], vB[j][ib]);
                        const float bound = (float)(a1 + b2 - 1);
                        lower = a1 >= 0 && b2 >= 0 && bound < lower ? bound : lower;
                    }
            }
            return lower > 1.0f ? lower : 1.0f;
        }
        // Two agents.  Per pair (ia, ib) the reference takes mA = min(b1A, b2A), mB = min(b1B,
        // b2B), doubles both when one agent is nearest on both sides (a tie counts for both), and
        // bounds max(mA, mB) + (man - 1) / 2.  Round 6 takes the min over the 16 pairs by side:
        // each approach is of type 0 (agent 1 strictly nearer), 1 (agent 2 strictly nearer) or 2
        // (a tie), and over a product of two approach sets min max(mA, mB) = max(min mA, min
        // mB); so the min is over six type combinations of the per-type minima, doubled unless
        // the types are (0, 1) or (1, 0).  Integers (distances, or the perimeter for an
        // unreachable node) until the last add: the same value as the pair loop, exactly.
        constexpr int kInf = 0x3FFFFFFF;
        auto side = [&](const int (&v)[4], int n, int (&M)[3]) OC_RL {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= n) continue;  // wave-uniform
                int t;
                const int b1 = (t = dn(u0, v[q])) < 0 ? L.perimeter : t;
                const int b2 = (t = dn(u1, v[q])) < 0 ? L.perimeter : t;
                const int m = b1 < b2 ? b1 : b2;
                M[0] = b1 < b2 && m < M[0] ? m : M[0];
                M[1] = b2 < b1 && m < M[1] ? m : M[1];
                M[2] = b1 == b2 && m < M[2] ? m : M[2];
            }
        };
        int MA[3] = {kInf, kInf, kInf};
        side(vA, nA, MA);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            int MB[3] = {kInf, kInf, kInf};
            side(vB[j], nB, MB);
            const float bound = type_bound(MA, MB, pa, xy(Bc[j]));
            lower = bound < lower ? bound : lower;
        }
        return lower > 1.0f ? lower : 1.0f;
    }
    // The two-agent (A, B) pair's bound from the per-type minima of its squares (helper_n above)
    static constexpr int kInfM = 0x3FFFFFFF;
    OC_RH static float type_bound(const int (&MA)[3], const int (&MB)[3], uint32_t pa, uint32_t pb) {
        auto mx = [](int x, int y) OC_RL { return x > y ? x : y; };
        auto mn = [](int x, int y) OC_RL { return x < y ? x : y; };
        const int dx = (int)(pa & 0xFFu) - (int)(pb & 0xFFu), dy = (int)(pa >> 8) - (int)(pb >> 8);
        const float man = (float)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
        const int single = mn(mx(MA[0], MB[1]), mx(MA[1], MB[0]));
        const int dbl = mn(mn(mx(MA[0], MB[0]), mx(MA[1], MB[1])),
                           mn(mx(MA[2], mn(mn(MB[0], MB[1]), MB[2])), mx(mn(mn(MA[0], MA[1]), MA[2]), MB[2])));
        const int best = mn(single, 2 * dbl);
        return (float)best + (man - 1.0f) * 0.5f;
    }
    // helper_n's two-agent form with the squares' per-type minima read from the agent-pair table
    // (one u32 per square instead of the walk's 8 distance reads per square; round 6)
    template <int NB>
    OC_RH float pair_bound(int u0, int u1, int Ac, const int (&Bc)[NB]) const {
        const uint32_t* row = PT + (uint32_t)(u0 * L.nnodes + u1) * (uint32_t)(L.W * L.H);
        auto unpack = [](uint32_t e, int (&M)[3]) OC_RL {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int b = (int)((e >> (8 * t)) & 0xFFu);
                M[t] = b == 0xFF ? kInfM : b;
            }
        };
        uint32_t eb[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) eb[j] = row[Bc[j]];
        int MA[3];
        unpack(row[Ac], MA);
        const uint32_t pa = xy(Ac);
        float lower = (float)L.perimeter + 1.0f;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            int MB[3];
            unpack(eb[j], MB);
            const float bound = type_bound(MA, MB, pa, xy(Bc[j]));
            lower = bound < lower ? bound : lower;
        }
        return lower > 1.0f ? lower : 1.0f;
    }

    // min over a static B side (every Cutboard for Chop, every Delivery for Deliver) of
    // helper(s, ag0, ag1, Ac, B), without walking the B squares:
    //  * one agent: bound = d(agent, A) + d(A, B) - 1 over reachable pairs, and min over B of
    //    d(A node, B node) is the level's per-node table dm (world.py:175-189);
    //  * two agents: bound = min(d1(A), d2(A)) + manhattan(A, B) - 1 (world.py:215, 242-244),
    //    where B enters only through manhattan(A, B): the nearest square of the side, whichever
    //    approach node.
    // helper() clamps each pair's result to >= 1 and starts from perimeter + 1; both are
    // monotone, so the min over B of helper() is this with the same clamp.  Exact in fp32.
    OC_RH float helper_static(const Sub& s, int u0, int u1, int Ac, int nb, int side,
                              const uint16_t* man_t) const {
        const float per = (float)L.perimeter;
        float lower = per + 1.0f;
        if (nb == 0) return lower;
        int vAs[4];
        const bool Acoll = approaches(Ac, vAs);
        const int nA = wave_any(Acoll) ? 4 : 1;  // wave-uniform (a Floor A repeats its node)
        if (s.n == 1) {
#pragma unroll
            for (int ia = 0; ia < 4; ++ia) {
                if (ia >= nA) continue;
                const int vA = vAs[ia];
                const int a1 = dn(u0, vA), m = dmin(side, vA);
                const float bound = (float)(a1 + m - 1);
                lower = vA != kNoNode && a1 >= 0 && m >= 0 && bound < lower ? bound : lower;
            }
        } else {
            const int man = man_t[Ac];  // min over the side's squares (the level's table)
            float mA = per;
#pragma unroll
            for (int ia = 0; ia < 4; ++ia) {
                if (ia >= nA) continue;
                const int vA = vAs[ia];
                int t;
                const float b1A = (t = dn(u0, vA)) < 0 ? per : (float)t;
                const float b2A = (t = dn(u1, vA)) < 0 ? per : (float)t;
                const float m2 = b1A < b2A ? b1A : b2A;
                mA = m2 < mA ? m2 : mA;
            }
            const float bound = mA + (float)man - 1.0f;
            if (bound < lower) lower = bound;
        }
        return lower > 1.0f ? lower : 1.0f;
    }

    // The row's facts that every configuration's bound reads, gathered once per row (round 6:
    // oc_bounds_kernel evaluates up to 64 configurations on one row, and each one re-derived
    // them; the rollout and likelihood rows build it once per bound).
    struct BoundRow {
        AcT cells = 0;         // agent a's cell: byte a (narrow), u16 field a (wide)
        uint32_t nodes[2] = {0u, 0u};  // HOIST: agent a's graph node (approach 4), u16 field a % 2 of word a / 2
        uint32_t held = 0;     // agent a's held item's mask in byte a (0 where a holds nothing)
        uint32_t avail = 0;    // bit k < K: slot k is live and held by no agent; bit K + a: agent a holds one
        uint32_t deliv = 0;    // HOIST: bit k < K: slot k lies on a Delivery square; bit K + a: agent a
                               // stands on one
    };
    // HOIST (oc_bounds_kernel): the agents' graph nodes and the Delivery bits too, read once for
    // all configurations; a single bound (rollout, likelihood) reads the ones it needs.
    template <bool HOIST>
    OC_RH BoundRow bound_row(const Row& r) const {
        BoundRow b;
        uint32_t heldslots = 0;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const int c = agent_cell(r, a), h = r.ah(a);
            if constexpr (WIDE) b.cells |= (AcT)c << (16 * a);
            else b.cells |= (AcT)c << (8 * a);
            if (HOIST) b.nodes[a >> 1] |= (uint32_t)nid(c, 4) << (16 * (a & 1));
            if (h != kNone) {
                heldslots |= 1u << (h & 31);
                b.held |= (uint32_t)r.im(h) << (8 * a);
                b.avail |= 1u << (K + a);
            }
            if (HOIST) b.deliv |= static_tile(c) == kDelivery ? 1u << (K + a) : 0u;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int c = r.il(k);
            b.avail |= c != kDead && !((heldslots >> k) & 1u) ? 1u << k : 0u;
            if (HOIST) b.deliv |= c != kDead && static_tile(c) == kDelivery ? 1u << k : 0u;
        }
        return b;
    }
    OC_RH int brow_cell(const BoundRow& b, int a) const {
        if constexpr (WIDE) return (int)((b.cells >> (16 * a)) & 0xFFFFu);
        else return (int)((b.cells >> (8 * a)) & 0xFFu);
    }

    // Locations of `m` as get_AB_locs_given_objs lists them, as a set of sources: bit k < K an
    // un-held item in slot k, bit K + a a subtask agent a holding one; `skip_deliv` drops
    // Delivery squares (Deliver's A_locs).  Built branch-free over every source, so the lanes
    // of a wave only part ways in the walk over the set bits (usually 0 or 1 per side).
    template <bool HOIST>
    OC_RH uint32_t obj_set(const BoundRow& b, const Row& r, int m, bool skip_deliv) const {
        uint32_t set = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) set |= r.im(k) == m ? 1u << k : 0u;
#pragma unroll
        for (int a = 0; a < A; ++a) set |= ((b.held >> (8 * a)) & 0xFFu) == (uint32_t)m ? 1u << (K + a) : 0u;
        set &= b.avail & (((1u << K) - 1u) | (active << K));
        if (HOIST || !skip_deliv) return skip_deliv ? set & ~b.deliv : set;
        uint32_t dl = 0;  // the members' squares only
#pragma unroll
        for (int k = 0; k < K; ++k)
            dl |= ((set >> k) & 1u) && static_tile(r.il(k) == kDead ? 0 : r.il(k)) == kDelivery ? 1u << k : 0u;
#pragma unroll
        for (int a = 0; a < A; ++a)
            dl |= ((set >> (K + a)) & 1u) && static_tile(brow_cell(b, a)) == kDelivery ? 1u << (K + a) : 0u;
        return set & ~dl;
    }
    OC_RH int src_cell(const BoundRow& b, const Row& r, int k) const { return k < K ? r.il(k) : brow_cell(b, k - K); }

    // f(cell) for every location of obj_set (slot order, then agents); one rolled loop with one
    // call site: f (a bound walk) is inlined once, not K + A times
    template <bool HOIST, class F>
    OC_RH void visit_objs(const BoundRow& b, const Row& r, int m, bool skip_deliv, F&& f) const {
#pragma unroll 1
        for (uint32_t set = obj_set<HOIST>(b, r, m, skip_deliv); set != 0u; set &= set - 1u) f(src_cell(b, r, __builtin_ctz(set)));
    }

    // The same, two locations per call (f(c1, c2); c2 = c1 for a lone last one)
    template <bool HOIST, class F>
    OC_RH void visit_obj_pairs(const BoundRow& b, const Row& r, int m, bool skip_deliv, F&& f) const {
        uint32_t set = obj_set<HOIST>(b, r, m, skip_deliv);
#pragma unroll 1
        while (set != 0u) {
            const int c1 = src_cell(b, r, __builtin_ctz(set));
            set &= set - 1u;
            const int c2 = set != 0u ? src_cell(b, r, __builtin_ctz(set)) : c1;
            set &= set == 0u ? 0u : set - 1u;
            f(c1, c2);
        }
    }

    // get_lower_bound_for_subtask_given_objs (overcooked_environment.py:594-664)
    OC_RH float lower_bound(const Row& r, const Sub& s) const {
        float pen;
        const float d = lower_bound_parts<false>(bound_row<false>(r), r, s, pen);
        return d + pen;
    }

    // The same, split: returns World.get_lower_bound_between's distance (world.py:115-146) and
    // sets `pen` to the holding penalty (overcooked_environment.py:611-640).
    // Its head: the subtask agents' graph nodes (u0 the first active agent's, u1 the second's)
    // and the holding penalty.
    template <bool HOIST>
    OC_RH void bound_agents(const BoundRow& b, const Sub& s, int& u0, int& u1, float& pen) const {
        pen = 0.0f;
        int ag0 = 0, ag1 = 0, na = 0;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            if (!((active >> a) & 1u)) continue;
            const int v = HOIST ? (int)((b.nodes[a >> 1] >> (16 * (a & 1))) & 0xFFFFu) : brow_cell(b, a);
            if (na == 0) ag0 = v; else ag1 = v;
            ++na;
            const int hm = (int)((b.held >> (8 * a)) & 0xFFu);
            if (((b.avail >> (K + a)) & 1u) && s.kind != 2 && hm != s.start[0] && hm != s.goal) pen = 1.0f;
        }
        u0 = HOIST ? ag0 : nid(ag0, 4);
        u1 = HOIST || s.n != 2 ? ag1 : nid(ag1, 4);  // read by the two-agent bounds only
    }
    // full_bound's configuration of this object: no Level-0 view, the subtask agents active
    OC_RH void bound_config(const Sub& s) {
        ac = kNoAc;
        active = 1u << s.agent[0];
        if (s.n == 2) active |= 1u << s.agent[1];
        blockers = active;
    }

    template <bool HOIST>
    OC_RH float lower_bound_parts(const BoundRow& br, const Row& r, const Sub& s, float& pen) const {
        int u0, u1;
        bound_agents<HOIST>(br, s, u0, u1, pen);
        float lower = (float)L.perimeter + 1.0f;
        if (s.kind == 1 || s.kind == 3) {  // static B side: one table lookup per A approach
            const int nb = s.kind == 1 ? L.ncut : L.ndeliv;
            const int side = s.kind == 1 ? 0 : 1;
            const uint16_t* man_t = (const uint16_t*)(T + L.man_off) + (s.kind == 1 ? 0 : L.man_stride);
            visit_objs<HOIST>(br, r, s.start[0], s.kind == 3, [&](int Ac) OC_RL {
                const float b = helper_static(s, u0, u1, Ac, nb, side, man_t);
                if (b < lower) lower = b;
            });
        } else if (s.kind == 2) {
            visit_objs<HOIST>(br, r, s.start[0], false, [&](int Ac) OC_RL {
                if constexpr (LEAN) {
                    visit_objs<HOIST>(br, r, s.start[1], false, [&](int Bc) OC_RL {
                        const float b = helper(s, u0, u1, Ac, Bc);
                        if (b < lower) lower = b;
                    });
                } else {
                    visit_obj_pairs<HOIST>(br, r, s.start[1], false, [&](int B1, int B2) OC_RL {
                        const int Bc[2] = {B1, B2};
                        const float b = helper_n<2>(s, u0, u1, Ac, Bc);
                        if (b < lower) lower = b;
                    });
                }
            });
        }
        return lower;
    }

    // oc_subtask_bounds on a full state (no Level-0 view): lb = get_lower_bound_for_subtask_
    // given_objs; returns BayesianDelegator.subtask_alloc_is_doable (bayesian_delegator.py:98-156):
    // None -> true, else the distance < world.perimeter.  `br` = bound_row<true>(r), built once
    // for all of the row's configurations.
    OC_RH bool full_bound(const BoundRow& br, const Row& r, const Sub& s, float& lb) {
        bound_config(s);
        float pen;
        const float d = lower_bound_parts<true>(br, r, s, pen);
        lb = d + pen;
        return s.kind == 0 || d < (float)L.perimeter;
    }
    OC_RH bool full_bound(const Row& r, const Sub& s, float& lb) { return full_bound(bound_row<true>(r), r, s, lb); }

    // The whole row: returns OC_ROLL_* flags; r becomes the Level-0 next state (unchanged when
    // the configuration raises).
    OC_RH int run(Row& r, const Sub& s, int c0, int c1, float& lb) {
        const Row r_in = r;
        if (level0(r, s)) {
            r = r_in;
            lb = 0.0f;
            return 8;  // OC_ROLL_RAISES
        }
        if (s.kind == 0) c0 = c1 = kNoop;
        c0 = c0 > kNoop ? kNoop : c0;
        c1 = c1 > kNoop ? kNoop : c1;
        const Target g0 = target(r, s.agent[0], c0), g1 = s.n == 2 ? target(r, s.agent[1], c1) : g0;
        int fl = action_legal(r, s, c0, c1, g0, g1) ? 1 : 0;
        interact(r, s.agent[0], c0, g0);
        if (s.n == 2) interact(r, s.agent[1], c1, g1);
        const bool asserted = s.n == 2 && agent_cell(r, s.agent[0]) == agent_cell(r, s.agent[1]);
        if (asserted) fl |= 4;
        else if (is_goal(r, s)) fl |= 2;
        lb = lower_bound(r, s);
        return fl;
    }

    // E2E_BRTDP.Q(state, action, v_l) with value_init's values (e2e_brtdp.py:736-760, :678-729);
    // false where T raises (joint co-location)
    OC_RH bool q_value(const Row& r0, const Sub& s, int c0, int c1, double& q) const {
        // agent[1]'s target only for a two-agent subtask (a one-agent q_value never reads g1)
        const Target g0 = target(r0, s.agent[0], c0);
        return q_value(r0, s, c0, c1, g0, s.n == 2 ? target(r0, s.agent[1], c1) : g0, q);
    }
    OC_RH bool q_value(const Row& r0, const Sub& s, int c0, int c1, const Target& g0, const Target& g1, double& q) const {
        Row r = r0;
        interact(r, s.agent[0], c0, g0);
        if (s.n == 2) {
            interact(r, s.agent[1], c1, g1);
            if (agent_cell(r, s.agent[0]) == agent_cell(r, s.agent[1])) return false;
        }
        double cost = 1.0;  // time_cost + action_cost per moving agent (:816-826)
        if (c0 != kNoop) cost += 0.1;
        if (s.n == 2 && c1 != kNoop) cost += 0.1;
        double v = 0.0;
        if (!is_goal(r, s)) v = (double)lower_bound(r, s) * (1.0 + 0.1) - 1.09;
        q = cost + 1.0 * v;
        return true;
    }

    // BayesianDelegator.prob_nav_actions(..., no_level_1=True) (bayesian_delegator.py:461-689).
    // taken: agent a's executed action in byte a.  Returns OC_LIK_* flags.
    OC_RH int likelihood(Row r, const Sub& s, uint32_t taken, int self_agent, double beta, double nap,
                         double& out) {
        out = 0.0;
        if (s.kind == 0) {  // None: one agent, the self agent's movable actions in the full state
            if (s.n != 1) return 4;
            active = blockers = (1u << A) - 1u;
            ac = kNoAc;
            int n = 0;
            for (int c = 0; c < 4; ++c) n += single_legal(r, self_agent, c) ? 1 : 0;
            if (n == 0) return 8;
            const double ap = (1.0 - nap) / n, x0 = beta * nap, x1 = beta * ap, m = x0 > x1 ? x0 : x1;
            double S = exp(x0 - m);
            for (int k = 0; k < n; ++k) S += exp(x1 - m);
            const bool moved = ((taken >> (8 * s.agent[0])) & 0xFFu) != kNoop;
            out = (moved ? exp(x1 - m) : exp(x0 - m)) / S;
            return 1;
        }
        if (level0(r, s)) return 4;
        int t0 = (int)((taken >> (8 * s.agent[0])) & 0xFFu), t1 = kNoop;
        if (s.n == 2) t1 = (int)((taken >> (8 * s.agent[1])) & 0xFFu);
        t0 = t0 > kNoop ? kNoop : t0;
        t1 = t1 > kNoop ? kNoop : t1;
        double old_q;
        if (!q_value(r, s, t0, t1, old_q)) return 4;
        if (!action_legal(r, s, t0, t1)) return 4;  // assert action in valid_nav_actions
        const int other = s.n == 2 ? (s.agent[0] == self_agent ? 1 : (s.agent[1] == self_agent ? 0 : -1)) : -1;
        // one rollout per valid candidate: x = beta * (old_q - Q) kept per candidate, then the
        // max and the softmax sum over them in candidate order (the reference's two passes
        // over the same values, bayesian_delegator.py:676-689)
        double xs[25];
        uint32_t valid = 0u;
        double m = -1.0e300, xt = 0.0;
        bool found = false;
        // kept rolled: each candidate is a whole rollout (interact + goal + bound walk)
#pragma unroll 1
        for (int a0 = 0; a0 < 5; ++a0)
#pragma unroll 1
            for (int a1 = 0; a1 < (s.n == 2 ? 5 : 1); ++a1) {
                const int c1 = s.n == 2 ? a1 : kNoop;
                if (!action_legal(r, s, a0, c1)) continue;
                if (other == 0 && a0 != t0) continue;
                if (other == 1 && c1 != t1) continue;
                double q;
                if (!q_value(r, s, a0, c1, q)) return 4;
                const double x = beta * (old_q - q);
                const int k = a0 * 5 + a1;
                xs[k] = x;
                valid |= 1u << k;
                m = x > m ? x : m;
                if (a0 == t0 && c1 == t1) { found = true; xt = x; }
            }
        if (!found) return 4;
        double S = 0.0;
        for (uint32_t v = valid; v; v &= v - 1u) S += exp(xs[__builtin_ctz(v)] - m);
        out = exp(xt - m) / S;
        return 1;
    }
};

}  // namespace ocro
