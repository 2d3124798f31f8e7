// oc_swar.h -- the env step of oc_step_kernel as SWAR over four envs per dword.
//
// Every state plane is loaded one dword per lane, i.e. byte q of a plane word belongs to
// env q of that lane (q = 0..3).  The step runs on those words directly: all per-env
// predicates are byte masks, computed with carry-free byte arithmetic and v_bitop3 logic,
// selects are v_bitop3 (m ? a : b), per-env table lookups are v_perm byte selects, and the
// tile class of a cell comes from a 256-entry LDS table.  Measured on MI355X (tools/
// valubench.hip): v_add / v_xor / shifts / v_bitop3 issue at ~2.9 cycles per wave-instruction,
// v_perm / v_bfi / v_bfe / v_cndmask / v_cmp at ~5, so the formulation leans on the former.
//
// Mask conventions (per byte lane):
//   "h80"  : 0x80 where true, 0x00 where false (only bit 7 used)
//   "full" : 0xFF where true, 0x00 where false (select operand)
//
// Semantics restated (reference file:line):
//   is_collision / check_collisions    gym_cooking/envs/overcooked_environment.py:671-762
//   interact                           gym_cooking/utils/interact.py:4-89
//   SimAgent.acquire/release/move_to   gym_cooking/utils/agent.py:408-423
//   Object predicates, mergeable       gym_cooking/utils/core.py:176-241
//   copy crash (ERR)                   overcooked_environment.py:289 -> :108-113 -> world.py:417
//   done / reward                      overcooked_environment.py:316-376
//
// The includer provides __host__/__device__/__forceinline__ (the HIP compiler; tests/swar_host/
// builds this header with plain clang++).  Every function here is host and device code: the
// device pass uses the two AMDGCN intrinsics (v_perm_b32, v_bitop3_b32), the host pass the
// bit-exact restatements below; the host pass is oc_cpu_step's step (include/oc_engine.h).
#pragma once

#include <stdint.h>

#define OC_SW __host__ __device__ __forceinline__

namespace ocsw {

constexpr uint32_t k01 = 0x01010101u, k04 = 0x04040404u, k07 = 0x07070707u, k08 = 0x08080808u,
                   k0F = 0x0F0F0F0Fu, k78 = 0x78787878u, k7F = 0x7F7F7F7Fu, k80 = 0x80808080u,
                   kFF = 0xFFFFFFFFu;
constexpr uint32_t kLanes = 0x03020100u;  // v_perm selector: byte q <- byte q

// ---- bitop3 with a truth table built from a boolean function of (a, b, c) ----
template <class F>
constexpr uint32_t lut3(F f) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r |= (uint32_t)(f((i >> 2) & 1, (i >> 1) & 1, i & 1) & 1) << i;
    return r;
}
#define OC_LUT(expr) ::ocsw::lut3([](int a, int b, int c) constexpr { (void)a; (void)b; (void)c; return (expr); })
// v_bitop3_b32: bit i of the result is IMM's bit (a_i << 2 | b_i << 1 | c_i).  On the host
// IMM is a constant, so the minterm loop folds to a few logic operations.
template <uint32_t IMM>
OC_SW uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
#else
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i)
        if (IMM & (1u << i)) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
#endif
}

OC_SW uint32_t sel(uint32_t m, uint32_t a, uint32_t b) { return bop3<OC_LUT(a ? b : c)>(m, a, b); }
OC_SW uint32_t and3(uint32_t a, uint32_t b, uint32_t c) { return bop3<OC_LUT(a & b & c)>(a, b, c); }
OC_SW uint32_t or3(uint32_t a, uint32_t b, uint32_t c) { return bop3<OC_LUT(a | b | c)>(a, b, c); }
OC_SW uint32_t andn(uint32_t a, uint32_t b) { return bop3<OC_LUT(a & !b)>(a, b, 0u); }  // a & ~b
// v_perm_b32: result byte i = selector byte s_i of {hi:lo}: 0-7 a source byte, 8-11 the sign
// of a 16-bit half replicated, 12 zero, 13 and up 0xFF.
OC_SW uint32_t perm(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, s);
#else
    // branch-free: a 16-entry byte table (8 source bytes, 4 sign bytes, 0x00, 3 x 0xFF)
    // indexed by min(q, 13)
    const uint64_t src = ((uint64_t)hi << 32) | lo;
    uint8_t tab[16];
    for (int i = 0; i < 8; ++i) tab[i] = (uint8_t)(src >> (8 * i));
    for (int i = 0; i < 4; ++i) tab[8 + i] = (uint8_t)(((src >> (16 * i + 15)) & 1u) ? 0xFFu : 0u);
    tab[12] = 0u;
    tab[13] = tab[14] = tab[15] = 0xFFu;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t q = (s >> (8 * i)) & 0xFFu;
        r |= (uint32_t)tab[q < 13u ? q : 13u] << (8 * i);
    }
    return r;
#endif
}

// In-place updates for the rare path of step4: x = m ? a : x, x &= ~m, x |= m.  Both builds
// (oc_engine.hip and the host test harness) use the plain-C forms below.  A device variant
// with inline asm tied to x (so that the common path, where x passes through, needs no copy
// at the join) was compiled and dropped: the step_n kernels came out larger (A = 2: 713 vs
// 699 VALU instructions; A = 3 with the loader wave: 1,115 vs 948), as the asm blocks pin
// the operands' registers and keep the compiler from folding the selects.  The hooks stay
// for such experiments.
#ifndef OC_TIED_SEL
#define OC_TIED_SEL(x, m, a) ((x) = ::ocsw::sel((m), (a), (x)))
#define OC_TIED_ANDN(x, m) ((x) = ::ocsw::andn((x), (m)))
#define OC_TIED_OR(x, m) ((x) |= (m))
#endif

// h80 -> full mask per byte: 0x80 -> 0xFF, 0x00 -> 0x00.  One v_perm_b32 with h as the
// selector: a selector byte >= 13 (0x80) yields 0xFF, and 0 picks byte 0 of the zero source
// (h | (h - (h >> 7)), the carry-free arithmetic form, takes three instructions).  Every h
// passed here has only bit 7 of a byte set.
OC_SW uint32_t full80(uint32_t h) { return perm(0u, 0u, h); }
// bytes <= 0x7F: h80 of (byte != 0) / (byte == 0)
OC_SW uint32_t nz80(uint32_t x) { return (x + k7F) & k80; }
OC_SW uint32_t z80(uint32_t x) { return andn(k80, x + k7F); }
// bytes may have bit 7 set (0xFF sentinels): h80 of (a == b) on the low 7 bits
OC_SW uint32_t eq80(uint32_t a, uint32_t b) { return z80(bop3<OC_LUT((a ^ b) & c)>(a, b, k7F)); }
// any bytes: h80 of (byte == 0) over all 8 bits
OC_SW uint32_t zf80(uint32_t x) { return andn(k80, ((x & k7F) + k7F) | x); }

// Per-level constants the SWAR step reads (all wave-uniform, kernel-argument resident).
struct SwarLevel {
    uint32_t W;              // grid width
    uint32_t yw_lo, yw_hi;   // v_perm LUT: y -> y*W (y = 0..7)
    uint32_t dc_lo, dc_hi;   // v_perm LUT: action code -> cell delta + 0x80
    uint32_t done_rep;       // first Delivery cell, replicated to every byte
    uint32_t goals_rep[4];   // Deliver goal masks, replicated
    int32_t ngoals;
    uint32_t maxT_rep;       // max_T replicated to both u16 halves (0 = no limit)
    uint32_t tmpl_x[4], tmpl_y[4], tmpl_l[16], tmpl_m[16];  // reset template, replicated
    int32_t tall;            // H > 8: y*W by multiply instead of the 8-entry LUT
    int32_t big;             // W*H > 128: cell ids reach bit 7, so cell compares use all 8 bits
                             // and the move delta is added as (positive part) - (negative part)
                             // (each byte stays in 0..254, no carry between envs)
    uint32_t dp_lo, dp_hi, dn_lo, dn_hi;  // big: v_perm LUTs action code -> max(delta, 0), max(-delta, 0)
    int32_t counts;          // item masks in OC_ENC_COUNTS (a food type repeats on the map): the
                             // content predicates below read 2-bit counts, a plate bit and a Fresh bit
    int32_t edge;            // a Floor square on the grid's border: an action can point off the grid
    uint32_t wm1_rep, hm1_rep;  // W - 1, H - 1 replicated (the off-grid test)
    // wide levels (more than 255 cells, u16 cell ids; step4w): done_rep and tmpl_l hold the low
    // bytes of the first Delivery cell and of the template's item cells, these the high bytes
    uint32_t done_hi_rep;
    uint32_t tmpl_lh[16];
};

// Host-side construction of the SwarLevel constants (called by oc_create after validation).
// cell/mask: item slot templates (OC_LOC_DEAD / 0 past the level's items).
__host__ __device__ inline void build_swar_level(SwarLevel& S, int W, int H, int done_cell, const uint8_t* goal_mask,
                             int ngoals, int max_T, const uint8_t* spawn_x, const uint8_t* spawn_y,
                             int num_agents, const uint8_t* cell, const uint8_t* mask, int encoding,
                             const uint8_t* tiles) {
    S = SwarLevel{};
    S.W = (uint32_t)W;
    S.counts = encoding != 0;
    for (int c = 0; c < W * H; ++c) {
        const int x = c % W, y = c / W;
        if (tiles[c] == 0 && (x == 0 || y == 0 || x == W - 1 || y == H - 1)) S.edge = 1;  // OC_TILE_FLOOR
    }
    S.wm1_rep = (uint32_t)(W - 1) * 0x01010101u;
    S.hm1_rep = (uint32_t)(H - 1) * 0x01010101u;
    S.tall = H > 8;
    S.big = W * H > 128;
    const int dcell[5] = {W, -W, -1, 1, 0};
    for (int c = 0; c < 8; ++c) {
        const int d = c < 5 ? dcell[c] : 0;
        const uint32_t pv = (uint32_t)(d > 0 ? d : 0), nv = (uint32_t)(d < 0 ? -d : 0);
        if (c < 4) {
            S.dp_lo |= pv << (8 * c);
            S.dn_lo |= nv << (8 * c);
        } else {
            S.dp_hi |= pv << (8 * (c - 4));
            S.dn_hi |= nv << (8 * (c - 4));
        }
    }
    for (int y = 0; y < 8; ++y) {
        const uint32_t v = (uint32_t)(y * W) & 0xFFu;
        if (y < 4) S.yw_lo |= v << (8 * y); else S.yw_hi |= v << (8 * (y - 4));
    }
    for (int c = 0; c < 8; ++c) {
        const uint32_t v = (uint32_t)((c < 5 ? dcell[c] : 0) + 128) & 0xFFu;
        if (c < 4) S.dc_lo |= v << (8 * c); else S.dc_hi |= v << (8 * (c - 4));
    }
    S.done_rep = (uint32_t)done_cell * 0x01010101u;
    for (int g = 0; g < 4; ++g) S.goals_rep[g] = (uint32_t)(g < ngoals ? goal_mask[g] : 0) * 0x01010101u;
    S.ngoals = ngoals;
    S.maxT_rep = (uint32_t)max_T * 0x00010001u;
    for (int a = 0; a < 4; ++a) {
        S.tmpl_x[a] = (uint32_t)(a < num_agents ? spawn_x[a] : 0) * 0x01010101u;
        S.tmpl_y[a] = (uint32_t)(a < num_agents ? spawn_y[a] : 0) * 0x01010101u;
    }
    for (int j = 0; j < 16; ++j) {  // cell / mask: 16 slots (OC_LOC_DEAD / 0 past the level's items)
        S.tmpl_l[j] = (uint32_t)cell[j] * 0x01010101u;
        S.tmpl_m[j] = (uint32_t)mask[j] * 0x01010101u;
    }
}

// Tile class byte of a cell (the LDS table) from its OC_TILE_* code: 0x80 Floor, 0x40 Delivery,
// 0x20 Cutboard, 0 Counter (and every cell id past the grid).
__host__ __device__ inline uint8_t tile_class(int tile) {
    return (uint8_t)(tile == 0 ? 0x80 : tile == 3 ? 0x40 : tile == 2 ? 0x20 : 0);
}

// dx + 1 / dy + 1 per action code (World.NAV_ACTIONS order, world.py:16, + no-op)
constexpr uint32_t kDXlo = 0x02000101u, kDXhi = 0x01010101u;  // codes 0..3 | 4..7
constexpr uint32_t kDYlo = 0x01010002u, kDYhi = 0x01010101u;

// Gather V[idx] per byte lane from K slot words; idx bits 1, 2, 3 given as full masks f1, f2, f3.
template <int K>
OC_SW uint32_t gather(const uint32_t (&V)[K], uint32_t s, uint32_t f1, uint32_t f2, uint32_t f3 = 0u) {
    // s: v_perm selector picking byte q of the even (bit0 = 0) or odd slot of a pair
    const uint32_t g01 = perm(V[1], V[0], s), g23 = perm(V[3], V[2], s);
    const uint32_t lo = sel(f1, g23, g01);
    if constexpr (K == 4) {
        (void)f2;
        (void)f3;
        return lo;
    } else {
        const uint32_t g45 = perm(V[5], V[4], s), g67 = perm(V[7], V[6], s);
        const uint32_t lo8 = sel(f2, sel(f1, g67, g45), lo);
        if constexpr (K == 8) {
            (void)f3;
            return lo8;
        } else {
            const uint32_t g89 = perm(V[9], V[8], s), gAB = perm(V[11], V[10], s);
            const uint32_t gCD = perm(V[13], V[12], s), gEF = perm(V[15], V[14], s);
            const uint32_t hi8 = sel(f2, sel(f1, gEF, gCD), sel(f1, gAB, g89));
            return sel(f3, hi8, lo8);
        }
    }
}

// h80 per env: some item of the env lies on the first Delivery square (done()'s square).
template <int K, int MODE = 1>
OC_SW uint32_t at_done80(const SwarLevel& L, const uint32_t (&Lc)[K]) {
    const bool big = MODE ? (bool)L.big : false;
    uint32_t hit = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) hit |= big ? zf80(Lc[j] ^ L.done_rep) : eq80(Lc[j], L.done_rep);
    return hit;
}

// One step of 4 envs x A agents x K item slots.  `cls_of(cellword)` returns per byte the
// tile class bits of that cell: 0x80 Floor, 0x40 Delivery, 0x20 Cutboard.
//
// Rare-event split.  done()'s success test, the auto-reset selects and the episode-end flags
// only matter in a step with a rare event: an env reset, the timeout, the copy crash (ERR),
// or a delivery.  Items reach a Delivery square only by being delivered and never leave it (no
// pick-up from, no merge onto a Delivery, interact.py:35-40, 73-84), and a state whose
// success test held was DONE and is reset in the next step; so in a state this step produced,
// success can newly hold only in a step that delivered.  `any_of(word)` is true when the word
// is nonzero in any env of the wave (a ballot; the host harness tests its own lane), and
// `pending` marks envs of a state that came from outside (a launch's loaded state): they take
// the full path once, since an item may already sit on the Delivery square (the gym shim
// clears DONE and steps again, as the reference keeps stepping a finished env).  Without a
// rare event in the wave the step leaves flags 0, keeps every item, and only advances t.
// Random play at the bench's shapes meets one in about 1 % of wave-steps.
// MODE 0 compiles the step for the common level class (H <= 8 rows, W*H <= 128 cells, presence
// masks: every shipped kitchen) with the tall / big / counts paths removed; MODE 1 reads the
// level's flags (wave-uniform branches).  Returns whether the wave took the full path.
template <int A, int K, int MODE = 1, class ClassOf, class AnyOf>
OC_SW bool step4(const SwarLevel& L, uint32_t (&X)[A], uint32_t (&Y)[A], uint32_t (&H)[A],
                 uint32_t (&Lc)[K], uint32_t (&M)[K], uint32_t& T0, uint32_t& T1, uint32_t& F,
                 const uint32_t (&ACT)[A], uint32_t (&EX)[A], uint32_t& CM, ClassOf cls_of, AnyOf any_of,
                 uint32_t& pending) {
    const bool tall = MODE ? (bool)L.tall : false, big = MODE ? (bool)L.big : false;
    const bool counts = MODE ? (bool)L.counts : false;
    const bool edge = MODE ? (bool)L.edge : false;
    const uint32_t rst = full80((F << 7) & k80);  // input DONE => next-step auto-reset

    // ---- positions, next squares, collidability (is_collision :692-700) ----
    uint32_t act[A], loc[A], nraw[A], cls[A], nn80[A], bump80[A], nxt[A], blk80[A], out80[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        uint32_t c = ACT[a];
        const uint32_t ge5 = bop3<OC_LUT((a | b) & c)>((c & k7F) + 0x7B7B7B7Bu, c, k80);
        act[a] = sel(full80(ge5), k04, c);  // codes > 4 act as (0, 0)
        out80[a] = 0u;
    }
    // A Floor on the border (wave-uniform): an action can point off the grid.  is_collision
    // looks the unclamped square up (get_gridsquare_at asserts there is exactly one: it
    // raises, :692-700), so with two or more agents such a step raises in check_collisions
    // before anything moves: the env gets DONE | ERR with its state unchanged but t (as the
    // copy crash), every action a no-op.  With one agent there is no pair
    // to check, and interact's World.inbounds clamps the square to the agent's own (no move).
    uint32_t raise80 = 0u;
    if (edge) {
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const uint32_t c = act[a];
            out80[a] = or3(and3(z80(c), z80(Y[a] ^ L.hm1_rep), k80), and3(z80(c ^ k01), z80(Y[a]), k80),
                           and3(z80(c ^ 0x02020202u), z80(X[a]), k80) | and3(z80(c ^ 0x03030303u), z80(X[a] ^ L.wm1_rep), k80));
            if (A >= 2) raise80 |= out80[a];
        }
        if (A >= 2) {
#pragma unroll
            for (int a = 0; a < A; ++a) {
                act[a] = sel(full80(raise80), k04, act[a]);
                out80[a] = 0u;
            }
        }
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
        const uint32_t c = act[a];
        nn80[a] = nz80(c ^ k04);
        uint32_t yw;
        if (tall)  // wave-uniform: H > 8 rows
            yw = Y[a] * L.W;
        else
            yw = perm(L.yw_hi, L.yw_lo, Y[a]);
        loc[a] = yw + X[a];
        if (big)  // wave-uniform: cells up to 254, loc + delta in two carry-free halves
            nraw[a] = loc[a] + perm(L.dp_hi, L.dp_lo, c) - perm(L.dn_hi, L.dn_lo, c);
        else  // cells < 128: loc + (delta + 0x80) stays in its byte, bias removed
            nraw[a] = (loc[a] + perm(L.dc_hi, L.dc_lo, c)) ^ k80;
        if (edge) nraw[a] = sel(full80(out80[a]), loc[a], nraw[a]);  // World.inbounds (one agent)
        cls[a] = cls_of(nraw[a]);
        const uint32_t onF80 = cls[a] & k80;
        nxt[a] = sel(full80(onF80), nraw[a], loc[a]);
        bump80[a] = andn(nn80[a], onF80);  // a != (0,0) but next square collidable
        blk80[a] = 0u;
    }

    // ---- check_collisions (:724-762): pairs in itertools.combinations order ----
    uint32_t cm = 0u;
    int p = 0;
#pragma unroll
    for (int i = 0; i < A; ++i) {
#pragma unroll
        for (int j = i + 1; j < A; ++j, ++p) {
            uint32_t eq, sw;
            if (big) {  // cell bytes reach bit 7: full-byte zero tests (no carry between envs)
                eq = zf80(nxt[i] ^ nxt[j]);
                sw = zf80(loc[i] ^ nxt[j]) & zf80(loc[j] ^ nxt[i]);
            } else {
                eq = z80(nxt[i] ^ nxt[j]);
                sw = bop3<OC_LUT((!a) & (!b) & c)>((loc[i] ^ nxt[j]) + k7F, (loc[j] ^ nxt[i]) + k7F, k80);
            }
            const uint32_t bi = bop3<OC_LUT(a ? !b : c)>(eq, bump80[i], sw);
            const uint32_t u = bop3<OC_LUT((a | !b) & c)>(bump80[i], bump80[j], k80);
            const uint32_t bj = sel(eq, u, sw);
            blk80[i] |= bi;
            blk80[j] |= bj;
            cm |= (bi | bj) >> (7 - p);
        }
    }

    if (edge && A >= 2) cm = andn(cm, full80(raise80));  // a raising step logs no collision (build-defined)

    // ---- execute_navigation: interact per agent, in order (:767-770, interact.py:4-89) ----
    uint32_t dlv = 0u;  // h80: some agent delivered
#pragma unroll
    for (int k = 0; k < A; ++k) {
        const uint32_t go80 = andn(nn80[k], blk80[k]);
        EX[k] = sel(full80(go80), act[k], k04);
        const uint32_t tc = nraw[k];  // inbounds(loc + a): identity on a non-Floor border
        const uint32_t isF80 = cls[k] & k80;
        const uint32_t isD80 = (cls[k] << 1) & k80;
        const uint32_t isC80 = (cls[k] << 2) & k80;
        const uint32_t h = H[k];
        const uint32_t hold80 = andn(k80, h);  // slot index < 0x80, none = 0xFF
        // un-held items at tc (a non-Delivery cell holds at most one; held items sit on Floor).
        // ne[j] has bit 7 set where slot j is NOT at tc, so the ORs over slots are ANDs of ne
        // (one bitop3 per three slots) and each slot costs two instructions, not three.
        uint32_t ne[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (big)
                ne[j] = ~zf80(Lc[j] ^ tc);
            else
                ne[j] = bop3<OC_LUT((a ^ b) & c)>(Lc[j], tc, k7F) + k7F;  // bit 7: low 7 bits differ
        }
        // h80 of "some slot of the set is at tc": bit 7 of ~AND(ne over the set)
        auto any_at = [&](auto pick) -> uint32_t {
            uint32_t all = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (pick(j)) all &= ne[j];
            return andn(k80, all);
        };
        const uint32_t seen = any_at([](int) { return true; });
        const uint32_t ob0 = any_at([](int j) { return (j & 1) != 0; });
        const uint32_t ob1 = any_at([](int j) { return (j & 2) != 0; });
        const uint32_t ob2 = K > 4 ? any_at([](int j) { return (j & 4) != 0; }) : 0u;
        const uint32_t ob3 = K > 8 ? any_at([](int j) { return (j & 8) != 0; }) : 0u;
        const uint32_t so1 = (ob0 >> 5) | kLanes;                            // (o & 1) * 4 + q
        const uint32_t sh = bop3<OC_LUT((a & b) | c)>(h << 2, k04, kLanes);  // (h & 1) * 4 + q
        // A held item lies on its holder's square: acquire sets its location to the agent's,
        // move_to moves it along, and a merge keeps the holder's object (agent.py:408-423,
        // core.py merge), so the held slot's location is loc[k] and needs no gather.
        uint32_t om, hm;
        if constexpr (K == 4) {  // the pair select is a second v_perm on the index's bit 1
            const uint32_t so2 = (ob1 >> 5) | kLanes, sh2 = bop3<OC_LUT(a | (b & c))>(kLanes, h << 1, k04);
            om = perm(perm(M[3], M[2], so1), perm(M[1], M[0], so1), so2);
            hm = perm(perm(M[3], M[2], sh), perm(M[1], M[0], sh), sh2);
        } else {
            const uint32_t fo1 = full80(ob1), fo2 = full80(ob2), fo3 = K == 16 ? full80(ob3) : 0u;
            const uint32_t fh1 = full80((h << 6) & k80), fh2 = full80((h << 5) & k80);
            const uint32_t fh3 = K == 16 ? full80((h << 4) & k80) : 0u;
            om = gather<K>(M, so1, fo1, fo2, fo3);
            hm = gather<K>(M, sh, fh1, fh2, fh3);
        }

        const uint32_t nf = andn(go80, isF80), mv = andn(go80 & isF80, out80[k]);  // clamped: no move
        // Content predicates as "raw" words: only bit 7 of each byte carries the predicate (or
        // its negation, n*_r); the other bits are don't-care, because every use ANDs it with a
        // clean h80 word (nfh, cnt, empty), which saves the per-predicate & 0x80.
        uint32_t two_r, nallch_r, nplate_r, nfood_r, nch_r, cu, chopped;
        if (counts) {  // wave-uniform: OC_ENC_COUNTS masks (T/L/O 2-bit counts, 0x40 Plate, 0x80 Fresh)
            const uint32_t x = hm & k7F;
            // >= 2 contents: the count bits are not a single unit (0x01, 0x04, 0x10, 0x40) nor zero;
            // ((x | 0x80) - 1) & x clears the lowest set bit without a borrow into the next env
            two_r = bop3<OC_LUT((a & b) | c)>((x | k80) - k01, x, x & 0x2A2A2A2Au) + k7F;
            nallch_r = 0u;  // a merged object is all-Chopped (mergeable admits last-state foods only)
            nplate_r = and3(hm, om, 0x40404040u) + k7F;
            nfood_r = hm | om;  // a Fresh food on either side
            nch_r = hm;         // Object.needs_chopped: a single fresh food (bit 7 = Fresh)
            cu = x + (om & k7F);  // contents add up; every field sum stays in its bits
            chopped = x;          // Object.chop: the Fresh bit goes
        } else {
            // Object.is_deliverable (core.py:214-219): >= 2 contents, all foods chopped
            const uint32_t c4 = hm & k0F;
            two_r = (((c4 | k80) - k01) & c4) + k7F;
            nallch_r = bop3<OC_LUT((!a) & b & c)>(hm >> 4, hm, k07) + k7F;
            // mergeable (core.py:222-241): <= 1 plate, every food chopped
            cu = hm | om;
            nplate_r = and3(hm, om, k08) + k7F;
            nfood_r = bop3<OC_LUT((!a) & b & c)>(cu >> 4, cu, k07) + k7F;
            // Object.needs_chopped (core.py:176-178): exactly one content, a fresh food
            nch_r = bop3<OC_LUT(a & !b & !c)>(c4 + k7F, two_r, (hm & k78) + k7F);
            // Object.chop (core.py:187-192): the single food's chopped bit (bits 4..6, no cross-byte spill)
            chopped = bop3<OC_LUT((a & b) | c)>(hm << 4, 0x70707070u, hm);
        }
        const uint32_t nfh = nf & hold80;
        const uint32_t deliver = bop3<OC_LUT(a & b & !c)>(nfh & isD80, two_r, nallch_r);  // :35-40
        const uint32_t cnt = andn(nfh, isD80);
        const uint32_t merge = bop3<OC_LUT(a & b & !c)>(cnt, seen, nplate_r | nfood_r);    // :43-56
        const uint32_t empty = andn(cnt, seen);                                              // :60-70
        const uint32_t chop = and3(empty, isC80, nch_r);
        const uint32_t put = andn(empty, chop);
        const uint32_t pick = andn(bop3<OC_LUT(a & !b & c)>(nf, hold80, seen), isD80);  // :73-84
        const uint32_t reloc = or3(mv, deliver, put);  // the held item ends on tc
        dlv |= deliver;

        // SimAgent.move_to (agent.py:420-423): an env that does not move reads its action code
        // as 4..7 (act | 4), whose delta is (0, 0) (each byte stays >= 1 before the - 1)
        const uint32_t amv = bop3<OC_LUT(a | ((!b) & c))>(act[k], mv >> 5, k04);
        X[k] = X[k] + perm(kDXhi, kDXlo, amv) - k01;
        Y[k] = Y[k] + perm(kDYhi, kDYlo, amv) - k01;
        // new values of the target slot o and the held slot h
        const uint32_t fmg = full80(merge), fpk = full80(pick);
        const uint32_t newOl = fmg | sel(fpk, loc[k], tc);  // merged away: dead (0xFF)
        const uint32_t newOm = andn(om, fmg);
        const uint32_t newHl = sel(full80(reloc), tc, loc[k]);
        const uint32_t newHm = sel(fmg, cu, sel(full80(chop), chopped, hm));
        // scatter: target slot on merge / pick, held slot on reloc / merge / chop.  The per-slot
        // select masks are one v_perm each: selector byte = slot index (h, or the target slot
        // oidx), table byte j = 0xFF.  Envs that write no slot get selector 0x0C, which v_perm
        // turns into a zero byte (a holding-none h = 0xFF never writes: fwh includes hold80).
        const uint32_t oidx = (ob0 >> 7) | (ob1 >> 6) | (ob2 >> 5) | (ob3 >> 4);
        const uint32_t fwo = full80(merge | pick);
        const uint32_t fwh = full80(and3(hold80, or3(reloc, merge, chop), k80));
        const uint32_t so = sel(fwo, oidx, 0x0C0C0C0Cu), shw = sel(fwh, h, 0x0C0C0C0Cu);
        // K = 16: slots 8..15 use the same tables on index - 8; each half's selector turns the
        // other half's indices into 0x0C (v_perm selectors >= 8 are not byte selects)
        uint32_t so_lo = so, shw_lo = shw, so_hi = 0x0C0C0C0Cu, shw_hi = 0x0C0C0C0Cu;
        if constexpr (K == 16) {
            // index bit 3 of the slots written (the no-write code 0x0C has bit 3 set too)
            const uint32_t o8 = full80(and3(oidx << 4, k80, fwo)), h8 = full80(and3(h << 4, k80, fwh));
            so_lo = sel(o8, 0x0C0C0C0Cu, so);
            shw_lo = sel(h8, 0x0C0C0C0Cu, shw);
            so_hi = sel(o8, oidx ^ 0x08080808u, 0x0C0C0C0Cu);
            shw_hi = sel(h8, h ^ 0x08080808u, 0x0C0C0C0Cu);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int jj = j & 7;
            const uint32_t lut_lo = jj < 4 ? 0xFFu << (8 * jj) : 0u, lut_hi = jj < 4 ? 0u : 0xFFu << (8 * (jj - 4));
            const uint32_t eo = perm(lut_hi, lut_lo, j < 8 ? so_lo : so_hi);
            const uint32_t eh = perm(lut_hi, lut_lo, j < 8 ? shw_lo : shw_hi);
            Lc[j] = sel(eh, newHl, sel(eo, newOl, Lc[j]));
            M[j] = sel(eh, newHm, sel(eo, newOm, M[j]));
        }
        // holding: released on deliver / put down, the target slot on pick-up
        H[k] = sel(full80(deliver | put), kFF, sel(fpk, oidx, h));
    }

    // ---- new_obs = copy.copy(self) raises: two co-located agents both holding (ERR) ----
    uint32_t err = 0u;
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = i + 1; j < A; ++j) {
            const uint32_t same = z80(bop3<OC_LUT((a ^ b) | c)>(X[i], X[j], Y[i] ^ Y[j]));
            err |= and3(same, andn(k80, H[i]), andn(k80, H[j]));
        }
    err |= raise80;

    // ---- done() (:316-363) and reward() (:365-376) ----
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
    u16x2 t0 = __builtin_bit_cast(u16x2, T0) + one, t1 = __builtin_bit_cast(u16x2, T1) + one;
    uint32_t tout = 0u;
    if (L.maxT_rep != 0u) {  // t >= max_T first (:328-332): sat(max_T - t) == 0
        const u16x2 mt = __builtin_bit_cast(u16x2, L.maxT_rep);
        const uint32_t d0 = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(mt, t0));
        const uint32_t d1 = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(mt, t1));
        const uint32_t z0 = andn(0x80008000u, ((d0 & 0x7FFF7FFFu) + 0x7FFF7FFFu) | d0);
        const uint32_t z1 = andn(0x80008000u, ((d1 & 0x7FFF7FFFu) + 0x7FFF7FFFu) | d1);
        tout = perm(z1, z0, 0x07050301u);  // high byte of each u16 half -> env byte
    }
    T0 = __builtin_bit_cast(uint32_t, t0);
    T1 = __builtin_bit_cast(uint32_t, t1);
    F = 0u;
    CM = cm;
    if (!any_of(or3(rst, tout | err, dlv | pending))) return false;  // wave-uniform: no rare event
    pending = 0u;
    uint32_t ok = k80;
    for (int g = 0; g < L.ngoals; ++g) {  // every Deliver goal: an item == goal at the delivery cell
        uint32_t hit = 0u;
        if (big) {  // masks are < 0x80, so bit 7 of the OR comes from the cell compare only
#pragma unroll
            for (int j = 0; j < K; ++j) hit |= zf80((Lc[j] ^ L.done_rep) | (M[j] ^ L.goals_rep[g]));
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j)
                hit |= z80(bop3<OC_LUT((a | b) & c)>(Lc[j] ^ L.done_rep, M[j] ^ L.goals_rep[g], k7F));
        }
        ok &= hit;
    }
    const uint32_t done80 = or3(err, tout, ok);
    const uint32_t succ80 = bop3<OC_LUT(a & !b & !c)>(ok, err, tout);
    uint32_t fl = or3(done80 >> 7, succ80 >> 6, err >> 5);

    // ---- auto-reset of envs that were done at the input: the level template ----
#pragma unroll
    for (int a = 0; a < A; ++a) {
        OC_TIED_SEL(X[a], rst, L.tmpl_x[a]);
        OC_TIED_SEL(Y[a], rst, L.tmpl_y[a]);
        OC_TIED_OR(H[a], rst);
        OC_TIED_SEL(EX[a], rst, k04);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        OC_TIED_SEL(Lc[j], rst, L.tmpl_l[j]);
        OC_TIED_SEL(M[j], rst, L.tmpl_m[j]);
    }
    OC_TIED_ANDN(T0, perm(rst, rst, 0x01010000u));
    OC_TIED_ANDN(T1, perm(rst, rst, 0x03030202u));
    OC_TIED_OR(F, andn(fl, rst));
    OC_TIED_ANDN(CM, rst);
    return true;
}

// ---- wide levels (more than 255 cells): cells are u16, held as two byte words ----
// A cell-valued quantity of four envs is a pair of dwords, its low bytes and its high bytes (the
// wide state layout's two item-cell planes), so the step stays four envs
// per dword and every byte-valued field (agent x / y / held slot, item masks, actions, flags)
// keeps step4's byte arithmetic.  Cell arithmetic (y * W + x, the move) runs in packed u16
// lanes (v_pk_mad_u16 / v_pk_add_u16 / v_pk_sub_u16: no carry or borrow crosses a lane), two
// envs per dword, and is repacked into the two byte words.
struct Cell2 {
    uint32_t lo, hi;
};
OC_SW Cell2 csel(uint32_t m, const Cell2& a, const Cell2& b) { return Cell2{sel(m, a.lo, b.lo), sel(m, a.hi, b.hi)}; }
// h80 of (a == b) per env, all 16 bits
OC_SW uint32_t ceq80(const Cell2& a, const Cell2& b) {
    return zf80(bop3<OC_LUT((a ^ b) | c)>(a.hi, b.hi, a.lo ^ b.lo));
}
// h80 per env: some item of the env lies on the first Delivery square (wide levels)
template <int K>
OC_SW uint32_t at_done80w(const SwarLevel& L, const uint32_t (&LL)[K], const uint32_t (&LH)[K]) {
    uint32_t hit = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) hit |= zf80(bop3<OC_LUT((a ^ b) | c)>(LH[j], L.done_hi_rep, LL[j] ^ L.done_rep));
    return hit;
}

// step4 for a wide level: the same rules, in the same order (see step4 for the reference
// citations and the rare-event split); cells as Cell2 (LL / LH: the item slots' low / high
// bytes).  `cls_of(Cell2)` returns the tile class byte per env.
template <int A, int K, class ClassOf, class AnyOf>
OC_SW bool step4w(const SwarLevel& L, uint32_t (&X)[A], uint32_t (&Y)[A], uint32_t (&H)[A], uint32_t (&LL)[K],
                  uint32_t (&LH)[K], uint32_t (&M)[K], uint32_t& T0, uint32_t& T1, uint32_t& F,
                  const uint32_t (&ACT)[A], uint32_t (&EX)[A], uint32_t& CM, ClassOf cls_of, AnyOf any_of,
                  uint32_t& pending) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const bool counts = (bool)L.counts, edge = (bool)L.edge;
    const uint32_t rst = full80((F << 7) & k80);  // input DONE => next-step auto-reset
    const u16x2 wv = {(unsigned short)L.W, (unsigned short)L.W};

    uint32_t act[A], cls[A], nn80[A], bump80[A], blk80[A], out80[A];
    Cell2 loc[A], nraw[A], nxt[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        uint32_t c = ACT[a];
        const uint32_t ge5 = bop3<OC_LUT((a | b) & c)>((c & k7F) + 0x7B7B7B7Bu, c, k80);
        act[a] = sel(full80(ge5), k04, c);  // codes > 4 act as (0, 0)
        out80[a] = 0u;
    }
    uint32_t raise80 = 0u;
    if (edge) {  // an action off the grid (a Floor on the border): step4's off-grid raise
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const uint32_t c = act[a];
            out80[a] = or3(and3(z80(c), z80(Y[a] ^ L.hm1_rep), k80), and3(z80(c ^ k01), z80(Y[a]), k80),
                           and3(z80(c ^ 0x02020202u), z80(X[a]), k80) | and3(z80(c ^ 0x03030303u), z80(X[a] ^ L.wm1_rep), k80));
            if (A >= 2) raise80 |= out80[a];
        }
        if (A >= 2) {
#pragma unroll
            for (int a = 0; a < A; ++a) {
                act[a] = sel(full80(raise80), k04, act[a]);
                out80[a] = 0u;
            }
        }
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
        const uint32_t c = act[a];
        nn80[a] = nz80(c ^ k04);
        // envs 0 and 2 (selector bytes 0 and 2), envs 1 and 3 (1 and 3) as u16 lanes
        const u16x2 y02 = __builtin_bit_cast(u16x2, perm(0u, Y[a], 0x0C020C00u));
        const u16x2 y13 = __builtin_bit_cast(u16x2, perm(0u, Y[a], 0x0C030C01u));
        const u16x2 x02 = __builtin_bit_cast(u16x2, perm(0u, X[a], 0x0C020C00u));
        const u16x2 x13 = __builtin_bit_cast(u16x2, perm(0u, X[a], 0x0C030C01u));
        const u16x2 l02 = y02 * wv + x02, l13 = y13 * wv + x13;
        // the move: + max(delta, 0) - max(-delta, 0) (LUTs on the action code; a selector byte
        // 0x0C reads zero, so each u16 lane gets the byte value)
        const uint32_t s02 = perm(0x0C0C0C0Cu, c, 0x04020400u), s13 = perm(0x0C0C0C0Cu, c, 0x04030401u);
        const u16x2 n02 = l02 + __builtin_bit_cast(u16x2, perm(L.dp_hi, L.dp_lo, s02)) -
                          __builtin_bit_cast(u16x2, perm(L.dn_hi, L.dn_lo, s02));
        const u16x2 n13 = l13 + __builtin_bit_cast(u16x2, perm(L.dp_hi, L.dp_lo, s13)) -
                          __builtin_bit_cast(u16x2, perm(L.dn_hi, L.dn_lo, s13));
        const uint32_t L02 = __builtin_bit_cast(uint32_t, l02), L13 = __builtin_bit_cast(uint32_t, l13);
        const uint32_t N02 = __builtin_bit_cast(uint32_t, n02), N13 = __builtin_bit_cast(uint32_t, n13);
        loc[a] = Cell2{perm(L13, L02, 0x06020400u), perm(L13, L02, 0x07030501u)};
        nraw[a] = Cell2{perm(N13, N02, 0x06020400u), perm(N13, N02, 0x07030501u)};
        if (edge) nraw[a] = csel(full80(out80[a]), loc[a], nraw[a]);  // World.inbounds (one agent)
        cls[a] = cls_of(nraw[a]);
        const uint32_t onF80 = cls[a] & k80;
        nxt[a] = csel(full80(onF80), nraw[a], loc[a]);
        bump80[a] = andn(nn80[a], onF80);
        blk80[a] = 0u;
    }

    // ---- check_collisions: pairs in itertools.combinations order ----
    uint32_t cm = 0u;
    int p = 0;
#pragma unroll
    for (int i = 0; i < A; ++i) {
#pragma unroll
        for (int j = i + 1; j < A; ++j, ++p) {
            const uint32_t eq = ceq80(nxt[i], nxt[j]);
            const uint32_t sw = ceq80(loc[i], nxt[j]) & ceq80(loc[j], nxt[i]);
            const uint32_t bi = bop3<OC_LUT(a ? !b : c)>(eq, bump80[i], sw);
            const uint32_t u = bop3<OC_LUT((a | !b) & c)>(bump80[i], bump80[j], k80);
            const uint32_t bj = sel(eq, u, sw);
            blk80[i] |= bi;
            blk80[j] |= bj;
            cm |= (bi | bj) >> (7 - p);
        }
    }
    if (edge && A >= 2) cm = andn(cm, full80(raise80));

    // ---- execute_navigation: interact per agent, in order ----
    uint32_t dlv = 0u;
#pragma unroll
    for (int k = 0; k < A; ++k) {
        const uint32_t go80 = andn(nn80[k], blk80[k]);
        EX[k] = sel(full80(go80), act[k], k04);
        const Cell2 tc = nraw[k];
        const uint32_t isF80 = cls[k] & k80;
        const uint32_t isD80 = (cls[k] << 1) & k80;
        const uint32_t isC80 = (cls[k] << 2) & k80;
        const uint32_t h = H[k];
        const uint32_t hold80 = andn(k80, h);
        uint32_t ne[K];  // bit 7: slot j is NOT at tc
#pragma unroll
        for (int j = 0; j < K; ++j) ne[j] = ~zf80(bop3<OC_LUT((a ^ b) | c)>(LH[j], tc.hi, LL[j] ^ tc.lo));
        auto any_at = [&](auto pick) -> uint32_t {
            uint32_t all = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (pick(j)) all &= ne[j];
            return andn(k80, all);
        };
        const uint32_t seen = any_at([](int) { return true; });
        const uint32_t ob0 = any_at([](int j) { return (j & 1) != 0; });
        const uint32_t ob1 = any_at([](int j) { return (j & 2) != 0; });
        const uint32_t ob2 = K > 4 ? any_at([](int j) { return (j & 4) != 0; }) : 0u;
        const uint32_t ob3 = K > 8 ? any_at([](int j) { return (j & 8) != 0; }) : 0u;
        const uint32_t so1 = (ob0 >> 5) | kLanes;
        const uint32_t sh = bop3<OC_LUT((a & b) | c)>(h << 2, k04, kLanes);
        uint32_t om, hm;
        if constexpr (K == 4) {
            const uint32_t so2 = (ob1 >> 5) | kLanes, sh2 = bop3<OC_LUT(a | (b & c))>(kLanes, h << 1, k04);
            om = perm(perm(M[3], M[2], so1), perm(M[1], M[0], so1), so2);
            hm = perm(perm(M[3], M[2], sh), perm(M[1], M[0], sh), sh2);
        } else {
            const uint32_t fo1 = full80(ob1), fo2 = full80(ob2), fo3 = K == 16 ? full80(ob3) : 0u;
            const uint32_t fh1 = full80((h << 6) & k80), fh2 = full80((h << 5) & k80);
            const uint32_t fh3 = K == 16 ? full80((h << 4) & k80) : 0u;
            om = gather<K>(M, so1, fo1, fo2, fo3);
            hm = gather<K>(M, sh, fh1, fh2, fh3);
        }
        const uint32_t nf = andn(go80, isF80), mv = andn(go80 & isF80, out80[k]);
        uint32_t two_r, nallch_r, nplate_r, nfood_r, nch_r, cu, chopped;
        if (counts) {
            const uint32_t x = hm & k7F;
            two_r = bop3<OC_LUT((a & b) | c)>((x | k80) - k01, x, x & 0x2A2A2A2Au) + k7F;
            nallch_r = 0u;
            nplate_r = and3(hm, om, 0x40404040u) + k7F;
            nfood_r = hm | om;
            nch_r = hm;
            cu = x + (om & k7F);
            chopped = x;
        } else {
            const uint32_t c4 = hm & k0F;
            two_r = (((c4 | k80) - k01) & c4) + k7F;
            nallch_r = bop3<OC_LUT((!a) & b & c)>(hm >> 4, hm, k07) + k7F;
            cu = hm | om;
            nplate_r = and3(hm, om, k08) + k7F;
            nfood_r = bop3<OC_LUT((!a) & b & c)>(cu >> 4, cu, k07) + k7F;
            nch_r = bop3<OC_LUT(a & !b & !c)>(c4 + k7F, two_r, (hm & k78) + k7F);
            chopped = bop3<OC_LUT((a & b) | c)>(hm << 4, 0x70707070u, hm);
        }
        const uint32_t nfh = nf & hold80;
        const uint32_t deliver = bop3<OC_LUT(a & b & !c)>(nfh & isD80, two_r, nallch_r);
        const uint32_t cnt = andn(nfh, isD80);
        const uint32_t merge = bop3<OC_LUT(a & b & !c)>(cnt, seen, nplate_r | nfood_r);
        const uint32_t empty = andn(cnt, seen);
        const uint32_t chop = and3(empty, isC80, nch_r);
        const uint32_t put = andn(empty, chop);
        const uint32_t pick = andn(bop3<OC_LUT(a & !b & c)>(nf, hold80, seen), isD80);
        const uint32_t reloc = or3(mv, deliver, put);
        dlv |= deliver;

        const uint32_t amv = bop3<OC_LUT(a | ((!b) & c))>(act[k], mv >> 5, k04);
        X[k] = X[k] + perm(kDXhi, kDXlo, amv) - k01;
        Y[k] = Y[k] + perm(kDYhi, kDYlo, amv) - k01;
        const uint32_t fmg = full80(merge), fpk = full80(pick);
        const Cell2 newOl = {fmg | sel(fpk, loc[k].lo, tc.lo), fmg | sel(fpk, loc[k].hi, tc.hi)};  // merged away: 0xFFFF
        const uint32_t newOm = andn(om, fmg);
        const Cell2 newHl = csel(full80(reloc), tc, loc[k]);
        const uint32_t newHm = sel(fmg, cu, sel(full80(chop), chopped, hm));
        const uint32_t oidx = (ob0 >> 7) | (ob1 >> 6) | (ob2 >> 5) | (ob3 >> 4);
        const uint32_t fwo = full80(merge | pick);
        const uint32_t fwh = full80(and3(hold80, or3(reloc, merge, chop), k80));
        const uint32_t so = sel(fwo, oidx, 0x0C0C0C0Cu), shw = sel(fwh, h, 0x0C0C0C0Cu);
        uint32_t so_lo = so, shw_lo = shw, so_hi = 0x0C0C0C0Cu, shw_hi = 0x0C0C0C0Cu;
        if constexpr (K == 16) {
            const uint32_t o8 = full80(and3(oidx << 4, k80, fwo)), h8 = full80(and3(h << 4, k80, fwh));
            so_lo = sel(o8, 0x0C0C0C0Cu, so);
            shw_lo = sel(h8, 0x0C0C0C0Cu, shw);
            so_hi = sel(o8, oidx ^ 0x08080808u, 0x0C0C0C0Cu);
            shw_hi = sel(h8, h ^ 0x08080808u, 0x0C0C0C0Cu);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int jj = j & 7;
            const uint32_t lut_lo = jj < 4 ? 0xFFu << (8 * jj) : 0u, lut_hi = jj < 4 ? 0u : 0xFFu << (8 * (jj - 4));
            const uint32_t eo = perm(lut_hi, lut_lo, j < 8 ? so_lo : so_hi);
            const uint32_t eh = perm(lut_hi, lut_lo, j < 8 ? shw_lo : shw_hi);
            LL[j] = sel(eh, newHl.lo, sel(eo, newOl.lo, LL[j]));
            LH[j] = sel(eh, newHl.hi, sel(eo, newOl.hi, LH[j]));
            M[j] = sel(eh, newHm, sel(eo, newOm, M[j]));
        }
        H[k] = sel(full80(deliver | put), kFF, sel(fpk, oidx, h));
    }

    // ---- the copy crash: two co-located agents both holding (ERR) ----
    uint32_t err = 0u;
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = i + 1; j < A; ++j) {
            const uint32_t same = z80(bop3<OC_LUT((a ^ b) | c)>(X[i], X[j], Y[i] ^ Y[j]));
            err |= and3(same, andn(k80, H[i]), andn(k80, H[j]));
        }
    err |= raise80;

    // ---- done() and reward() ----
    const u16x2 one = {1, 1};
    u16x2 t0 = __builtin_bit_cast(u16x2, T0) + one, t1 = __builtin_bit_cast(u16x2, T1) + one;
    uint32_t tout = 0u;
    if (L.maxT_rep != 0u) {
        const u16x2 mt = __builtin_bit_cast(u16x2, L.maxT_rep);
        const uint32_t d0 = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(mt, t0));
        const uint32_t d1 = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(mt, t1));
        const uint32_t z0 = andn(0x80008000u, ((d0 & 0x7FFF7FFFu) + 0x7FFF7FFFu) | d0);
        const uint32_t z1 = andn(0x80008000u, ((d1 & 0x7FFF7FFFu) + 0x7FFF7FFFu) | d1);
        tout = perm(z1, z0, 0x07050301u);
    }
    T0 = __builtin_bit_cast(uint32_t, t0);
    T1 = __builtin_bit_cast(uint32_t, t1);
    F = 0u;
    CM = cm;
    if (!any_of(or3(rst, tout | err, dlv | pending))) return false;  // wave-uniform: no rare event
    pending = 0u;
    uint32_t ok = k80;
    for (int g = 0; g < L.ngoals; ++g) {
        uint32_t hit = 0u;
#pragma unroll
        for (int j = 0; j < K; ++j)
            hit |= zf80(or3(LL[j] ^ L.done_rep, LH[j] ^ L.done_hi_rep, M[j] ^ L.goals_rep[g]));
        ok &= hit;
    }
    const uint32_t done80 = or3(err, tout, ok);
    const uint32_t succ80 = bop3<OC_LUT(a & !b & !c)>(ok, err, tout);
    uint32_t fl = or3(done80 >> 7, succ80 >> 6, err >> 5);
#pragma unroll
    for (int a = 0; a < A; ++a) {
        OC_TIED_SEL(X[a], rst, L.tmpl_x[a]);
        OC_TIED_SEL(Y[a], rst, L.tmpl_y[a]);
        OC_TIED_OR(H[a], rst);
        OC_TIED_SEL(EX[a], rst, k04);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        OC_TIED_SEL(LL[j], rst, L.tmpl_l[j]);
        OC_TIED_SEL(LH[j], rst, L.tmpl_lh[j]);
        OC_TIED_SEL(M[j], rst, L.tmpl_m[j]);
    }
    OC_TIED_ANDN(T0, perm(rst, rst, 0x01010000u));
    OC_TIED_ANDN(T1, perm(rst, rst, 0x03030202u));
    OC_TIED_OR(F, andn(fl, rst));
    OC_TIED_ANDN(CM, rst);
    return true;
}

// The step without the rare-event split (every wave takes the full path).
template <int A, int K, class ClassOf>
OC_SW void step4(const SwarLevel& L, uint32_t (&X)[A], uint32_t (&Y)[A], uint32_t (&H)[A],
                 uint32_t (&Lc)[K], uint32_t (&M)[K], uint32_t& T0, uint32_t& T1, uint32_t& F,
                 const uint32_t (&ACT)[A], uint32_t (&EX)[A], uint32_t& CM, ClassOf cls_of) {
    uint32_t pending = kFF;
    step4<A, K>(L, X, Y, H, Lc, M, T0, T1, F, ACT, EX, CM, cls_of, [](uint32_t) { return true; }, pending);
}

}  // namespace ocsw
