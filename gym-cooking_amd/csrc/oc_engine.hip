// oc_engine.hip -- MI355X (gfx950) batched Overcooked step engine + its C-ABI (include/oc_engine.h).
//
// Kernels:
//   oc_step_kernel    one env transition over the batch.  The state is structure-of-arrays byte
//                     planes; a lane owns 4 consecutive envs (one dword per
//                     plane, 256 B per wave-instruction) and steps them as SWAR (oc_swar.h):
//                       pairwise collision resolution  <- check_collisions / is_collision
//                                                         (gym_cooking/envs/overcooked_environment.py:671-762)
//                       sequential per-agent interact  <- execute_navigation + interact
//                                                         (overcooked_environment.py:767-770, utils/interact.py:4-89)
//                       the copy-crash (ERR) condition <- new_obs = copy.copy(self) (:289, :108-113)
//                       done() / reward()              <- overcooked_environment.py:316-376
//                     Tile classes come from a 256-byte LDS table per block; the grid is
//                     persistent and software-pipelined (next chunk's loads before this step).
//   oc_step_n_kernel  n steps per launch with the state in registers; every step's state,
//                     executed actions and collision mask are still written.
//   oc_rollout_kernel navigation-planner rollout rows (oc_rollout.h).
//   oc_bounds_kernel  full-state subtask lower bounds + allocation feasibility (oc_subtask_bounds).
//   oc_render_kernel  image observations.
//   reset / gen_actions / checksum / stats_reduce helpers.
// All of them accumulate nothing on the host; statistics are per-block rows of no-return
// 64-bit atomics reduced by oc_stats_reduce for the all-gather of episode summaries.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "../../include/oc_engine.h"
#include "oc_rollout.h"
#include "oc_swar.h"

namespace {

constexpr int kBlock = 256;  // 4 waves
constexpr int kStepBlock = 128;  // oc_step_kernel: 2 waves
constexpr int kEPL = 4;      // envs per lane: one dword per byte plane
constexpr int kEnvsPerBlock = kBlock * kEPL;

// Kernel argument block: everything static about the level, passed by value (SGPRs).
struct LevelArgs {
    uint32_t cls4[64];    // tile class byte of cell c (ocsw::tile_class) in byte c % 4 of word c / 4;
                          // cells >= W*H (up to 255, 0xFF = dead) read 0
    uint64_t dcell_lut;   // per action code: signed cell delta + 128 (byte lanes 0..4)
    int32_t W, H;
    int32_t done_cell;    // first Delivery in scan order (done() reads only it, :349)
    int32_t max_T;        // 0 = no limit
    uint32_t goals;       // up to 4 goal masks, one per byte
    int32_t ngoals;
    uint32_t tmpl_x, tmpl_y;          // spawn x / y of agents 0..3, one per byte
    uint32_t tmpl_cell[4], tmpl_mask[4];  // item slots 0..15, one per byte
    int64_t pitch;
    int64_t B;
    ocsw::SwarLevel sw;  // replicated constants / LUTs of the SWAR step
};

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int j) { return (w >> (8 * j)) & 0xFFu; }
__device__ __forceinline__ uint32_t byte_of4(const uint32_t (&w)[4], int j) { return byte_of(w[j >> 2], j & 3); }

// Statistics partial sums, one row of OC_NSTATS uint64 per block.  Wave sum over DPP (VALU
// lane moves, no LDS round trips): an inclusive scan inside each 16-lane row (row_shr 1, 2,
// 4, 8), then row 0's and row 1's totals broadcast into the rows above (row_bcast 15 / 31);
// lane 63 ends with the wave total.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Wave-uniform "some env of the wave": the step's rare-event split (ocsw::step4).
struct WaveAny {
    __device__ __forceinline__ bool operator()(uint32_t v) const { return __ballot(v != 0u) != 0ull; }
};

// One lane's slice of the batch: kEPL consecutive envs, one dword per byte plane.
template <int A, int K>
struct Chunk {
    uint32_t wx[A], wy[A], wh[A], wa[A], wl[K], wm[K];
    uint2 wt;
    uint32_t wf;
};

// Buffer resources of one launch: every plane access is a buffer load/store with the lane's
// 32-bit byte offset in a VGPR and the plane offset (plane * pitch) in an SGPR, so no per-
// access 64-bit address arithmetic is spent on the VALU.
struct Bufs {
    __amdgpu_buffer_rsrc_t sin, sout, act, ex, coll;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <int CP = 0>
__device__ __forceinline__ uint32_t bld32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, CP);
}
// Store cache policy (gfx950 CPol bits of the buffer intrinsics): 0 plain, 2 nt, 16 sc1,
// 17 sc0 sc1.  sc1 stores leave no dirty line in the XCD's L2, so the bytes go out to HBM
// while the kernel still computes instead of in the write-back at the kernel boundary (which
// costs about B / 6 TB/s for B dirty bytes, MI355X_MICROARCH.md "boundary").
// oc_step_n, whose trajectory stream is far larger than L2, is faster with nt stores instead
// (tools/stepexp.hip: 4.3 vs 5.2-5.3 us/step at 2^20 envs; sc1 5.3).
constexpr int kCPsc1 = 16, kCPnt = 2;
#ifndef OC_STEP_CP
// oc_step's store policy.  nt measured slower for it (hipGraphs of 20 oc_step launches,
// tools/step_ab.py --per-step, profiles/r04/perstep_nt/: 8.03 vs 8.9-9.5 us/step at A = 2,
// 9.4-9.5 vs 12.0-12.2 at A = 3, same outputs), so oc_step keeps sc1.
#define OC_STEP_CP kCPsc1
#endif
template <int CP = 0>
__device__ __forceinline__ void bst32(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, (int)soff, CP);
}

template <int A, int K, bool kActs = true>
__device__ __forceinline__ void load_chunk(Chunk<A, K>& c, const Bufs& b, uint32_t P, uint32_t g) {
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    const uint32_t vo = g * 4u;
#pragma unroll
    for (int a = 0; a < A; ++a) {
        c.wx[a] = bld32(b.sin, vo, a * P);
        c.wy[a] = bld32(b.sin, vo, (kPY + a) * P);
        c.wh[a] = bld32(b.sin, vo, (kPH + a) * P);
        if (kActs) c.wa[a] = bld32(b.act, vo, a * P);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        c.wl[j] = bld32(b.sin, vo, (kPL + j) * P);
        c.wm[j] = bld32(b.sin, vo, (kPM + j) * P);
    }
    const auto t = __builtin_amdgcn_raw_buffer_load_b64(b.sin, (int)(g * 8u), (int)(kPT * P), 0);
    c.wt = make_uint2(t[0], t[1]);
    c.wf = bld32(b.sin, vo, kPF * P);
}

// Per-lane episode counters; at the end of the kernel a wave sums them and lane 0 adds them
// to the block's stats row with no-return 64-bit atomics.
struct StepStats {
    uint32_t eps = 0u, succ = 0u, err = 0u, coll = 0u, steps = 0u;
};

// Step the kEPL envs of chunk c (SWAR, oc_swar.h) and store every output plane word of lane g.
template <int A, int K, int CP = 0, int MODE = 1>
__device__ __forceinline__ void step_chunk(const LevelArgs& L, const uint8_t* tbl, Chunk<A, K>& c, const Bufs& b,
                                           bool has_ex, bool has_coll, uint32_t P, uint32_t g, StepStats& st) {
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    auto cls_of = [tbl](uint32_t cells) -> uint32_t {
        const uint32_t b0 = tbl[cells & 0xFFu], b1 = tbl[(cells >> 8) & 0xFFu], b2 = tbl[(cells >> 16) & 0xFFu],
                       b3 = tbl[cells >> 24];
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    };
    const uint32_t f_in = c.wf;
    uint32_t T0 = c.wt.x, T1 = c.wt.y, ex[A], cm;
    uint32_t pending = ocsw::at_done80<K, MODE>(L.sw, c.wl);  // a loaded state: the full path once
    const bool full = ocsw::step4<A, K, MODE>(L.sw, c.wx, c.wy, c.wh, c.wl, c.wm, T0, T1, c.wf, c.wa, ex, cm,
                                              cls_of, WaveAny{}, pending);

    // statistics over the valid envs: an episode ended iff DONE is newly set (only on the
    // full path: without a rare event no flag is set)
    const int64_t rem = L.B - (int64_t)g * kEPL;
    const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (1u << (8 * (uint32_t)rem)) - 1u);
    st.coll += __popc(cm & vmask);
    if (full) {
        const uint32_t ended = (c.wf & ~f_in & vmask) & ocsw::k01;  // bit0 per env
        st.eps += __popc(ended);
        st.succ += __popc(c.wf & (ended << 1));
        st.err += __popc(c.wf & (ended << 2));
        const uint32_t efull = (0x80808080u - ended) ^ 0x80808080u;  // 0x01 -> 0xFF per byte, no multiply
        const uint32_t e16a = __builtin_amdgcn_perm(0u, efull, 0x01010000u);  // env 0,1 -> u16 masks
        const uint32_t e16b = __builtin_amdgcn_perm(0u, efull, 0x03030202u);  // env 2,3
        const uint32_t sa = T0 & e16a, sb = T1 & e16b;
        st.steps += (sa & 0xFFFFu) + (sa >> 16) + (sb & 0xFFFFu) + (sb >> 16);
    }

    const uint32_t vo = g * 4u;
#pragma unroll
    for (int a = 0; a < A; ++a) {
        bst32<CP>(b.sout, c.wx[a], vo, a * P);
        bst32<CP>(b.sout, c.wy[a], vo, (kPY + a) * P);
        bst32<CP>(b.sout, c.wh[a], vo, (kPH + a) * P);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        bst32<CP>(b.sout, c.wl[j], vo, (kPL + j) * P);
        bst32<CP>(b.sout, c.wm[j], vo, (kPM + j) * P);
    }
    typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
    const u32x2 tw = {T0, T1};
    __builtin_amdgcn_raw_buffer_store_b64(tw, b.sout, (int)(g * 8u), (int)(kPT * P), CP);
    bst32<CP>(b.sout, c.wf, vo, kPF * P);
    if (has_ex) {
#pragma unroll
        for (int a = 0; a < A; ++a) bst32<CP>(b.ex, ex[a], vo, a * P);
    }
    if (has_coll) bst32<CP>(b.coll, cm, vo, 0u);
}

// One step over the batch: one chunk (kEPL envs) per lane, 128-thread blocks, a grid that
// covers the whole batch at once (P / 512 blocks, ~4 waves per SIMD resident at 2^20 envs).
// Each lane issues its chunk's loads first, then the block builds its tile-class table while
// they are in flight.  Measured on MI355X (tools/stepexp.hip, 2^20 envs, hipGraph of 100
// ping-pong steps): 9.1 us/step, against 11.1 for a persistent 2-blocks-per-CU grid with a
// software-pipelined chunk loop (2 chunks per lane at this size: mostly ramp and drain),
// 10.2 with 256-thread blocks, 9.1 with 2 chunks per lane, and 6.5 for the same loads and
// stores with no compute.  Staggering block start times did not help (9.2-9.3).
template <int A, int K, int MODE>
__global__ __launch_bounds__(kStepBlock) void oc_step_kernel(LevelArgs L, const uint8_t* __restrict__ sin,
                                                             uint8_t* __restrict__ sout,
                                                             const uint8_t* __restrict__ actions,
                                                             uint8_t* __restrict__ exec_out,
                                                             uint8_t* __restrict__ coll_out,
                                                             uint64_t* __restrict__ stats, uint32_t stat_rows) {
    const uint32_t P = (uint32_t)L.pitch;  // state <= 2 GiB (checked on the host)
    constexpr int NP = 3 * A + 2 * K + 3;
    Bufs b;
    b.sin = make_rsrc(sin, (int64_t)NP * P);
    b.sout = make_rsrc(sout, (int64_t)NP * P);
    b.act = make_rsrc(actions, (int64_t)A * P);
    const bool has_ex = exec_out != nullptr, has_coll = coll_out != nullptr;
    b.ex = make_rsrc(has_ex ? (const void*)exec_out : (const void*)sout, (int64_t)A * P);
    b.coll = make_rsrc(has_coll ? (const void*)coll_out : (const void*)sout, (int64_t)P);
    const uint32_t g = blockIdx.x * (uint32_t)kStepBlock + threadIdx.x;  // grid * kStepBlock == P / kEPL
    Chunk<A, K> c;
    load_chunk<A, K>(c, b, P, g);  // in flight while the block builds its table
    // tile class per cell (bit7 Floor, bit6 Delivery, bit5 Cutboard); cells past the grid read 0.
    // Lane 0 writes the 64 table words from scalar kernel-argument loads (no vector memory
    // access, so nothing waits behind the chunk loads) and the table is published with an
    // LDS-only workgroup fence around the barrier (a plain __syncthreads would also wait for
    // the chunk loads).
    __shared__ uint32_t tbl4[64];
    if (threadIdx.x == 0u) {
#pragma unroll
        for (int i = 0; i < 64; ++i) tbl4[i] = L.cls4[i];
    }
    const uint8_t* tbl = (const uint8_t*)tbl4;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    StepStats st;
    step_chunk<A, K, OC_STEP_CP, MODE>(L, tbl, c, b, has_ex, has_coll, P, g, st);
    if (stats != nullptr) {  // wave sums, then fire-and-forget 64-bit atomics into this block's row
        const uint32_t v[OC_NSTATS] = {wave_sum(st.eps), wave_sum(st.succ), wave_sum(st.steps), wave_sum(st.coll),
                                       wave_sum(st.err)};
        if ((threadIdx.x & 63u) == 0u) {
            unsigned long long* row = (unsigned long long*)stats + (int64_t)(blockIdx.x % stat_rows) * OC_NSTATS;
#pragma unroll
            for (int q = 0; q < OC_NSTATS; ++q)
                if (v[q]) atomicAdd(row + q, (unsigned long long)v[q]);
        }
    }
}

// oc_step_n: n consecutive steps per launch.  Each lane loads its chunk's state once, then
// for every step reads that step's actions (prefetched two steps ahead), steps in registers
// and writes the step's outputs: the full state into traj[r] (when given), the executed
// actions and the collision mask; the state after the last step goes to sout (null when sout
// is the trajectory's last state: that store already wrote it).  Outputs are
// byte-identical to n oc_step launches with ping-pong buffers.
// oc_step_n's completion tickets, after the statistics rows (at a 128-byte boundary, one
// 128-byte line each): [0] counts finished groups, [1 + g] the finished blocks of group g
// (kTicketGroup consecutive blocks).  Every counter is back at zero when a launch ends.
constexpr int kTicketGroup = 32, kTicketStride = 16;  // u64 units
constexpr int64_t kStatRows = 256;  // statistics rows (stats_rows: fewer for small batches)
__host__ __device__ constexpr int64_t ticket_base(int64_t stat_rows) {
    return (stat_rows * OC_NSTATS + kTicketStride - 1) / kTicketStride * kTicketStride;
}

// Loader wave (LW).  A wave that has stores outstanding and consumes a loaded word waits for
// every one of those stores: the compiler emits vmcnt(0) there (loads and stores share the
// counter on gfx950, and it does not take them to complete in order).  With each step's action
// words loaded by the stepping wave, every wave waited at every step for the stores of the step
// before to drain: C3 (3 agents) ran 6.4 us/step, and 5.1 with the action loads taken out of
// the loop (tools/c3_floor.py, profiles/r03/lw/).  With LW, a block has a fifth wave that only
// loads: it fetches the next kLwSteps steps' action words of the block's 256 lanes into one half
// of an LDS ring while the four stepping waves read theirs from the other half, and an
// LDS-only barrier per kLwSteps steps hands the halves over (no vmcnt wait; the stepping waves
// issue no vector load after their state).  Only the loader waits on memory, for loads alone.
// Handing the ring over with per-step LDS flags instead (the loader publishes steps filled,
// each stepping wave the steps it took; a ring of 8 steps, s_sleep polls, no barrier) was
// measured slower: C3 100-step launches 6.28-6.41 us/step against 6.06-6.12 with the barrier,
// four alternating rounds on one box, outputs identical (profiles/r04/lw_flags_ab.jsonl).
#ifndef OC_LW_STEPS
#define OC_LW_STEPS 4
#endif

// Also measured and dropped (round 4, profiles/r04/lw_stagger/): a staggered hand-over, the odd
// stepping waves meeting batch k's barrier between the compute and the stores of step 4k - 1
// (so that at each release the even waves compute while the odd ones store): 6.46-6.51 us/step
// against 6.04-6.07, four alternating rounds on one box, C3 parity tests green on it; and the
// loader's loads as 16-byte loads (16 lanes per 256-byte group, a quarter of the load and LDS
// write instructions): 6.18-6.29 against 6.05-6.12 (profiles/r04/lw_x4/).
constexpr int kLwSteps = OC_LW_STEPS;  // steps per ring half (one barrier per kLwSteps steps)
// A = 3 only: there the stepping waves' drains were a fifth of the time (C3, 100-step launches,
// one box: 6.42 -> 6.07 us/step, outputs identical).  At A <= 2 the step is store-bound and the
// block-wide barrier every kLwSteps steps costs more than the drains (2 agents, 20-step launch:
// 4.60 -> 4.70 us/step; 100-step: 4.20 -> 4.22); A = 4 needs more than 102 VGPRs.
constexpr bool kLoaderWave = true;
template <int A, int K, int MODE>
constexpr bool use_loader_wave() { return kLoaderWave && A == 3 && K == 4; }
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int A, int K, int CP, int LCP, int MODE, bool LW = use_loader_wave<A, K, MODE>()>
__global__ __launch_bounds__(kBlock + (LW ? 64 : 0), LW ? 5 : 1) void oc_step_n_kernel(LevelArgs L, const uint8_t* __restrict__ sin,
                                                           uint8_t* __restrict__ sout,
                                                           const uint8_t* __restrict__ actions,
                                                           uint8_t* __restrict__ traj, uint8_t* __restrict__ exec_out,
                                                           uint8_t* __restrict__ coll_out,
                                                           uint64_t* __restrict__ stats, uint64_t* __restrict__ totals,
                                                           uint32_t stat_rows, int n) {
    __shared__ uint32_t tbl4[64];
    __shared__ uint32_t waves_done;
    __shared__ unsigned long long fold[OC_NSTATS][64 + 8];  // the folding wave's partial sums
    // LW: [half][step of the batch][stepping wave][agent][lane] action words
    __shared__ uint32_t ring[LW ? 2 * kLwSteps * (kBlock / 64) * A * 64 : 1];
    if (threadIdx.x < 64u) tbl4[threadIdx.x] = L.cls4[threadIdx.x];
    if (threadIdx.x == 0u) waves_done = 0u;
    __syncthreads();
    const bool loader = LW && threadIdx.x >= (uint32_t)kBlock;  // wave-uniform
    const uint32_t lane = threadIdx.x & 63u;
    const uint8_t* tbl = (const uint8_t*)tbl4;
    const uint32_t P = (uint32_t)L.pitch, nlanes = P / kEPL, stride = gridDim.x * (uint32_t)kBlock;
    constexpr int NP = 3 * A + 2 * K + 3;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    auto cls_of = [&](uint32_t cells) -> uint32_t {
        const uint32_t b0 = tbl[cells & 0xFFu], b1 = tbl[(cells >> 8) & 0xFFu], b2 = tbl[(cells >> 16) & 0xFFu],
                       b3 = tbl[cells >> 24];
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    };
    Bufs b;
    b.sin = make_rsrc(sin, (int64_t)NP * P);
    b.sout = make_rsrc(sout ? (const void*)sout : (const void*)sin, sout ? (int64_t)NP * P : 0);  // null: stores dropped
    b.act = make_rsrc(actions, (int64_t)n * A * P);
    const bool has_tr = traj != nullptr, has_ex = exec_out != nullptr, has_coll = coll_out != nullptr;
    const __amdgpu_buffer_rsrc_t tr = make_rsrc(has_tr ? (const void*)traj : (const void*)sin, has_tr ? (int64_t)n * NP * P : 0);
    b.ex = make_rsrc(has_ex ? (const void*)exec_out : (const void*)sin, has_ex ? (int64_t)n * A * P : 0);
    b.coll = make_rsrc(has_coll ? (const void*)coll_out : (const void*)sin, has_coll ? (int64_t)n * P : 0);
    StepStats st;
    typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
    for (uint32_t gb = blockIdx.x * (uint32_t)kBlock; gb < nlanes; gb += stride) {  // block-uniform
        if (loader) {
            // the action words of steps r0 .. r0 + kLwSteps - 1 (those < n) into ring half h;
            // this wave issues no store, so its waits are for its own loads only
            auto fill = [&](int r0, int h) {
                uint32_t w[kLwSteps][kBlock / 64][A];
#pragma unroll
                for (int q = 0; q < kLwSteps; ++q)
#pragma unroll
                    for (int v = 0; v < kBlock / 64; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            w[q][v][a] = r0 + q < n ? bld32<LCP>(b.act, (gb + 64u * v + lane) * 4u,
                                                                 (uint32_t)((r0 + q) * A + a) * P)
                                                    : 0u;
#pragma unroll
                for (int q = 0; q < kLwSteps; ++q)
#pragma unroll
                    for (int v = 0; v < kBlock / 64; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            ring[(((h * kLwSteps + q) * (kBlock / 64) + v) * A + a) * 64 + lane] = w[q][v][a];
            };
            fill(0, 0);
            for (int r0 = 0; r0 < n; r0 += kLwSteps) {
                lds_barrier();  // half (r0 / kLwSteps) & 1 is full; the other one has been read
                if (r0 + kLwSteps < n) fill(r0 + kLwSteps, ((r0 / kLwSteps) & 1) ^ 1);
            }
            lds_barrier();  // the chunk's last batch has been read: the next chunk may refill
            continue;
        }
        const uint32_t g = gb + threadIdx.x;
        Chunk<A, K> c;
        load_chunk<A, K, !LW>(c, b, P, g);
        // the state words land before the step loop: waited for at their first use inside the
        // loop, the wait (vmcnt(0) for the last of them) would stay in the loop body and drain
        // every step's stores (an s_waitcnt the compiler's waitcnt pass sees and accounts for)
        if (LW) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt untouched
        const uint32_t vo = g * 4u;
        uint32_t T0 = c.wt.x, T1 = c.wt.y, nxt[A];
        uint32_t pending = ocsw::at_done80<K, MODE>(L.sw, c.wl);  // the loaded state: the full path once
        const int64_t rem = L.B - (int64_t)g * kEPL;
        const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (1u << (8 * (uint32_t)rem)) - 1u);
        if (!LW) {
#pragma unroll
            for (int a = 0; a < A; ++a) nxt[a] = n > 1 ? bld32<LCP>(b.act, vo, (uint32_t)(A + a) * P) : 0u;
        }
        for (int r = 0; r < n; ++r) {
            uint32_t act[A], ex[A], cm;
            if (LW) {
                const int q = r % kLwSteps;
                if (q == 0) lds_barrier();  // the loader has filled this batch's half
                const int h = (r / kLwSteps) & 1;
#pragma unroll
                for (int a = 0; a < A; ++a)
                    act[a] = ring[(((h * kLwSteps + q) * (kBlock / 64) + (threadIdx.x >> 6)) * A + a) * 64 + lane];
            } else {
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    act[a] = c.wa[a];
                    c.wa[a] = nxt[a];
                }
                if (r + 2 < n) {
#pragma unroll
                    for (int a = 0; a < A; ++a) nxt[a] = bld32<LCP>(b.act, vo, (uint32_t)((r + 2) * A + a) * P);
                }
            }
            const uint32_t f_in = c.wf;
            const bool full = ocsw::step4<A, K, MODE>(L.sw, c.wx, c.wy, c.wh, c.wl, c.wm, T0, T1, c.wf, act, ex,
                                                      cm, cls_of, WaveAny{}, pending);
            st.coll += __popc(cm & vmask);
            if (full) {  // episode ends only on the full path
                const uint32_t ended = (c.wf & ~f_in & vmask) & ocsw::k01;
                st.eps += __popc(ended);
                st.succ += __popc(c.wf & (ended << 1));
                st.err += __popc(c.wf & (ended << 2));
                const uint32_t efull = (0x80808080u - ended) ^ 0x80808080u;  // no multiply
                const uint32_t sa = T0 & __builtin_amdgcn_perm(0u, efull, 0x01010000u);
                const uint32_t sb2 = T1 & __builtin_amdgcn_perm(0u, efull, 0x03030202u);
                st.steps += (sa & 0xFFFFu) + (sa >> 16) + (sb2 & 0xFFFFu) + (sb2 >> 16);
            }
            // Unconditional stores: an absent output's descriptor has num_records 0, so its
            // stores are dropped by the buffer range check.  Guarding them with branches made
            // the waitcnt pass merge a store-free path into the loop back-edge and wait for
            // every store of the step (vmcnt(0)) before taking the next step's action words.
            const uint32_t base = (uint32_t)r * NP * P;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                bst32<CP>(tr, c.wx[a], vo, base + a * P);
                bst32<CP>(tr, c.wy[a], vo, base + (kPY + a) * P);
                bst32<CP>(tr, c.wh[a], vo, base + (kPH + a) * P);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                bst32<CP>(tr, c.wl[j], vo, base + (kPL + j) * P);
                bst32<CP>(tr, c.wm[j], vo, base + (kPM + j) * P);
            }
            const u32x2 tw = {T0, T1};
            __builtin_amdgcn_raw_buffer_store_b64(tw, tr, (int)(g * 8u), (int)(base + kPT * P), CP);
            bst32<CP>(tr, c.wf, vo, base + kPF * P);
#pragma unroll
            for (int a = 0; a < A; ++a) bst32<CP>(b.ex, ex[a], vo, (uint32_t)(r * A + a) * P);
            bst32<CP>(b.coll, cm, vo, (uint32_t)r * P);
        }
        if (LW) lds_barrier();  // pairs with the loader's end-of-chunk barrier
#pragma unroll
        for (int a = 0; a < A; ++a) {
            bst32<CP>(b.sout, c.wx[a], vo, a * P);
            bst32<CP>(b.sout, c.wy[a], vo, (kPY + a) * P);
            bst32<CP>(b.sout, c.wh[a], vo, (kPH + a) * P);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bst32<CP>(b.sout, c.wl[j], vo, (kPL + j) * P);
            bst32<CP>(b.sout, c.wm[j], vo, (kPM + j) * P);
        }
        const u32x2 tw = {T0, T1};
        __builtin_amdgcn_raw_buffer_store_b64(tw, b.sout, (int)(g * 8u), (int)(kPT * P), CP);
        bst32<CP>(b.sout, c.wf, vo, kPF * P);
    }
    if (loader) return;  // the stepping waves count and fold the statistics
    if (stats != nullptr) {
        const uint32_t v[OC_NSTATS] = {wave_sum(st.eps), wave_sum(st.succ), wave_sum(st.steps), wave_sum(st.coll),
                                       wave_sum(st.err)};
        unsigned long long* const part = (unsigned long long*)stats;
        unsigned long long* const tickets = part + ticket_base(stat_rows);
        uint32_t last = 0u;
        if ((threadIdx.x & 63u) == 0u) {
            unsigned long long* row = part + (int64_t)(blockIdx.x % stat_rows) * OC_NSTATS;
#pragma unroll
            for (int c = 0; c < OC_NSTATS; ++c)
                if (v[c]) atomicAdd(row + c, (unsigned long long)v[c]);
            if (totals != nullptr) {
                // Completion is counted in three levels, so that no counter takes more than
                // kTicketGroup returning atomics (one counter for all 4,096 waves of a 2^20-env
                // launch serialised them at the memory side: ~48 us on a one-step launch).  A
                // wave's adds are performed (vmcnt drained: atomics execute at the memory side,
                // MI355X_MICROARCH.md "Global float atomics") before it counts itself done in
                // LDS; the block's last wave counts the block done in its group, the group's
                // last block counts the group done, and the last group's block folds.
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (atomicAdd(&waves_done, 1u) == (uint32_t)(kBlock / 64) - 1u) {
                    const uint32_t grp = blockIdx.x / (uint32_t)kTicketGroup, ngrp = (gridDim.x + kTicketGroup - 1) / kTicketGroup;
                    const uint32_t gsize = min((uint32_t)kTicketGroup, gridDim.x - grp * (uint32_t)kTicketGroup);
                    unsigned long long* gc = tickets + (int64_t)(1 + grp) * kTicketStride;
                    if ((uint32_t)atomicAdd(gc, 1ull) == gsize - 1u) {
                        atomicExch(gc, 0ull);  // the group's counter ready for the next launch
                        last = (uint32_t)atomicAdd(tickets, 1ull) == ngrp - 1u ? 1u : 0u;
                    }
                }
            }
        }
        if (totals != nullptr && __builtin_amdgcn_readfirstlane((int)last) != 0) {
            // Last wave: fold the partial rows into totals (what oc_stats_reduce does after the
            // launch).  The rows are read with returning atomics, which are served at the memory
            // side, so no XCD's L2 can hand back a stale copy.
            // All of a lane's reads are issued before any is summed (a rolled loop waited for
            // each round's reads before issuing the next), and the 64 lanes' sums are added up
            // in LDS in two rounds of 8 instead of 6 dependent 64-bit shuffle steps per counter.
            const uint32_t lane = threadIdx.x & 63u;
            constexpr int kIt = (int)(kStatRows / 64);
            unsigned long long got[kIt][OC_NSTATS], acc[OC_NSTATS] = {0ull, 0ull, 0ull, 0ull, 0ull};
#pragma unroll
            for (int it = 0; it < kIt; ++it) {  // rows past stat_rows read row 0 again and count 0
                const uint32_t r = lane + 64u * (uint32_t)it, rr = r < stat_rows ? r : 0u;
#pragma unroll
                for (int c = 0; c < OC_NSTATS; ++c) got[it][c] = atomicAdd(part + (int64_t)rr * OC_NSTATS + c, 0ull);
            }
#pragma unroll
            for (int it = 0; it < kIt; ++it)
#pragma unroll
                for (int c = 0; c < OC_NSTATS; ++c)
                    acc[c] += lane + 64u * (uint32_t)it < stat_rows ? got[it][c] : 0ull;
#pragma unroll
            for (int c = 0; c < OC_NSTATS; ++c) fold[c][lane] = acc[c];
            __builtin_amdgcn_wave_barrier();  // LDS is in order within a wave; keep the compiler from moving reads up
            if (lane < 8u * OC_NSTATS) {
                const uint32_t c = lane >> 3, q = lane & 7u;
                unsigned long long v = 0ull;
#pragma unroll
                for (int i = 0; i < 8; ++i) v += fold[c][8u * q + i];
                fold[c][64 + q] = v;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane < (uint32_t)OC_NSTATS) {
                unsigned long long v = 0ull;
#pragma unroll
                for (int i = 0; i < 8; ++i) v += fold[lane][64 + i];
                totals[lane] = v;
            }
            if (lane == 0u) atomicExch(tickets, 0ull);  // ready for the next launch
        }
    }
}

// Planner rollout (oc_rollout): one row per lane, scalar (oc_rollout.h).  Each block stages
// the level's table blob (tile classes, graph nodes, Cutboard / Delivery lists, reachability
// distances: dynamic LDS sized for this level, oc_rollout.h blob_bytes) and the subtask
// configurations in LDS, then walks rows with a grid stride.  Rows are independent;
// byte-plane loads of 64 contiguous bytes per wave instruction.
struct RollArgs {
    ocro::RollLevel L;
    ocro::Sub subs[OC_MAX_SUBTASKS];
    int32_t nsub;
    int32_t blob_words;  // roll.lds_bytes / 4: the whole blob, or (dist_global: a wide level, a narrow
                         // one past kMaxNodes) the tables up to dist_off (distances in device memory)
    int64_t pitch, B;
};

// Stage the level's table blob and the subtask configurations in LDS.
template <int NT = kBlock>
__device__ __forceinline__ void stage_roll_tables(const RollArgs& R, const uint8_t* blob_g, uint32_t* blob_w,
                                                  ocro::Sub* subs) {
    // 16-byte loads (a quarter of the load instructions; round 6), then the last < 4 words
    const int n16 = R.blob_words >> 2;
    for (int i = threadIdx.x; i < n16; i += NT) ((uint4*)blob_w)[i] = ((const uint4*)blob_g)[i];
    for (int i = 4 * n16 + threadIdx.x; i < R.blob_words; i += NT) blob_w[i] = ((const uint32_t*)blob_g)[i];
    constexpr int kSubWords = (int)(sizeof(ocro::Sub) / 4);
    for (int i = threadIdx.x; i < R.nsub * kSubWords; i += NT)
        ((uint32_t*)subs)[i] = ((const uint32_t*)R.subs)[i];
    __syncthreads();
}

// Plane indices of the state layout (oc_get_layout): a wide level (u16 cells) has its item
// cells' high bytes in K planes after the low ones.
template <int A, int K, bool W>
struct Planes {
    static constexpr int X = 0, Y = A, H = 2 * A, L = 3 * A, LH = 3 * A + K, M = 3 * A + (W ? 2 : 1) * K;
    static constexpr int T = M + K, F = T + 2, NP = F + 1;
};

template <int A, int K, bool W = false>
__device__ __forceinline__ ocro::RowT<K, W> load_row(const uint8_t* __restrict__ sin, int64_t P, int64_t e) {
    using PL = Planes<A, K, W>;
    using Row = ocro::RowT<K, W>;
    Row r;
#pragma unroll
    for (int a = 0; a < A; ++a) {
        r.x |= (uint32_t)sin[a * P + e] << (8 * a);
        r.y |= (uint32_t)sin[(PL::Y + a) * P + e] << (8 * a);
        r.h |= (uint32_t)sin[(PL::H + a) * P + e] << (8 * a);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        uint64_t c = sin[(PL::L + j) * P + e];
        if (W) c |= (uint64_t)sin[(PL::LH + j) * P + e] << 8;
        r.loc[j / Row::LPW] |= c << (Row::kLocBits * (j % Row::LPW));
        r.mask[j >> 3] |= (uint64_t)sin[(PL::M + j) * P + e] << (8 * (j & 7));
    }
    return r;
}

// the row's agent and item planes (t and flags are the caller's).  NT: non-temporal stores
// (the rollout's outputs: 11.39-11.43 against 11.47-11.55 us per C5 launch; the bounds kernel's
// outputs stored that way were slower, 0.095 against 0.091 ms, profiles/r05/ab/ab_nt_stores.jsonl)
template <int A, int K, bool W = false, bool NT = false>
__device__ __forceinline__ void store_row(uint8_t* __restrict__ sout, int64_t P, int64_t e, const ocro::RowT<K, W>& r) {
    using PL = Planes<A, K, W>;
    auto st = [&](int64_t i, uint32_t v) {
        if constexpr (NT) __builtin_nontemporal_store((uint8_t)v, sout + i);
        else sout[i] = (uint8_t)v;
    };
#pragma unroll
    for (int a = 0; a < A; ++a) {
        st(a * P + e, (uint32_t)r.ax(a));
        st((PL::Y + a) * P + e, (uint32_t)r.ay(a));
        st((PL::H + a) * P + e, (uint32_t)r.ah(a));
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t c = (uint32_t)r.il(j);
        st((PL::L + j) * P + e, c);
        if (W) st((PL::LH + j) * P + e, c >> 8);
        st((PL::M + j) * P + e, (uint32_t)r.im(j));
    }
}

#ifndef OC_ROLL_BLOCK
#define OC_ROLL_BLOCK 256
#endif
// The agent-pair table (oc_rollout.h pair_off: the two-agent bound's per-type minima, device
// memory) in the rollout kernels: 2^18 rows 11.35-11.40 -> 10.78-10.83 us, 4,096 rows unchanged;
// in the likelihood kernels 188-192 -> 193-195 us, so off there (profiles/r06/pass_z); the bounds
// kernel always reads it (85 -> 70 us, pass_y).  Every output byte identical.
#ifndef OC_PT_LIK
#define OC_PT_LIK 0
#endif
#ifndef OC_PT_ROLL
#define OC_PT_ROLL 1
#endif
#ifndef OC_ROLL_GROUP
#define OC_ROLL_GROUP 4
#endif
// The rollout kernel's block (one row per lane).  512- and 1,024-lane blocks (fewer blocks to
// dispatch, each staging the tables with more lanes) measured slower at C5: 12.0-12.3 and
// 12.2-12.4 us against 11.6 (profiles/r05/ab/ab_merge_pairs_blocks.jsonl).  One-wave blocks for
// launches under 16 Ki rows (the planner's 4,096-row launches on 64 CUs instead of 16) were
// slower too: 6.79-6.81 against 5.98-5.99 us for 4,096 rows, 11.28-11.37 against 11.32-11.37 at
// 2^18 (profiles/r06/pass_b/ab_roll_small.jsonl, round 6): a block's table staging by one wave
// takes four times as many load rounds, and that staging is on every row's critical path.
constexpr int kRollBlock = OC_ROLL_BLOCK;
template <int A, int K, bool W, bool GD>
__global__ __launch_bounds__(kRollBlock) void oc_rollout_kernel(RollArgs R, const uint8_t* __restrict__ sin,
                                                            uint8_t* __restrict__ sout,
                                                            const uint8_t* __restrict__ act,
                                                            const uint8_t* __restrict__ alloc,
                                                            const uint8_t* __restrict__ blob_g,
                                                            uint8_t* __restrict__ out_flags,
                                                            float* __restrict__ lb) {
    extern __shared__ __attribute__((aligned(16))) uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    const int64_t P = R.pitch;
    using PL = Planes<A, K, W>;
    // A lane's row: its state, t, flags, allocation id and every agent's action (the subtask's
    // agents are known only once the configuration table is in LDS).  The first row's loads are
    // issued before the table staging, so their latency overlaps it (round 6).
    struct In {
        ocro::RowT<K, W> r;
        uint16_t t;
        uint8_t fl;
        int ai;
        uint32_t acts;  // agent a's action in byte a
    };
    auto load_in = [&](int64_t e) {
        In v;
        v.r = load_row<A, K, W>(sin, P, e);
        v.t = ((const uint16_t*)(sin + PL::T * P))[e];
        v.fl = sin[PL::F * P + e];
        v.ai = alloc != nullptr ? alloc[e] : 0;
        v.acts = 0u;
#pragma unroll
        for (int a = 0; a < A; ++a) v.acts |= (uint32_t)act[a * P + e] << (8 * a);
        return v;
    };
    int64_t e = blockIdx.x * (int64_t)kRollBlock + threadIdx.x;
    In in;
    if (e < R.B) in = load_in(e);
    stage_roll_tables<kRollBlock>(R, blob_g, blob_w, subs);
    const uint8_t* blob = (const uint8_t*)blob_w;
    for (bool first = true; e < R.B; e += (int64_t)gridDim.x * kRollBlock, first = false) {
        if (!first) in = load_in(e);
        ocro::RowT<K, W> r = in.r;
        const uint16_t t = in.t;
        const uint8_t fl_in = in.fl;
        const int ai = in.ai;
        float bound = 0.0f;
        int f = OC_ROLL_BADALLOC;  // an alloc id past num_subtasks: the row is copied unchanged
        if (ai < R.nsub) {
            const ocro::Sub& s = subs[ai];
            const int c0 = (in.acts >> (8 * s.agent[0])) & 0xFFu, c1 = s.n == 2 ? (in.acts >> (8 * s.agent[1])) & 0xFFu : ocro::kNoop;
            ocro::RowOps<A, K, W, false, GD> ops(R.L, blob, GD ? blob_g + R.L.dist_off : blob + R.L.dist_off);  // distances: LDS (narrow), device memory (wide)
            if (OC_PT_ROLL) ops.PT = R.L.pair_off != 0 ? (const uint32_t*)(blob_g + R.L.pair_off) : nullptr;
            f = ops.run(r, s, c0, c1, bound);
        }
        store_row<A, K, W, true>(sout, P, e, r);
        __builtin_nontemporal_store(t, (uint16_t*)(sout + PL::T * P) + e);
        __builtin_nontemporal_store(fl_in, sout + PL::F * P + e);
        __builtin_nontemporal_store((uint8_t)f, out_flags + e);
        __builtin_nontemporal_store(bound, lb + e);
    }
}

// Lane-group rollout rows (round 6), for launches that fit one round of blocks with G lanes per
// row: the planner's own launches (<= 4,096 rows), where the launch lasts as long as its slowest
// wave's row chain.  The G lanes of a group run one row together: every lane builds the Level-0
// view and runs legality, interact and the goal test (one chain), and the lower bound -- the
// longest phase (2.4 of the 8.8 us of a 4,096-row launch, tools/rollx.hip ablations) -- splits
// its approach walks: lane q takes A approach q * 4 / G .. (one-agent rows and the static Chop /
// Deliver side) or B square q & 1 of each Merge pair (two agents, whose per-type minima need both
// sides whole).  The group's minima meet by DPP swaps inside a quad; lane 0 stores.  4,096 rows:
// 8.91 us one row per lane, 7.96 lane pairs, 7.76 lane quads; splitting a two-agent row's
// legality by agent as well, 8.02 / 7.82 (profiles/r06/pass_n/rollx.log).  Narrow levels with LDS
// distances only (every kitchen the reference ships); the others keep one row per lane.
constexpr int kRollGroup = OC_ROLL_GROUP;
template <int G>
__device__ __forceinline__ float group_min(float v) {
    static_assert(G == 2 || G == 4, "lane groups of 2 or 4");
    int o = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    v = __int_as_float(o) < v ? __int_as_float(o) : v;
    if (G == 4) {
        o = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
        v = __int_as_float(o) < v ? __int_as_float(o) : v;
    }
    return v;
}
template <int G, int A, int K>
struct GroupRowOps : ocro::RowOps<A, K> {
    using Base = ocro::RowOps<A, K>;
    using typename Base::Row;
    using typename Base::Target;
    using Base::L;
    using Base::T;
    static constexpr int NA = 4 / G;  // A approaches per lane when the walk takes four
    int q;                            // this lane's index in its group
    __device__ GroupRowOps(const ocro::RollLevel& l, const uint8_t* blob, int lane) : Base(l, blob), q(lane) {}
    __device__ int approach(bool four, int k) const { return four ? NA * q + k : 0; }

    // Base::helper_static over this lane's A approaches
    __device__ float helper_static(const ocro::Sub& s, int u0, int u1, int Ac, int nb, int side, const uint16_t* man_t) const {
        const float per = (float)L.perimeter;
        float lower = per + 1.0f;
        if (nb == 0) return lower;
        int vAs[4];
        const bool four = ocro::wave_any(this->approaches(Ac, vAs));
        if (s.n == 1) {
#pragma unroll
            for (int k = 0; k < NA; ++k) {
                const int vA = vAs[approach(four, k)];
                const int a1 = this->dn(u0, vA), m = this->dmin(side, vA);
                const float bound = (float)(a1 + m - 1);
                lower = vA != ocro::kNoNode && a1 >= 0 && m >= 0 && bound < lower ? bound : lower;
                if (!four) break;  // wave-uniform: a Floor square's one node
            }
        } else {
            const int man = man_t[Ac];
            float mA = per;
#pragma unroll
            for (int k = 0; k < NA; ++k) {
                const int vA = vAs[approach(four, k)];
                int t;
                const float b1A = (t = this->dn(u0, vA)) < 0 ? per : (float)t;
                const float b2A = (t = this->dn(u1, vA)) < 0 ? per : (float)t;
                const float m2 = b1A < b2A ? b1A : b2A;
                mA = m2 < mA ? m2 : mA;
                if (!four) break;
            }
            const float bound = mA + (float)man - 1.0f;
            if (bound < lower) lower = bound;
        }
        return lower > 1.0f ? lower : 1.0f;
    }
    // Base::helper_n<2>(Ac, {B1, B2}): one agent, this lane's A approaches (the node-to-square
    // table when the level has one); two agents, B square q & 1
    __device__ float helper_pair(const ocro::Sub& s, int u0, int u1, int Ac, int B1, int B2) const {
        if (s.n == 1 && L.sq_off != 0) {
            float lower = (float)L.perimeter + 1.0f;
            int vA[4];
            const bool four = ocro::wave_any(this->approaches(Ac, vA));
#pragma unroll
            for (int k = 0; k < NA; ++k) {
                const int v = vA[approach(four, k)];
                const int a1 = this->dn(u0, v), b1 = this->dsq(v, B1), b2 = this->dsq(v, B2);
                const float x1 = (float)(a1 + b1 - 1), x2 = (float)(a1 + b2 - 1);
                lower = a1 >= 0 && b1 >= 0 && x1 < lower ? x1 : lower;
                lower = a1 >= 0 && b2 >= 0 && x2 < lower ? x2 : lower;
                if (!four) break;
            }
            return lower > 1.0f ? lower : 1.0f;
        }
        const int Bc[1] = {(q & 1) ? B2 : B1};
        return this->template helper_n<1>(s, u0, u1, Ac, Bc);
    }
    // Base::lower_bound with the walks split; the group's min (the clamps are monotone)
    __device__ float lower_bound(const Row& r, const ocro::Sub& s) const {
        const auto br = this->template bound_row<false>(r);
        int u0, u1;
        float pen;
        this->template bound_agents<false>(br, s, u0, u1, pen);
        float lower = (float)L.perimeter + 1.0f;
        if (s.kind == 1 || s.kind == 3) {
            const int nb = s.kind == 1 ? L.ncut : L.ndeliv;
            const int side = s.kind == 1 ? 0 : 1;
            const uint16_t* man_t = (const uint16_t*)(T + L.man_off) + (s.kind == 1 ? 0 : L.man_stride);
            this->template visit_objs<false>(br, r, s.start[0], s.kind == 3, [&](int Ac) {
                const float b = helper_static(s, u0, u1, Ac, nb, side, man_t);
                if (b < lower) lower = b;
            });
        } else if (s.kind == 2) {
            this->template visit_objs<false>(br, r, s.start[0], false, [&](int Ac) {
                this->template visit_obj_pairs<false>(br, r, s.start[1], false, [&](int B1, int B2) {
                    const float b = helper_pair(s, u0, u1, Ac, B1, B2);
                    if (b < lower) lower = b;
                });
            });
        }
        return group_min<G>(lower) + pen;
    }
    // Base::run
    __device__ int run(Row& r, const ocro::Sub& s, int c0, int c1, float& lb) {
        const Row r_in = r;
        if (this->level0(r, s)) {
            r = r_in;
            lb = 0.0f;
            return 8;  // OC_ROLL_RAISES
        }
        if (s.kind == 0) c0 = c1 = ocro::kNoop;
        c0 = c0 > ocro::kNoop ? ocro::kNoop : c0;
        c1 = c1 > ocro::kNoop ? ocro::kNoop : c1;
        const Target g0 = this->target(r, s.agent[0], c0), g1 = s.n == 2 ? this->target(r, s.agent[1], c1) : g0;
        int fl = this->action_legal(r, s, c0, c1, g0, g1) ? 1 : 0;
        this->interact(r, s.agent[0], c0, g0);
        if (s.n == 2) this->interact(r, s.agent[1], c1, g1);
        const bool asserted = s.n == 2 && this->agent_cell(r, s.agent[0]) == this->agent_cell(r, s.agent[1]);
        if (asserted) fl |= 4;
        else if (this->is_goal(r, s)) fl |= 2;
        lb = lower_bound(r, s);
        return fl;
    }
};
// One round of blocks: G * B <= the grid's lanes (oc_rollout checks), so no grid-stride loop.
template <int A, int K>
__global__ __launch_bounds__(kRollBlock) void oc_rollout_group_kernel(RollArgs R, const uint8_t* __restrict__ sin,
                                                                  uint8_t* __restrict__ sout,
                                                                  const uint8_t* __restrict__ act,
                                                                  const uint8_t* __restrict__ alloc,
                                                                  const uint8_t* __restrict__ blob_g,
                                                                  uint8_t* __restrict__ out_flags,
                                                                  float* __restrict__ lb) {
    constexpr int G = kRollGroup;
    extern __shared__ __attribute__((aligned(16))) uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    const int64_t P = R.pitch;
    using PL = Planes<A, K, false>;
    const int q = (int)(threadIdx.x & (G - 1));
    const int64_t e = (blockIdx.x * (int64_t)kRollBlock + threadIdx.x) / G;
    const bool live = e < R.B;  // whole groups: B ends on a group boundary
    ocro::RowT<K> r;
    uint16_t t = 0;
    uint8_t fl_in = 0;
    int ai = 0;
    uint32_t acts = 0;
    if (live) {  // every lane of the group loads the row (the same bytes: one transaction)
        r = load_row<A, K>(sin, P, e);
        t = ((const uint16_t*)(sin + PL::T * P))[e];
        fl_in = sin[PL::F * P + e];
        ai = alloc != nullptr ? alloc[e] : 0;
#pragma unroll
        for (int a = 0; a < A; ++a) acts |= (uint32_t)act[a * P + e] << (8 * a);
    }
    stage_roll_tables<kRollBlock>(R, blob_g, blob_w, subs);
    if (!live) return;
    float bound = 0.0f;
    int f = OC_ROLL_BADALLOC;
    if (ai < R.nsub) {
        const ocro::Sub& s = subs[ai];
        const int c0 = (acts >> (8 * s.agent[0])) & 0xFFu, c1 = s.n == 2 ? (acts >> (8 * s.agent[1])) & 0xFFu : ocro::kNoop;
        GroupRowOps<G, A, K> ops(R.L, (const uint8_t*)blob_w, q);
        if (OC_PT_ROLL) ops.PT = R.L.pair_off != 0 ? (const uint32_t*)(blob_g + R.L.pair_off) : nullptr;
        f = ops.run(r, s, c0, c1, bound);
    }
    if (q == 0) {
        store_row<A, K, false, true>(sout, P, e, r);
        __builtin_nontemporal_store(t, (uint16_t*)(sout + PL::T * P) + e);
        __builtin_nontemporal_store(fl_in, sout + PL::F * P + e);
        __builtin_nontemporal_store((uint8_t)f, out_flags + e);
        __builtin_nontemporal_store(bound, lb + e);
    }
}

// Bayesian-delegation likelihood (oc_nav_likelihood): a group of G lanes per row; candidate
// action k (k = a0 for one subtask agent, a0*5 + a1 for two: the reference's loop order,
// bayesian_delegator.py:676-689) belongs to lane k % G, slot k / G (32 / G slots per lane).  Every
// lane of a group builds the row's Level-0 view, tests its candidates' legality and evaluates
// Q(s, k) with one rollout (interact + goal + lower bound) for each legal candidate and for
// the taken action.  The group then takes Q(s, taken) from the taken action's lane, the max of
// x = beta * (Q(s, taken) - Q(s, k)) over the legal candidates (a butterfly max: order-free),
// exp(x - max) per candidate, and the softmax sum over k in ascending order (every lane adds
// the group's terms in that order, so the sum is the sequential one bit for bit).  A lane
// walking all candidates of its row kept 22 % of the lanes active per VALU instruction
// (profiles/r02/c5_grouped); spreading them over the group leaves the candidates' own path
// differences.  G = 32 (one candidate per lane) when the call's table has a two-agent
// configuration; G = 8 when every configuration has one agent (5 candidates: a 32-lane group
// would idle 27 lanes).  Measured on the C5 rows (profiles/r02/c5_order_probe.json): G = 32
// 0.35 ms configuration-major, 0.55 ms random order, against 0.44 / 1.29 ms with G = 8; a
// one-agent table 0.19 ms with G = 8, 0.41 with G = 32.  The None subtask's closed form runs
// on the group's first lane.
template <int A, int K, int G, bool W, bool GD>
__global__ __launch_bounds__(kBlock) void oc_likelihood_kernel(RollArgs R, const uint8_t* __restrict__ sin,
                                                               const uint8_t* __restrict__ taken_p,
                                                               const uint8_t* __restrict__ alloc,
                                                               const uint8_t* __restrict__ blob_g, int self_agent,
                                                               double beta, double nap, double* __restrict__ out,
                                                               uint8_t* __restrict__ out_flags) {
    extern __shared__ __attribute__((aligned(16))) uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    stage_roll_tables(R, blob_g, blob_w, subs);
    const uint8_t* blob = (const uint8_t*)blob_w;
    const int64_t P = R.pitch;
    constexpr int kLikGroup = G, kLikSlots = 32 / G;  // G x slots >= 25 candidates
    const int lane = (int)(threadIdx.x & (kLikGroup - 1));
    const int64_t ngroups = (int64_t)gridDim.x * (kBlock / kLikGroup);
    for (int64_t e = (int64_t)blockIdx.x * (kBlock / kLikGroup) + threadIdx.x / kLikGroup; e < R.B; e += ngroups) {
        const int ai = alloc != nullptr ? alloc[e] : 0;  // group-uniform from here on
        double v = 0.0;
        int f = OC_LIK_BADALLOC;
        if (ai < R.nsub) {
            const ocro::Sub& s = subs[ai];
            ocro::RowT<K, W> r = load_row<A, K, W>(sin, P, e);
            uint32_t taken = 0;
#pragma unroll
            for (int a = 0; a < A; ++a) taken |= (uint32_t)taken_p[a * P + e] << (8 * a);
            ocro::RowOps<A, K, W, true, GD> ops(R.L, blob, GD ? blob_g + R.L.dist_off : blob + R.L.dist_off);  // distances: LDS (narrow), device memory (wide)
            if (OC_PT_LIK) ops.PT = R.L.pair_off != 0 ? (const uint32_t*)(blob_g + R.L.pair_off) : nullptr;
            if (s.kind == 0) {
                f = 0;
                if (lane == 0) f = ops.likelihood(r, s, taken, self_agent, beta, nap, v);
            } else if (ops.level0(r, s)) {
                f = OC_LIK_RAISES;  // two removed agents on one square
            } else {
                const bool joint = s.n == 2;
                int t0 = (int)((taken >> (8 * s.agent[0])) & 0xFFu), t1 = ocro::kNoop;
                if (joint) t1 = (int)((taken >> (8 * s.agent[1])) & 0xFFu);
                t0 = t0 > ocro::kNoop ? ocro::kNoop : t0;
                t1 = t1 > ocro::kNoop ? ocro::kNoop : t1;
                const int ncand = joint ? 25 : 5, kt = joint ? t0 * 5 + t1 : t0;
                const int other = joint ? (s.agent[0] == self_agent ? 1 : (s.agent[1] == self_agent ? 0 : -1)) : -1;
                double q[kLikSlots], ex[kLikSlots];
                bool legal[kLikSlots];
                int bad = 0, taken_ok = 0;
                double qt = 0.0;
                // candidate k's legality and Q (one rollout when legal or taken)
                auto eval = [&](int k, double& qj, bool& lg) OC_RL {
                    const int a0 = joint ? k / 5 : k, c1 = joint ? k % 5 : ocro::kNoop;
                    lg = k < ncand && ops.action_legal(r, s, a0, c1);
                    if (other == 0 && a0 != t0) lg = false;
                    if (other == 1 && c1 != t1) lg = false;
                    qj = 0.0;
                    bool ok = true;
                    if (lg || k == kt) ok = ops.q_value(r, s, a0, c1, qj);
                    bad |= (int)(lg && !ok);
                    if (k == kt) {
                        qt = qj;
                        taken_ok = (int)(ok && lg);
                    }
                };
                if constexpr (kLikSlots == 1) {
                    eval(lane, q[0], legal[0]);
                } else {
                    // one rolled loop, one rollout call site (the row code is large); its results
                    // go to the slot registers by static selects (no scratch)
#pragma unroll 1
                    for (int j = 0; j < kLikSlots; ++j) {
                        double qj;
                        bool lg;
                        eval(lane + kLikGroup * j, qj, lg);
#pragma unroll
                        for (int i = 0; i < kLikSlots; ++i)
                            if (i == j) {
                                q[i] = qj;
                                legal[i] = lg;
                            }
                    }
                }
                // Q(s, taken) and its legality from the taken action's lane; the row raises when
                // that rollout or any legal candidate's rollout hits the co-location assert, or
                // when the taken action is not among get_actions
                const double old_q = __shfl(qt, kt % kLikGroup, kLikGroup);
                taken_ok = __shfl(taken_ok, kt % kLikGroup, kLikGroup);
#pragma unroll
                for (int off = 1; off < kLikGroup; off <<= 1) bad |= __shfl_xor(bad, off, kLikGroup);
                if (!taken_ok || bad) {
                    f = OC_LIK_RAISES;
                } else {
                    double m = -1.0e300;
#pragma unroll
                    for (int j = 0; j < kLikSlots; ++j) {
                        q[j] = legal[j] ? beta * (old_q - q[j]) : -1.0e300;  // q now holds x
                        m = q[j] > m ? q[j] : m;
                    }
#pragma unroll
                    for (int off = 1; off < kLikGroup; off <<= 1) {
                        const double o = __shfl_xor(m, off, kLikGroup);
                        m = o > m ? o : m;
                    }
                    double et = 0.0;
#pragma unroll
                    for (int j = 0; j < kLikSlots; ++j) {
                        ex[j] = legal[j] ? exp(q[j] - m) : 0.0;
                        if (lane + kLikGroup * j == kt) et = ex[j];
                    }
                    double S = 0.0;  // ascending k = 8 j + c: the reference's summation order
#pragma unroll
                    for (int j = 0; j < kLikSlots; ++j)
                        for (int c = 0; c < kLikGroup && kLikGroup * j + c < ncand; ++c) S += __shfl(ex[j], c, kLikGroup);
                    v = __shfl(et, kt % kLikGroup, kLikGroup) / S;
                    f = OC_LIK_OK;
                }
            }
        }
        if (lane == 0) {
            out[e] = f == OC_LIK_OK ? v : 0.0;
            out_flags[e] = (uint8_t)f;
        }
    }
}

// Full-state subtask bounds (oc_subtask_bounds): one env per lane, the configurations of the
// block's chunk (blockIdx.y of gridDim.y contiguous chunks of the call's table) in turn
// (configurations and tables in LDS).  Output [subtask][pitch], so each store instruction of a
// wave covers 64 consecutive envs of one configuration.  Chunking the table multiplies the
// waves of a launch: the walk is LDS-latency bound and one chunk left 4 waves per SIMD.
// LDS ordering between the lanes of one wave (its LDS operations run in order; this keeps the
// compiler from moving them and waits for the outstanding ones)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

#ifndef OC_LIK_COMPACT
#define OC_LIK_COMPACT 1
#endif
#ifndef OC_LIK_ROUND_SCALE
#define OC_LIK_ROUND_SCALE 2
#endif
// rows a wave takes per round: 16 with 32-lane groups (8 batches of 2), 32 with 8-lane groups
// (OC_LIK_ROUND_SCALE 2; half that: the same at C5 configuration-major, 2-5 % slower in random
// order and on a one-agent table, profiles/r04/lik_compact/lik_ab_rounds.jsonl; twice that: 10-20 %
// slower, lik_ab_rounds4.jsonl)
constexpr int lik_rows_per_round(int G) { return (G == 32 ? 8 : 16) * OC_LIK_ROUND_SCALE; }
// the compacted form's static LDS beyond the subtask table (16,768 B with 32-lane groups)
constexpr int kLikCompactLds = 9 * 1024 * OC_LIK_ROUND_SCALE;
// The likelihood with the wave's rollouts compacted (OC_LIK_COMPACT).  In the grouped form above
// a rollout lane idles when its candidate is illegal and not the taken one, and a 32-lane group
// idles 7 lanes always (27 on a one-agent row of a joint table).  Here a wave takes kNR rows per
// round, in kNB batches of 64 / G rows (a G-lane group per row, as above):
//   1. each group tests its row's candidates' legality and lists the ones that need a rollout
//      (legal, or the taken action) in the wave's LDS item list, (row << 5) | k, by ballot;
//      rows that need none (None subtask, a level0 raise, a bad alloc id) are written here;
//   2. the wave's lanes take the list 64 items at a time: load the item's row, level0, one
//      rollout (q_value), Q(s, k) and its raise bit into the row's LDS slots;
//   3. each group reads its row's Q values back and takes the softmax as above (the same max,
//      exp and ascending sum, so the outputs are bit-identical to the grouped form).
template <int A, int K, int G, bool W, bool GD>
__global__ __launch_bounds__(kBlock) void oc_likelihood_compact_kernel(RollArgs R, const uint8_t* __restrict__ sin,
                                                                       const uint8_t* __restrict__ taken_p,
                                                                       const uint8_t* __restrict__ alloc,
                                                                       const uint8_t* __restrict__ blob_g,
                                                                       int self_agent, double beta, double nap,
                                                                       double* __restrict__ out,
                                                                       uint8_t* __restrict__ out_flags) {
    constexpr int kCand = G == 32 ? 25 : 5;  // candidates a row can have with this table
    constexpr int kSlots = 32 / G;           // candidate k = lane + G * j, j < kSlots
    constexpr int kRPB = 64 / G;             // rows per batch (one group each)
    constexpr int kNR = lik_rows_per_round(G);  // rows per wave per round
    constexpr int kNB = kNR / kRPB;             // batches per round
    constexpr int kWaves = kBlock / 64;
    constexpr uint32_t kNotPending = 0xFFFFu;
    extern __shared__ __attribute__((aligned(16))) uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    __shared__ double lq[kWaves][kNR][kCand];     // Q(s, k)
    __shared__ uint32_t lok[kWaves][kNR];         // bit k: candidate k's rollout did not raise
    __shared__ uint32_t llg[kWaves][kNR];         // bit k: candidate k is legal
    __shared__ uint32_t lrow[kWaves][kNR];        // kt | ncand << 8, or kNotPending
    __shared__ uint16_t items[kWaves][kNR * kCand];
    stage_roll_tables(R, blob_g, blob_w, subs);
    const uint8_t* blob = (const uint8_t*)blob_w;
    const int64_t P = R.pitch;
    const int wv = (int)(threadIdx.x >> 6), wl = (int)(threadIdx.x & 63), lane = wl & (G - 1), grp = wl / G;
    const uint64_t below = (1ull << wl) - 1ull;
    const int64_t stride = (int64_t)gridDim.x * kWaves * kNR;
    for (int64_t base = ((int64_t)blockIdx.x * kWaves + wv) * kNR; base < R.B; base += stride) {
        wave_lds_sync();  // the previous round's phase 3 has read its slots
        // ---- 1: legality, the rollout list ----
        int n = 0;  // wave-uniform
        for (int b = 0; b < kNB; ++b) {
            const int rs = b * kRPB + grp;
            const int64_t e = base + rs;
            bool pending = false;
            int kt = 0, ncand = 0;
            bool need[kSlots], lgs[kSlots];
#pragma unroll
            for (int j = 0; j < kSlots; ++j) need[j] = lgs[j] = false;
            if (e < R.B) {
                const int ai = alloc != nullptr ? alloc[e] : 0;
                int f = OC_LIK_BADALLOC;
                double v = 0.0;
                if (ai < R.nsub) {
                    const ocro::Sub& s = subs[ai];
                    ocro::RowT<K, W> r = load_row<A, K, W>(sin, P, e);
                    uint32_t taken = 0;
#pragma unroll
                    for (int a = 0; a < A; ++a) taken |= (uint32_t)taken_p[a * P + e] << (8 * a);
                    ocro::RowOps<A, K, W, true, GD> ops(R.L, blob, GD ? blob_g + R.L.dist_off : blob + R.L.dist_off);
                    if (OC_PT_LIK) ops.PT = R.L.pair_off != 0 ? (const uint32_t*)(blob_g + R.L.pair_off) : nullptr;
                    if (s.kind == 0) {
                        f = 0;
                        if (lane == 0) f = ops.likelihood(r, s, taken, self_agent, beta, nap, v);
                    } else if (ops.level0(r, s)) {
                        f = OC_LIK_RAISES;  // two removed agents on one square
                    } else {
                        const bool joint = s.n == 2;
                        int t0 = (int)((taken >> (8 * s.agent[0])) & 0xFFu), t1 = ocro::kNoop;
                        if (joint) t1 = (int)((taken >> (8 * s.agent[1])) & 0xFFu);
                        t0 = t0 > ocro::kNoop ? ocro::kNoop : t0;
                        t1 = t1 > ocro::kNoop ? ocro::kNoop : t1;
                        ncand = joint ? 25 : 5;
                        kt = joint ? t0 * 5 + t1 : t0;
                        const int other =
                            joint ? (s.agent[0] == self_agent ? 1 : (s.agent[1] == self_agent ? 0 : -1)) : -1;
#pragma unroll
                        for (int j = 0; j < kSlots; ++j) {
                            const int k = lane + G * j;
                            const int a0 = joint ? k / 5 : k, c1 = joint ? k % 5 : ocro::kNoop;
                            bool lg = k < ncand && ops.action_legal(r, s, a0, c1);
                            if (other == 0 && a0 != t0) lg = false;
                            if (other == 1 && c1 != t1) lg = false;
                            lgs[j] = lg;
                            need[j] = lg || k == kt;
                        }
                        pending = true;
                    }
                }
                if (!pending && lane == 0) {
                    out[e] = f == OC_LIK_OK ? v : 0.0;
                    out_flags[e] = (uint8_t)f;
                }
            }
            uint32_t lgm = 0;
#pragma unroll
            for (int j = 0; j < kSlots; ++j) {
                const uint64_t bn = __ballot(need[j]), bl = __ballot(lgs[j]);
                if (need[j]) items[wv][n + __popcll(bn & below)] = (uint16_t)((rs << 5) | (lane + G * j));
                n += __popcll(bn);
                lgm |= (uint32_t)((bl >> (grp * G)) & (G == 32 ? 0xFFFFFFFFull : ((1ull << G) - 1ull))) << (G * j);
            }
            if (lane == 0) {
                llg[wv][rs] = lgm;
                lok[wv][rs] = 0u;
                lrow[wv][rs] = pending ? (uint32_t)kt | ((uint32_t)ncand << 8) : kNotPending;
            }
        }
        wave_lds_sync();
        // ---- 2: the rollouts, 64 at a time ----
        for (int p = 0; p < n; p += 64) {
            if (p + wl < n) {
                const uint32_t it = items[wv][p + wl];
                const int rs = (int)(it >> 5), k = (int)(it & 31u);
                const int64_t e = base + rs;
                const int ai = alloc != nullptr ? alloc[e] : 0;
                const ocro::Sub& s = subs[ai];
                ocro::RowT<K, W> r = load_row<A, K, W>(sin, P, e);
                ocro::RowOps<A, K, W, true, GD> ops(R.L, blob, GD ? blob_g + R.L.dist_off : blob + R.L.dist_off);
                if (OC_PT_LIK) ops.PT = R.L.pair_off != 0 ? (const uint32_t*)(blob_g + R.L.pair_off) : nullptr;
                ops.level0(r, s);
                const bool joint = s.n == 2;
                const int a0 = joint ? k / 5 : k, c1 = joint ? k % 5 : ocro::kNoop;
                double q = 0.0;
                const bool ok = ops.q_value(r, s, a0, c1, q);
                lq[wv][rs][k] = q;
                if (ok) atomicOr(&lok[wv][rs], 1u << k);
            }
        }
        wave_lds_sync();
        // ---- 3: each pending row's softmax (the grouped form's arithmetic) ----
        for (int b = 0; b < kNB; ++b) {
            const int rs = b * kRPB + grp;
            const int64_t e = base + rs;
            const uint32_t rw = lrow[wv][rs];
            if (e >= R.B || rw == kNotPending) continue;  // group-uniform
            const int kt = (int)(rw & 0xFFu), ncand = (int)(rw >> 8);
            const uint32_t lgm = llg[wv][rs], okm = lok[wv][rs];
            int f;
            double v = 0.0;
            if ((lgm & ~okm) != 0u || !((okm & lgm) >> kt & 1u)) {
                f = OC_LIK_RAISES;
            } else {
                const double old_q = lq[wv][rs][kt];
                double q[kSlots], ex[kSlots];
                bool legal[kSlots];
                double m = -1.0e300;
#pragma unroll
                for (int j = 0; j < kSlots; ++j) {
                    const int k = lane + G * j;
                    legal[j] = (lgm >> k) & 1u;
                    q[j] = legal[j] ? beta * (old_q - lq[wv][rs][k < kCand ? k : 0]) : -1.0e300;
                    m = q[j] > m ? q[j] : m;
                }
#pragma unroll
                for (int off = 1; off < G; off <<= 1) {
                    const double o = __shfl_xor(m, off, G);
                    m = o > m ? o : m;
                }
                double et = 0.0;
#pragma unroll
                for (int j = 0; j < kSlots; ++j) {
                    ex[j] = legal[j] ? exp(q[j] - m) : 0.0;
                    if (lane + G * j == kt) et = ex[j];
                }
                double S = 0.0;  // ascending k: the reference's summation order
#pragma unroll
                for (int j = 0; j < kSlots; ++j)
                    for (int c = 0; c < G && G * j + c < ncand; ++c) S += __shfl(ex[j], c, G);
                v = __shfl(et, kt % G, G) / S;
                f = OC_LIK_OK;
            }
            if (lane == 0) {
                out[e] = v;
                out_flags[e] = (uint8_t)f;
            }
        }
    }
}

// One lane per env, every configuration of the block's chunk.  The bound is a min over the
// env's A locations (Chop, Deliver: bound_static per location) or its (A, B) location pairs
// (Merge: helper per pair), whose count depends on where the items are: walked per lane, lanes
// with fewer locations idle while the others finish (0.58 of the lanes active per VALU
// instruction, profiles/r04/c5/pmc_c5.json).  A wave-compacted walk (the wave's (env, location)
// items by a prefix sum, one per lane, folded by LDS atomics) gave the same outputs with 0.70 of
// the lanes active but ran 0.129 ms against 0.118 at C5, where most (env, configuration) pairs
// have 0 or 1 location; it was removed in round 5 (profiles/r04/bounds_compact/).
template <int A, int K, bool W, bool GD>
__global__ __launch_bounds__(kBlock) void oc_bounds_kernel(RollArgs R, const uint8_t* __restrict__ sin,
                                                           const uint8_t* __restrict__ blob_g,
                                                           float* __restrict__ lb, uint8_t* __restrict__ doable) {
    extern __shared__ __attribute__((aligned(16))) uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    stage_roll_tables(R, blob_g, blob_w, subs);
    const uint8_t* blob = (const uint8_t*)blob_w;
    const int64_t P = R.pitch;
    const int i0 = (int)(blockIdx.y * R.nsub / gridDim.y), i1 = (int)((blockIdx.y + 1) * R.nsub / gridDim.y);
    for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < R.B; e += (int64_t)gridDim.x * kBlock) {
        const ocro::RowT<K, W> r = load_row<A, K, W>(sin, P, e);
        ocro::RowOps<A, K, W, false, GD> ops(R.L, blob, GD ? blob_g + R.L.dist_off : blob + R.L.dist_off);  // distances: LDS (narrow), device memory (wide)
        ops.PT = R.L.pair_off != 0 ? (const uint32_t*)(blob_g + R.L.pair_off) : nullptr;  // the agent-pair table (device memory)
        const auto br = ops.template bound_row<true>(r);  // the row's agent nodes, slot sets: once for its configurations
        for (int i = i0; i < i1; ++i) {
            float v;
            const bool ok = ops.full_bound(br, r, subs[i], v);
            lb[i * P + e] = v;
            doable[i * P + e] = ok ? 1 : 0;
        }
    }
}

// ---- wide levels (more than 255 cells: u16 cell ids) ----------------------------------------
// A wide level (more than 255 cells, u16 cell ids) is stepped by ocsw::step4w: the SWAR step
// with every cell-valued quantity as two byte words (its low and high bytes, the wide layout's
// two item-cell planes), four envs per lane like oc_step_n_kernel (round 6; rounds 4-5 ran the
// scalar RowOps::env_step, one env after another).  Such levels are user kitchens; the shipped
// ones are all narrow.
struct WideArgs {
    ocro::RollLevel L;   // W, H, enc; tile_off 0: the table below
    ocro::StepLevel S;
    ocsw::SwarLevel sw;  // the SWAR step's constants (step4w reads the wide fields)
    int32_t tile_words;  // the tile table's words (W * H bytes rounded up to 4)
    int64_t pitch, B;
};

// n steps of every env (oc_step: n = 1, no trajectory): the state stays in registers between
// the steps; step r's state goes to traj[r] (when given), its executed actions and collision
// mask to exec_out / coll_out at r * A * pitch / r * pitch; the final state to sout.  Four envs
// per lane, every plane read and written one dword per lane (256 B per wave instruction)
// through buffer resources (an absent output's stores are dropped by its num_records = 0, so
// every store is unconditional), nt stores, the next step's action words loaded before the
// current step runs.
template <int A, int K>
__global__ __launch_bounds__(kBlock) void oc_step_wide_kernel(WideArgs R, const uint8_t* __restrict__ tiles_g,
                                                              const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                                              const uint8_t* __restrict__ act,
                                                              uint8_t* __restrict__ traj, uint8_t* __restrict__ exec_out,
                                                              uint8_t* __restrict__ coll_out, uint64_t* __restrict__ stats,
                                                              uint32_t stat_rows, int n) {
    // tile class bytes (ocsw::tile_class: Floor 0x80, Counter 0, Cutboard 0x20, Delivery 0x40)
    // of the OC_TILE_* codes, one v_perm per word
    __shared__ uint32_t cls_w[ocro::kMaxCellsWide / 4];
    for (int i = threadIdx.x; i < R.tile_words; i += kBlock)
        cls_w[i] = __builtin_amdgcn_perm(0u, 0x40200080u, ((const uint32_t*)tiles_g)[i]);
    __syncthreads();
    const uint8_t* cls_b = (const uint8_t*)cls_w;
    auto cls_of = [&](const ocsw::Cell2& c) -> uint32_t {  // per env: the class of cell (hi << 8 | lo)
        uint32_t r = 0u;
#pragma unroll
        for (int q = 0; q < kEPL; ++q) {
            const uint32_t idx = __builtin_amdgcn_perm(c.hi >> (8 * q), c.lo >> (8 * q), 0x0C0C0400u) & 0x3FFu;
            r |= (uint32_t)cls_b[idx] << (8 * q);
        }
        return r;
    };
    using PL = Planes<A, K, true>;
    const uint32_t P = (uint32_t)R.pitch;
    const uint32_t nlanes = (uint32_t)((R.B + kEPL - 1) / kEPL);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(sin, (int64_t)PL::NP * P);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(sout ? (const void*)sout : (const void*)sin, sout ? (int64_t)PL::NP * P : 0);
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(act, (int64_t)n * A * P);
    const __amdgpu_buffer_rsrc_t rt = make_rsrc(traj ? (const void*)traj : (const void*)sin, traj ? (int64_t)n * PL::NP * P : 0);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(exec_out ? (const void*)exec_out : (const void*)sin,
                                                exec_out ? (int64_t)n * A * P : 0);
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(coll_out ? (const void*)coll_out : (const void*)sin,
                                                coll_out ? (int64_t)n * P : 0);
    StepStats st;
    typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
    for (uint32_t g = blockIdx.x * (uint32_t)kBlock + threadIdx.x; g < nlanes; g += gridDim.x * (uint32_t)kBlock) {
        const uint32_t vo = g * 4u;
        uint32_t X[A], Y[A], H[A], LO[K], HI[K], M[K], wa[A], nx[A];
#pragma unroll
        for (int a = 0; a < A; ++a) {
            X[a] = bld32(rs, vo, a * P);
            Y[a] = bld32(rs, vo, (PL::Y + a) * P);
            H[a] = bld32(rs, vo, (PL::H + a) * P);
            wa[a] = bld32(ra, vo, a * P);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            LO[j] = bld32(rs, vo, (PL::L + j) * P);
            HI[j] = bld32(rs, vo, (PL::LH + j) * P);
            M[j] = bld32(rs, vo, (PL::M + j) * P);
        }
        const auto tw0 = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(g * 8u), (int)(PL::T * P), 0);
        uint32_t T0 = tw0[0], T1 = tw0[1], F = bld32(rs, vo, PL::F * P);
        uint32_t pending = ocsw::at_done80w<K>(R.sw, LO, HI);  // the loaded state: the full path once
        const int64_t rem = R.B - (int64_t)g * kEPL;
        const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (1u << (8 * (uint32_t)rem)) - 1u);
        for (int q = 0; q < n; ++q) {
#pragma unroll
            for (int a = 0; a < A; ++a) nx[a] = q + 1 < n ? bld32(ra, vo, (uint32_t)((q + 1) * A + a) * P) : 0u;
            uint32_t EX[A], CM;
            const uint32_t f_in = F;
            const bool full = ocsw::step4w<A, K>(R.sw, X, Y, H, LO, HI, M, T0, T1, F, wa, EX, CM, cls_of, WaveAny{},
                                                 pending);
            st.coll += __popc(CM & vmask);
            if (full) {  // episode ends only on the full path
                const uint32_t ended = (F & ~f_in & vmask) & ocsw::k01;
                st.eps += __popc(ended);
                st.succ += __popc(F & (ended << 1));
                st.err += __popc(F & (ended << 2));
                const uint32_t efull = (0x80808080u - ended) ^ 0x80808080u;
                const uint32_t sa = T0 & __builtin_amdgcn_perm(0u, efull, 0x01010000u);
                const uint32_t sb2 = T1 & __builtin_amdgcn_perm(0u, efull, 0x03030202u);
                st.steps += (sa & 0xFFFFu) + (sa >> 16) + (sb2 & 0xFFFFu) + (sb2 >> 16);
            }
            const uint32_t base = (uint32_t)q * PL::NP * P;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                bst32<kCPnt>(rt, X[a], vo, base + a * P);
                bst32<kCPnt>(rt, Y[a], vo, base + (PL::Y + a) * P);
                bst32<kCPnt>(rt, H[a], vo, base + (PL::H + a) * P);
                bst32<kCPnt>(rx, EX[a], vo, (uint32_t)(q * A + a) * P);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                bst32<kCPnt>(rt, LO[j], vo, base + (PL::L + j) * P);
                bst32<kCPnt>(rt, HI[j], vo, base + (PL::LH + j) * P);
                bst32<kCPnt>(rt, M[j], vo, base + (PL::M + j) * P);
            }
            const u32x2 tv = {T0, T1};
            __builtin_amdgcn_raw_buffer_store_b64(tv, rt, (int)(g * 8u), (int)(base + PL::T * P), kCPnt);
            bst32<kCPnt>(rt, F, vo, base + PL::F * P);
            bst32<kCPnt>(rc, CM, vo, (uint32_t)q * P);
#pragma unroll
            for (int a = 0; a < A; ++a) wa[a] = nx[a];
        }
#pragma unroll
        for (int a = 0; a < A; ++a) {
            bst32<kCPnt>(ro, X[a], vo, a * P);
            bst32<kCPnt>(ro, Y[a], vo, (PL::Y + a) * P);
            bst32<kCPnt>(ro, H[a], vo, (PL::H + a) * P);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bst32<kCPnt>(ro, LO[j], vo, (PL::L + j) * P);
            bst32<kCPnt>(ro, HI[j], vo, (PL::LH + j) * P);
            bst32<kCPnt>(ro, M[j], vo, (PL::M + j) * P);
        }
        const u32x2 tv = {T0, T1};
        __builtin_amdgcn_raw_buffer_store_b64(tv, ro, (int)(g * 8u), (int)(PL::T * P), kCPnt);
        bst32<kCPnt>(ro, F, vo, PL::F * P);
    }
    if (stats != nullptr) {
        const uint32_t v[OC_NSTATS] = {wave_sum(st.eps), wave_sum(st.succ), wave_sum(st.steps), wave_sum(st.coll),
                                       wave_sum(st.err)};
        if ((threadIdx.x & 63u) == 0u) {
            unsigned long long* row = (unsigned long long*)stats + (int64_t)(blockIdx.x % stat_rows) * OC_NSTATS;
#pragma unroll
            for (int c = 0; c < OC_NSTATS; ++c)
                if (v[c]) atomicAdd(row + c, (unsigned long long)v[c]);
        }
    }
}

// reset() of a wide level: the template in every env of the pitch
template <int A, int K>
__global__ __launch_bounds__(kBlock) void oc_reset_wide_kernel(WideArgs R, uint8_t* __restrict__ s) {
    using PL = Planes<A, K, true>;
    const int64_t P = R.pitch, e = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    if (e >= P) return;
#pragma unroll
    for (int a = 0; a < A; ++a) {
        s[a * P + e] = R.S.spawn_x[a];
        s[(PL::Y + a) * P + e] = R.S.spawn_y[a];
        s[(PL::H + a) * P + e] = (uint8_t)OC_HOLD_NONE;
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        s[(PL::L + j) * P + e] = (uint8_t)R.S.item_cell[j];
        s[(PL::LH + j) * P + e] = (uint8_t)(R.S.item_cell[j] >> 8);
        s[(PL::M + j) * P + e] = R.S.item_mask[j];
    }
    ((uint16_t*)(s + PL::T * P))[e] = 0;
    s[PL::F * P + e] = 0;
}

// Image observation (oc_render, GameImage.get_image_obs: gym_cooking/misc/game/gameimage.py:31-51,
// Game.on_render / draw_*: game.py:56-186).  Two blocks per (env, cell row), each taking half
// of the row's pixel groups in whole waves.  In each block the first W lanes
// build each cell's ordered draw list in LDS (items not held in slot order or the caller's
// draw rank, then every agent
// in order followed by its held item).  The block then writes the row's tile*W*tile*3 output
// bytes in iterations of 16 pixels per lane (48 output bytes), consecutive lanes on consecutive
// pixels, so a wave's 64 lanes cover 1,024 pixels that span every cell of one to three image
// rows.  A pixel starts from the static level image and blends every sprite of its cell's list
// that covers it; everything is tile-local (every sprite lies inside its cell).  Only the lanes
// over a cell with sprites have blending to do, so the wave does it together: those lanes put
// their 16 pixels in the wave's LDS slice and list themselves, and the wave then blends the
// listed pixels one per lane (16 c / 64 passes for c listed lanes) instead of the listed lanes
// looping over 16 pixels each while the others idle.
struct RenderArgs {
    int32_t W, H, tile;
    int32_t size[OC_RENDER_SIZES], offset[OC_RENDER_SIZES], food_base[OC_RENDER_SIZES];
    int32_t plate_off[2], agent_off[OC_MAX_AGENTS];
    uint32_t chan_map;
    int32_t parts;  // blocks per (env, cell row), each a contiguous run of whole waves of groups
    int32_t counts; // item masks in OC_ENC_COUNTS: translated to the presence masks food_sprite reads
    int64_t pitch;
    uint8_t food_sprite[128];
};
// A render block lists the draws of its cell row (one lane per column, so a row of up to 255
// columns: every width a level may have) in one compact list: a cell row holds every object at
// most once, so it draws at most kRenderMaxDraw sprites (a plate and a food per item, an agent
// and its held item's two), whatever its width.  Round 4's per-column lists (kRenderMaxDraw
// entries for each of 32 or 64 columns) capped the width at 32 (narrow) / 64 (wide) columns.
constexpr int kRenderMaxW = 255, kRenderMaxDraw = 2 * OC_MAX_ITEMS + 3 * OC_MAX_AGENTS;
constexpr int kRenderPx = 16;  // pixels per lane and iteration: 48 output bytes, three 16-byte stores

// SDL 1.2 per-pixel alpha blit of an RGBA source pixel onto an RGB destination pixel
// (BlitNtoNPixelAlpha / ALPHA_BLEND: d = (((s - d) * a + 255) >> 8) + d per channel, a = 0
// skipped).  ((s - d) a + 255 >> 8) + d = (s a + d (256 - a) + 255) >> 8 exactly, and that
// numerator is at most 65,535, so R and B share one 24-bit multiply-add pair in 16-bit fields
// without carries; a = 0 gives (256 d + 255) >> 8 = d, the skipped blit, with no branch.
__device__ __forceinline__ uint32_t sdl_blend(uint32_t d, uint32_t s) {
    const uint32_t a = s >> 24, na = 256u - a;
    const uint32_t rb = __umul24(d & 0xFF00FFu, na) + __umul24(s & 0xFF00FFu, a) + 0xFF00FFu;
    const uint32_t g = __umul24((d >> 8) & 0xFFu, na) + __umul24((s >> 8) & 0xFFu, a) + 0xFFu;
    return ((rb >> 8) & 0xFF00FFu) | (g & 0xFF00u);
}

// floor(n / d) for 0 <= n < 2^22 and 0 < d <= 2^11, from a float reciprocal and one correction
__device__ __forceinline__ int div_small(int n, int d, float rcp) {
    int q = (int)((float)n * rcp);
    const int rem = n - q * d;
    q += rem >= d ? 1 : 0;
    q -= rem < 0 ? 1 : 0;
    return q;
}

template <int A, int K, bool WIDE>
__global__ __launch_bounds__(kBlock) void oc_render_kernel(RenderArgs R, const uint8_t* __restrict__ state,
                                                           const uint8_t* __restrict__ rank,
                                                           const uint32_t* __restrict__ atlas,
                                                           const uint32_t* __restrict__ bg,
                                                           uint8_t* __restrict__ out) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    __shared__ uint32_t dl_off[kRenderMaxDraw];
    __shared__ uint32_t dl_geo[kRenderMaxDraw];    // size | offset << 16
    __shared__ uint16_t col_start[kBlock + 1];     // column c's draws: [col_start[c], col_start[c + 1])
    __shared__ uint32_t wave_tot[kBlock / 64];
    __shared__ u32x4 pix4[kBlock / 64][64 * kRenderPx / 4];
    __shared__ uint32_t work[kBlock / 64][64];  // listed lane | row << 6 | cell column << 16 | (x in cell) / 16 << 24
    const uint32_t part = blockIdx.x % (uint32_t)R.parts, strip = blockIdx.x / (uint32_t)R.parts;
    const int64_t e = strip / (uint32_t)R.H;
    const int ty = (int)(strip % (uint32_t)R.H);
    const int W = R.W, tile = R.tile;
    // planes: a wide level's item cells are u16, low bytes then high bytes, before the masks
    constexpr int kPX = 0, kPY = A, kPH = 2 * A, kPL = 3 * A, kPLH = 3 * A + K, kPM = 3 * A + (WIDE ? 2 : 1) * K;
    // The cell row's draw list: every column lane counts its draws, a block prefix sum places
    // them, and the lanes write them in the same order (draw order within a column).
    const int tx = (int)threadIdx.x, cell = ty * W + tx;
    const uint8_t* s = state + e;
    const int64_t P = R.pitch;
    auto column = [&](bool write, int n) -> int {  // this column's draws from slot n on; returns the end
        uint32_t held = 0u;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const uint32_t h = s[(kPH + a) * P];
            if (h < (uint32_t)K) held |= 1u << h;
        }
        auto push = [&](int32_t off, int cls) {
            if (write) {
                dl_off[n] = (uint32_t)off;
                dl_geo[n] = (uint32_t)R.size[cls] | ((uint32_t)R.offset[cls] << 16);
            }
            ++n;
        };
        // an item: a plate first, its contents at the container class; else the food itself
        auto push_item = [&](uint32_t m, int cls_plain, int cls_in_plate, int plate) {
            if (R.counts) {  // counts -> presence; two of one food have no sprite (the reference's
                             // draw opens "<full_name>.png", which does not exist: it raises)
                const uint32_t c = m & 0x3Fu, pres = (c & 1u) | ((c >> 1) & 2u) | ((c >> 2) & 4u);
                const uint32_t pl = (m & OC_MC_PLATE) ? OC_M_PLATE : 0u;
                m = (c & 0x2Au) ? pl : pl | pres | ((m & OC_MC_FRESH) ? 0u : pres << OC_M_CHOPPED_SHIFT);
            }
            const uint32_t f = m & ~OC_M_PLATE;
            if (m & OC_M_PLATE) push(R.plate_off[plate], cls_plain);
            const int cls = (m & OC_M_PLATE) ? cls_in_plate : cls_plain;
            if (f != 0u && R.food_sprite[f] != 0xFFu)
                push(R.food_base[cls] + (int32_t)R.food_sprite[f] * R.size[cls] * R.size[cls], cls);
        };
        // Game.on_render: objects not held (draw_object, game.py:138-160), in world.objects order
        // when the caller gives ranks (render.DrawOrder), else in slot order ...
        uint32_t here = 0u;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int c = WIDE ? (int)s[(kPL + j) * P] | (int)s[(kPLH + j) * P] << 8 : (int)s[(kPL + j) * P];
            if (c == cell) here |= 1u << j;  // a dead slot (0xFF / 0xFFFF) is no cell
        }
        here &= ~held;
        while (here != 0u) {
            int j = __builtin_ctz(here);
            if (rank != nullptr && (here & (here - 1u)) != 0u) {  // several objects on this square
                uint32_t best = 0xFFFFFFFFu;
                for (uint32_t m = here; m != 0u; m &= m - 1u) {
                    const int k = __builtin_ctz(m);
                    const uint32_t key = ((uint32_t)rank[(int64_t)k * P + e] << 5) | (uint32_t)k;
                    if (key < best) best = key;
                }
                j = (int)(best & 31u);
            }
            here &= ~(1u << j);
            push_item(s[(kPM + j) * P], 0, 1, 0);
        }
        // ... then the agents in order, each with its held object (draw_agent / draw_agent_object, :98-136)
#pragma unroll
        for (int a = 0; a < A; ++a) {
            if ((int)s[(kPY + a) * P] * W + (int)s[(kPX + a) * P] != cell) continue;
            push(R.agent_off[a], 0);
            const uint32_t h = s[(kPH + a) * P];
            if (h < (uint32_t)K) push_item(s[(kPM + h) * P], 2, 3, 1);
        }
        return n;
    };
    const int cnt = tx < W ? column(false, 0) : 0;
    int incl = cnt;  // inclusive scan over the wave, then over the block's waves
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if ((tx & 63) >= off) incl += o;
    }
    if ((tx & 63) == 63) wave_tot[tx >> 6] = (uint32_t)incl;
    __syncthreads();
    int before = 0;
    for (int w = 0; w < (tx >> 6); ++w) before += (int)wave_tot[w];
    const int start = before + incl - cnt;
    col_start[tx] = (uint16_t)start;
    if (tx == kBlock - 1) col_start[kBlock] = (uint16_t)(start + cnt);
    if (tx < W) column(true, start);
    __syncthreads();
    const int row_px = W * tile, G = row_px / kRenderPx;  // 16-pixel groups per image row
    // this block's share of the strip's 16-pixel groups: whole waves of them
    const int per_part = (tile * G + 64 * R.parts - 1) / (64 * R.parts) * 64;
    const int i_begin = (int)part * per_part, items = min(tile * G, i_begin + per_part);
    const float rcpG = 1.0f / (float)G, rcpT = 1.0f / (float)tile;
    const int64_t img_bytes = (int64_t)R.H * tile * row_px * 3;
    uint8_t* img = out + e * img_bytes;
    // chan_map -> v_perm selector: output byte c <- pixel byte (chan_map >> 8c), 0x0C = zero
    uint32_t psel = 0x0C000000u;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t ch = (R.chan_map >> (8 * c)) & 0xFFu;
        psel |= (ch >= 3u ? 0x0Cu : ch) << (8 * c);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* const pix = (uint32_t*)pix4[wave];
    uint8_t* const blk_out = img + (int64_t)ty * tile * row_px * 3;
    for (int base = i_begin; base < items; base += kBlock) {
        const int w0 = base + wave * 64;  // the wave's first group
        const int i = w0 + lane;
        uint32_t p[kRenderPx];
        bool need = false;
        int r = 0, tx = 0, lx0 = 0;
        if (i < items) {
            r = div_small(i, G, rcpG);
            const int py = ty * tile + r, px0 = kRenderPx * (i - r * G);
            tx = div_small(px0, tile, rcpT);  // a group never straddles two cells
            lx0 = px0 - tx * tile;
            const u32x4* bsrc = (const u32x4*)(bg + (int64_t)py * row_px + px0);
#pragma unroll
            for (int q = 0; q < kRenderPx / 4; ++q) {
                const u32x4 v = bsrc[q];
                p[4 * q] = v.x;
                p[4 * q + 1] = v.y;
                p[4 * q + 2] = v.z;
                p[4 * q + 3] = v.w;
            }
            const int d1 = col_start[tx + 1];
            for (int d = col_start[tx]; d < d1; ++d) {
                const uint32_t geo = dl_geo[d];
                const int sz = (int)(geo & 0xFFFFu), o = (int)(geo >> 16);
                need |= (unsigned)(r - o) < (unsigned)sz && lx0 + kRenderPx > o && lx0 < o + sz;
            }
        }
        const uint64_t mask = __ballot(need);
        if (mask != 0ull) {
            if (need) {
#pragma unroll
                for (int q = 0; q < kRenderPx / 4; ++q)
                    pix4[wave][4 * lane + q] = u32x4{p[4 * q], p[4 * q + 1], p[4 * q + 2], p[4 * q + 3]};
                const uint32_t slot =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
                work[wave][slot] = (uint32_t)lane | ((uint32_t)r << 6) | ((uint32_t)tx << 16) | ((uint32_t)(lx0 >> 4) << 24);
            }
            __builtin_amdgcn_wave_barrier();  // LDS is in order within a wave; keep the compiler from moving reads up
            const int npx = kRenderPx * __popcll(mask);
            for (int t = lane; t < npx; t += 64) {
                const uint32_t ent = work[wave][t >> 4];
                const int k = t & (kRenderPx - 1), gl = (int)(ent & 63u);
                const int rr = (int)((ent >> 6) & 0x3FFu), ctx = (int)((ent >> 16) & 0xFFu), lx = (int)(ent >> 24) * 16 + k;
                uint32_t dpx = pix[kRenderPx * gl + k];
                const int d1 = col_start[ctx + 1];
                for (int d = col_start[ctx]; d < d1; ++d) {
                    const uint32_t geo = dl_geo[d];
                    const int sz = (int)(geo & 0xFFFFu), o = (int)(geo >> 16);
                    const int dy = rr - o, dx = lx - o;
                    if ((unsigned)dy < (unsigned)sz && (unsigned)dx < (unsigned)sz)
                        dpx = sdl_blend(dpx, atlas[dl_off[d] + dy * sz + dx]);
                }
                pix[kRenderPx * gl + k] = dpx;
            }
            __builtin_amdgcn_wave_barrier();
            if (need) {
#pragma unroll
                for (int q = 0; q < kRenderPx / 4; ++q) {
                    const u32x4 v = pix4[wave][4 * lane + q];
                    p[4 * q] = v.x;
                    p[4 * q + 1] = v.y;
                    p[4 * q + 2] = v.z;
                    p[4 * q + 3] = v.w;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        // The block's output rows are contiguous and group i lands at byte 48 i, so a wave's 64
        // groups are 3 KB contiguous.  Each lane packs its 48 bytes into the wave's LDS slice, and
        // the wave then stores the slice as three fully contiguous 1 KB instructions (16 B per
        // lane) instead of three 16 B-per-lane instructions at a 48 B stride.
        if (i < items) {
            uint32_t w[12];  // 16 pixels -> 48 bytes: per 4 pixels three dwords of packed 3-byte pixels
#pragma unroll
            for (int q = 0; q < kRenderPx / 4; ++q) {
                const uint32_t a0 = __builtin_amdgcn_perm(0u, p[4 * q], psel),
                               a1 = __builtin_amdgcn_perm(0u, p[4 * q + 1], psel),
                               a2 = __builtin_amdgcn_perm(0u, p[4 * q + 2], psel),
                               a3 = __builtin_amdgcn_perm(0u, p[4 * q + 3], psel);
                w[3 * q] = a0 | (a1 << 24);
                w[3 * q + 1] = (a1 >> 8) | (a2 << 16);
                w[3 * q + 2] = (a2 >> 16) | (a3 << 8);
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) pix4[wave][3 * lane + q] = u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        }
        __builtin_amdgcn_wave_barrier();
        const int nbytes = 48 * (items - w0 < 64 ? (items - w0 > 0 ? items - w0 : 0) : 64);
        u32x4* dst = (u32x4*)(blk_out + (int64_t)w0 * 48);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int off = q * 64 + lane;  // 16-byte units
            if (off * 16 < nbytes) __builtin_nontemporal_store(pix4[wave][off], dst + off);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// reset(): broadcast the level template (overcooked_environment.py:201-250).
template <int A, int K>
__global__ __launch_bounds__(kBlock) void oc_reset_kernel(LevelArgs L, uint8_t* __restrict__ s) {
    const int64_t P = L.pitch;
    const int64_t e0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kEPL;
    auto rep = [](uint32_t b) { return (b & 0xFFu) * 0x01010101u; };
    auto st32 = [&](int plane, uint32_t v) { *reinterpret_cast<uint32_t*>(s + plane * P + e0) = v; };
#pragma unroll
    for (int a = 0; a < A; ++a) {
        st32(a, rep(byte_of(L.tmpl_x, a)));
        st32(A + a, rep(byte_of(L.tmpl_y, a)));
        st32(2 * A + a, rep(OC_HOLD_NONE));
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        st32(3 * A + j, rep(byte_of4(L.tmpl_cell, j)));
        st32(3 * A + K + j, rep(byte_of4(L.tmpl_mask, j)));
    }
    *reinterpret_cast<uint2*>(s + (3 * A + 2 * K) * P + 2 * e0) = make_uint2(0u, 0u);
    st32(3 * A + 2 * K + 2, 0u);
}

// Order-sensitive 64-bit checksum of the state of envs [0, B):
//   sum_e (2e + 1) * sum_p (byte_p(e) + 1) * M_p,   M_p = 0x9E3779B97F4A7C15 * (2p + 1)  (mod 2^64)
// over the byte planes p (the u16 t plane as its low / high byte planes).  It reads the state
// exactly like oc_step does (one dword per plane per lane), so it doubles as the known-byte
// read pass that calibrates the FETCH_SIZE counter for this access pattern.
template <int NP>
__global__ __launch_bounds__(kBlock) void oc_checksum_kernel(const uint8_t* __restrict__ s, int64_t pitch,
                                                             int64_t B,
                                                             unsigned long long* __restrict__ out) {
    constexpr int plane_t = NP - 3;  // t precedes the flags plane (oc_layout)
    const uint32_t g = blockIdx.x * (uint32_t)kBlock + threadIdx.x;
    const int64_t e0 = (int64_t)g * kEPL;
    uint64_t h[kEPL] = {};
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const uint64_t Mp = 0x9E3779B97F4A7C15ull * (uint64_t)(2 * p + 1);
        if (p == plane_t) {
            const uint2 w = reinterpret_cast<const uint2*>(s + p * pitch)[g];
            const uint64_t Mq = 0x9E3779B97F4A7C15ull * (uint64_t)(2 * p + 3);
#pragma unroll
            for (int q = 0; q < kEPL; ++q) {
                const uint32_t v = ((q < 2 ? w.x : w.y) >> (16 * (q & 1))) & 0xFFFFu;
                h[q] += (uint64_t)((v & 0xFFu) + 1u) * Mp + (uint64_t)((v >> 8) + 1u) * Mq;
            }
        } else if (p != plane_t + 1) {
            const uint32_t w = reinterpret_cast<const uint32_t*>(s + p * pitch)[g];
#pragma unroll
            for (int q = 0; q < kEPL; ++q) h[q] += (uint64_t)(((w >> (8 * q)) & 0xFFu) + 1u) * Mp;
        }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int q = 0; q < kEPL; ++q)
        acc += (e0 + q < B) ? h[q] * (uint64_t)(2 * (e0 + q) + 1) : 0ull;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void oc_gen_actions_kernel(uint8_t* __restrict__ act, int A, int64_t B,
                                                                int64_t pitch, int64_t env_offset,
                                                                uint64_t step, uint64_t seed) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= pitch) return;
    const uint64_t base = seed ^ ((uint64_t)(env_offset + e) * 0x9E3779B97F4A7C15ull) ^
                          (step * 0xC2B2AE3D27D4EB4Full);
    for (int a = 0; a < A; ++a)
        act[a * pitch + e] = e < B ? (uint8_t)(splitmix64(base ^ (uint64_t)a) % 5u) : (uint8_t)OC_ACT_NOOP;
}

__global__ __launch_bounds__(kBlock) void oc_stats_reduce_kernel(const uint64_t* __restrict__ part,
                                                                 int64_t nrows, uint64_t* __restrict__ out) {
    __shared__ uint64_t red[kBlock];
    for (int c = 0; c < OC_NSTATS; ++c) {
        uint64_t s = 0;
        for (int64_t r = threadIdx.x; r < nrows; r += kBlock) s += part[r * OC_NSTATS + c];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int w = kBlock / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[c] = red[0];
        __syncthreads();
    }
}

thread_local std::string g_last_error;
thread_local uint64_t g_err_gen = 0;  // failures on this thread so far (ErrScope compares)

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    ++g_err_gen;
    return code;
}

int hip_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(OC_EHIP, "%s: %s", what, hipGetErrorString(e));
    return OC_OK;
}

// Statistics rows: blocks add into row blockIdx % rows (no-return 64-bit atomics); 256 rows
// keep the adds to one address to a few dozen per launch and let one wave fold them.


int64_t pitch_for(int64_t B) {
    int64_t p = (B + OC_PITCH_ALIGN - 1) / OC_PITCH_ALIGN * OC_PITCH_ALIGN;
    return p < OC_PITCH_ALIGN ? OC_PITCH_ALIGN : p;
}

}  // namespace

struct oc_handle {
    oc_level_desc level;
    int32_t A, K, max_T, device;
    int32_t cus;                // compute units of the device (persistent grids: <= 5 blocks per CU)
    LevelArgs args;
    ocro::RollLevel roll;       // planner rollout tables (nnodes < 0: graph too large)
    uint8_t* roll_blob = nullptr;  // device: the level's rollout table blob (oc_rollout.h)
    int32_t roll_blob_bytes = 0;
    std::vector<uint8_t> roll_blob_host;  // the same blob on the host
    // wide levels (more than 255 cells): the scalar step's tables
    bool wide = false;
    ocro::StepLevel step;
    ocro::RollLevel step_lv;         // W, H, enc; tile_off 0 (the tile table alone)
    uint8_t* wide_tiles = nullptr;   // device: tile class per cell (W * H rounded up to 4 bytes)
    uint8_t wide_tiles_host[ocro::kMaxCellsWide];
    int32_t lik_form = OC_LIK_FORM_AUTO;  // oc_set_likelihood_form
    mutable std::string last_error;       // oc_get_last_error: the last failed call on this handle
};

// An entry point's failure is also recorded on its handle (oc_get_last_error): the scope sees
// whether fail() ran on this thread while the call was in progress.
struct ErrScope {
    const oc_handle* h;
    uint64_t gen;
    explicit ErrScope(const oc_handle* hh) : h(hh), gen(g_err_gen) {}
    ~ErrScope() {
        if (h != nullptr && g_err_gen != gen) h->last_error = g_last_error;
    }
};

// Device entry points refuse a host-only handle (oc_create with OC_DEVICE_HOST).
#define OC_NEED_DEVICE(h_) \
    if ((h_)->device < 0) return fail(OC_EINVAL, "host-only handle (OC_DEVICE_HOST): this entry point needs a device")

// Statistics rows, shared by the blocks of every kernel modulo the row count; oc_step_n's
// completion tickets follow them (ticket_base; zero between launches).
int64_t stats_rows(const oc_handle*, int64_t B) {
    const int64_t need = pitch_for(B) / kEnvsPerBlock;
    return need < kStatRows ? need : kStatRows;
}

// oc_cpu_step's worker: the host pass of the same SWAR step (oc_swar.h), words [g0, g1) of
// the batch (4 envs each, as one lane of oc_step_kernel), per-word rare-event split.
template <int A, int K, int MODE>
static void cpu_step_words(const oc_handle* h, const uint8_t* sin, uint8_t* sout, const uint8_t* act,
                           uint8_t* exo, uint8_t* coll, int64_t B, int64_t P, int64_t g0, int64_t g1,
                           uint64_t* st) {
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    const LevelArgs& L = h->args;
    const uint8_t* tbl = (const uint8_t*)L.cls4;
    auto cls_of = [tbl](uint32_t c) -> uint32_t {
        return (uint32_t)tbl[c & 0xFFu] | ((uint32_t)tbl[(c >> 8) & 0xFFu] << 8) |
               ((uint32_t)tbl[(c >> 16) & 0xFFu] << 16) | ((uint32_t)tbl[c >> 24] << 24);
    };
    auto rd = [P](const uint8_t* base, int plane, int64_t g) {
        uint32_t v;
        memcpy(&v, base + plane * P + 4 * g, 4);
        return v;
    };
    auto wr = [P](uint8_t* base, int plane, int64_t g, uint32_t v) { memcpy(base + plane * P + 4 * g, &v, 4); };
    uint64_t eps = 0, succ = 0, steps = 0, ncoll = 0, err = 0;
    for (int64_t g = g0; g < g1; ++g) {
        uint32_t X[A], Y[A], Hh[A], Lc[K], M[K], AC[A], EX[A], T0, T1, F, CM;
        for (int a = 0; a < A; ++a) {
            X[a] = rd(sin, a, g);
            Y[a] = rd(sin, kPY + a, g);
            Hh[a] = rd(sin, kPH + a, g);
            AC[a] = rd(act, a, g);
        }
        for (int j = 0; j < K; ++j) {
            Lc[j] = rd(sin, kPL + j, g);
            M[j] = rd(sin, kPM + j, g);
        }
        memcpy(&T0, sin + kPT * P + 8 * g, 4);
        memcpy(&T1, sin + kPT * P + 8 * g + 4, 4);
        F = rd(sin, kPF, g);
        const uint32_t f_in = F;
        uint32_t pending = ocsw::at_done80<K, MODE>(L.sw, Lc);
        const bool full = ocsw::step4<A, K, MODE>(L.sw, X, Y, Hh, Lc, M, T0, T1, F, AC, EX, CM, cls_of,
                                                  [](uint32_t v) { return v != 0u; }, pending);
        const int64_t rem = B - g * kEPL;
        const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (1u << (8 * (uint32_t)rem)) - 1u;
        ncoll += (uint64_t)__builtin_popcount(CM & vmask);
        if (full) {
            const uint32_t ended = (F & ~f_in & vmask) & ocsw::k01;
            for (int q = 0; q < kEPL; ++q) {
                if (!((ended >> (8 * q)) & 1u)) continue;
                ++eps;
                succ += (F >> (8 * q + 1)) & 1u;
                err += (F >> (8 * q + 2)) & 1u;
                steps += ((q < 2 ? T0 : T1) >> (16 * (q & 1))) & 0xFFFFu;
            }
        }
        for (int a = 0; a < A; ++a) {
            wr(sout, a, g, X[a]);
            wr(sout, kPY + a, g, Y[a]);
            wr(sout, kPH + a, g, Hh[a]);
            if (exo != nullptr) wr(exo, a, g, EX[a]);
        }
        for (int j = 0; j < K; ++j) {
            wr(sout, kPL + j, g, Lc[j]);
            wr(sout, kPM + j, g, M[j]);
        }
        memcpy(sout + kPT * P + 8 * g, &T0, 4);
        memcpy(sout + kPT * P + 8 * g + 4, &T1, 4);
        wr(sout, kPF, g, F);
        if (coll != nullptr) wr(coll, 0, g, CM);
    }
    st[OC_STAT_EPISODES] = eps;
    st[OC_STAT_SUCCESSES] = succ;
    st[OC_STAT_STEPS] = steps;
    st[OC_STAT_COLLISIONS] = ncoll;
    st[OC_STAT_ERRORS] = err;
}

// oc_cpu_step on a wide level: words [g0, g1) (4 envs each) through the host pass of the
// wide SWAR step (ocsw::step4w), per-word rare-event split, as oc_step_wide_kernel
template <int A, int K>
static void cpu_step_wide(const oc_handle* h, const uint8_t* sin, uint8_t* sout, const uint8_t* act, uint8_t* exo,
                          uint8_t* coll, int64_t B, int64_t P, int64_t g0, int64_t g1, uint64_t* st) {
    using PL = Planes<A, K, true>;
    const ocsw::SwarLevel& SL = h->args.sw;
    uint8_t cls[ocro::kMaxCellsWide];
    for (int c = 0; c < ocro::kMaxCellsWide; ++c) cls[c] = ocsw::tile_class(h->wide_tiles_host[c]);
    auto cls_of = [&cls](const ocsw::Cell2& c) -> uint32_t {
        uint32_t r = 0u;
        for (int q = 0; q < kEPL; ++q) {
            const uint32_t idx = ((((c.hi >> (8 * q)) & 0xFFu) << 8) | ((c.lo >> (8 * q)) & 0xFFu)) & 0x3FFu;
            r |= (uint32_t)cls[idx] << (8 * q);
        }
        return r;
    };
    auto rd = [P](const uint8_t* base, int plane, int64_t g) {
        uint32_t v;
        memcpy(&v, base + plane * P + 4 * g, 4);
        return v;
    };
    auto wr = [P](uint8_t* base, int plane, int64_t g, uint32_t v) { memcpy(base + plane * P + 4 * g, &v, 4); };
    uint64_t eps = 0, succ = 0, steps = 0, ncoll = 0, err = 0;
    for (int64_t g = g0; g < g1; ++g) {
        uint32_t X[A], Y[A], Hh[A], LL[K], LH[K], M[K], AC[A], EX[A], T0, T1, F, CM;
        for (int a = 0; a < A; ++a) {
            X[a] = rd(sin, PL::X + a, g);
            Y[a] = rd(sin, PL::Y + a, g);
            Hh[a] = rd(sin, PL::H + a, g);
            AC[a] = rd(act, a, g);
        }
        for (int j = 0; j < K; ++j) {
            LL[j] = rd(sin, PL::L + j, g);
            LH[j] = rd(sin, PL::LH + j, g);
            M[j] = rd(sin, PL::M + j, g);
        }
        memcpy(&T0, sin + PL::T * P + 8 * g, 4);
        memcpy(&T1, sin + PL::T * P + 8 * g + 4, 4);
        F = rd(sin, PL::F, g);
        const uint32_t f_in = F;
        uint32_t pending = ocsw::at_done80w<K>(SL, LL, LH);
        const bool full = ocsw::step4w<A, K>(SL, X, Y, Hh, LL, LH, M, T0, T1, F, AC, EX, CM, cls_of,
                                             [](uint32_t v) { return v != 0u; }, pending);
        const int64_t rem = B - g * kEPL;
        const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (1u << (8 * (uint32_t)rem)) - 1u;
        ncoll += (uint64_t)__builtin_popcount(CM & vmask);
        if (full) {
            const uint32_t ended = (F & ~f_in & vmask) & ocsw::k01;
            for (int q = 0; q < kEPL; ++q) {
                if (!((ended >> (8 * q)) & 1u)) continue;
                ++eps;
                succ += (F >> (8 * q + 1)) & 1u;
                err += (F >> (8 * q + 2)) & 1u;
                steps += ((q < 2 ? T0 : T1) >> (16 * (q & 1))) & 0xFFFFu;
            }
        }
        // the batch's last word: only its columns below B are written (a host caller's buffer
        // may be exactly B bytes per plane past the pitch's start)
        const int ncol = rem >= kEPL ? kEPL : (int)rem;
        auto put = [&](uint8_t* base, int plane, uint32_t v) {
            if (ncol == kEPL) wr(base, plane, g, v);
            else memcpy(base + plane * P + 4 * g, &v, (size_t)ncol);
        };
        for (int a = 0; a < A; ++a) {
            put(sout, PL::X + a, X[a]);
            put(sout, PL::Y + a, Y[a]);
            put(sout, PL::H + a, Hh[a]);
            if (exo != nullptr) put(exo, a, EX[a]);
        }
        for (int j = 0; j < K; ++j) {
            put(sout, PL::L + j, LL[j]);
            put(sout, PL::LH + j, LH[j]);
            put(sout, PL::M + j, M[j]);
        }
        uint8_t tb[8];
        memcpy(tb, &T0, 4);
        memcpy(tb + 4, &T1, 4);
        memcpy(sout + PL::T * P + 8 * g, tb, (size_t)(2 * ncol));
        put(sout, PL::F, F);
        if (coll != nullptr) put(coll, 0, CM);
    }
    st[OC_STAT_EPISODES] = eps;
    st[OC_STAT_SUCCESSES] = succ;
    st[OC_STAT_STEPS] = steps;
    st[OC_STAT_COLLISIONS] = ncoll;
    st[OC_STAT_ERRORS] = err;
}

extern "C" {

int oc_abi_version(void) { return OC_ABI_VERSION; }

const char* oc_last_error(void) { return g_last_error.c_str(); }

int oc_get_last_error(const oc_handle* h, char* buf, int64_t size) {
    if (h == nullptr) return fail(OC_EINVAL, "bad argument");
    const int64_t n = (int64_t)h->last_error.size();
    if (buf != nullptr && size > 0) {
        const int64_t c = n < size - 1 ? n : size - 1;
        memcpy(buf, h->last_error.data(), (size_t)c);
        buf[c] = '\0';
    }
    return (int)n;
}

int oc_set_likelihood_form(oc_handle* h, int32_t form) {
    if (h == nullptr) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    if (form != OC_LIK_FORM_AUTO && form != OC_LIK_FORM_GROUPED) return fail(OC_EINVAL, "likelihood form %d", form);
    h->lik_form = form;
    return OC_OK;
}

int oc_create(const oc_level_desc* lv, int32_t num_agents, int32_t max_T, int32_t device, oc_handle** out) {
    if (lv == nullptr || out == nullptr) return fail(OC_EINVAL, "null argument");
    const int W = lv->width, H = lv->height;
    if (W < 3 || H < 3 || W > 255 || H > 255 || W * H > OC_MAX_CELLS)
        return fail(OC_ELEVEL, "grid %dx%d: width and height 3..255 and at most %d cells", W, H, OC_MAX_CELLS);
    if (num_agents < 1 || num_agents > OC_MAX_AGENTS) return fail(OC_EINVAL, "num_agents %d", num_agents);
    if (lv->num_spawns < num_agents || lv->num_spawns > OC_MAX_AGENTS) return fail(OC_ELEVEL, "num_spawns %d", lv->num_spawns);
    if (lv->num_items < 0 || lv->num_items > OC_MAX_ITEMS) return fail(OC_ELEVEL, "num_items %d", lv->num_items);
    if (lv->num_goals < 1 || lv->num_goals > OC_MAX_GOALS) return fail(OC_ELEVEL, "num_goals %d", lv->num_goals);
    if (max_T < 0 || max_T > 65535) return fail(OC_EINVAL, "max_T %d", max_T);
    if (device < OC_DEVICE_HOST) return fail(OC_EINVAL, "device %d", device);
    const bool host_only = device == OC_DEVICE_HOST;  // no HIP call at all
    const bool wide = W * H > ocro::kMaxCells;  // u16 cell ids: the scalar step (oc_step_wide_kernel)
    LevelArgs L{};
    L.W = W;
    L.H = H;
    L.done_cell = -1;
    for (int c = 0; c < W * H; ++c) {
        const int t = lv->tiles[c];
        if (t < OC_TILE_FLOOR || t > OC_TILE_DELIVERY) return fail(OC_ELEVEL, "tile %d at cell %d", t, c);
        if (!wide) L.cls4[c >> 2] |= (uint32_t)ocsw::tile_class(t) << (8 * (c & 3));
        if (t == OC_TILE_DELIVERY && L.done_cell < 0) L.done_cell = c;
    }
    if (L.done_cell < 0) return fail(OC_ELEVEL, "no Delivery tile");
    if (lv->encoding != OC_ENC_PRESENCE && lv->encoding != OC_ENC_COUNTS)
        return fail(OC_EINVAL, "encoding %d", lv->encoding);
    const bool counts = lv->encoding == OC_ENC_COUNTS;
    uint32_t seen_food = 0;
    int per_food[3] = {0, 0, 0};
    const int K = lv->num_items <= 4 ? 4 : (lv->num_items <= 8 ? 8 : 16);
    uint16_t cell[16];
    uint8_t mask[16], cell8[16];
    for (int j = 0; j < 16; ++j) {
        cell[j] = wide ? (uint16_t)OC_LOC_DEAD16 : (uint16_t)OC_LOC_DEAD;
        mask[j] = 0;
    }
    for (int j = 0; j < lv->num_items; ++j) {
        const int c = lv->item_cell[j], m = lv->item_mask[j];
        if (c >= W * H || lv->tiles[c] == OC_TILE_FLOOR) return fail(OC_ELEVEL, "item %d not on a counter", j);
        if (counts) {  // a level item is one content: a fresh food (Fresh bit + count 1) or a Plate
            const int f = m == (int)(OC_MC_FRESH | OC_MC_TOMATO) ? 0 : m == (int)(OC_MC_FRESH | OC_MC_LETTUCE) ? 1
                          : m == (int)(OC_MC_FRESH | OC_MC_ONION) ? 2 : -1;
            if (f < 0 && m != (int)OC_MC_PLATE) return fail(OC_ELEVEL, "item mask 0x%x (counts encoding)", m);
            if (f >= 0 && ++per_food[f] > OC_MC_MAX_PER_FOOD)
                return fail(OC_ELEVEL, "more than %d of one food type (2-bit counts)", OC_MC_MAX_PER_FOOD);
        } else {
            if (m == 0 || (m & 0x80) || (((m >> OC_M_CHOPPED_SHIFT) & 7) & ~(m & 7)))
                return fail(OC_ELEVEL, "item mask 0x%x", m);
            if (seen_food & m & 7u)
                return fail(OC_ELEVEL, "food type present twice: the level needs OC_ENC_COUNTS");
            seen_food |= m & 7u;
        }
        cell[j] = (uint16_t)c;
        mask[j] = (uint8_t)m;
    }
    for (int j = 0; j < 16; ++j) cell8[j] = (uint8_t)cell[j];
    for (int a = 0; a < num_agents; ++a) {
        const int x = lv->spawn_x[a], y = lv->spawn_y[a];
        if (x >= W || y >= H || lv->tiles[y * W + x] != OC_TILE_FLOOR) return fail(OC_ELEVEL, "spawn %d not on Floor", a);
        L.tmpl_x |= (uint32_t)x << (8 * a);
        L.tmpl_y |= (uint32_t)y << (8 * a);
    }
    for (int j = 0; j < 16; ++j) {
        L.tmpl_cell[j >> 2] |= (uint32_t)cell8[j] << (8 * (j & 3));
        L.tmpl_mask[j >> 2] |= (uint32_t)mask[j] << (8 * (j & 3));
    }
    for (int g = 0; g < lv->num_goals; ++g) L.goals |= (uint32_t)lv->goal_mask[g] << (8 * g);
    L.ngoals = lv->num_goals;
    L.max_T = max_T;
    const int dcell[5] = {W, -W, -1, 1, 0};
    for (int c = 0; c < 5; ++c) L.dcell_lut |= (uint64_t)((dcell[c] + 128) & 0xFF) << (8 * c);
    ocsw::build_swar_level(L.sw, W, H, L.done_cell, lv->goal_mask, lv->num_goals, max_T, lv->spawn_x, lv->spawn_y,
                           num_agents, cell8, mask, lv->encoding, lv->tiles);
    if (wide) {  // step4w: u16 cells as low / high byte words (the LUTs, x / y and W - 1 stay bytes)
        L.sw.done_rep = (uint32_t)(L.done_cell & 0xFF) * 0x01010101u;
        L.sw.done_hi_rep = (uint32_t)(L.done_cell >> 8) * 0x01010101u;
        for (int j = 0; j < 16; ++j) {
            L.sw.tmpl_l[j] = (uint32_t)(cell[j] & 0xFF) * 0x01010101u;
            L.sw.tmpl_lh[j] = (uint32_t)(cell[j] >> 8) * 0x01010101u;
        }
    }
    oc_handle* h = new oc_handle;
    h->wide = wide;
    h->step = ocro::StepLevel{};
    h->step.done_cell = L.done_cell;
    h->step.max_T = max_T;
    h->step.ngoals = lv->num_goals;
    for (int g = 0; g < lv->num_goals; ++g) h->step.goal[g] = lv->goal_mask[g];
    for (int a = 0; a < num_agents; ++a) {
        h->step.spawn_x[a] = lv->spawn_x[a];
        h->step.spawn_y[a] = lv->spawn_y[a];
    }
    for (int j = 0; j < 16; ++j) {
        h->step.item_cell[j] = cell[j];
        h->step.item_mask[j] = mask[j];
    }
    h->step_lv = ocro::RollLevel{};
    h->step_lv.W = W;
    h->step_lv.H = H;
    h->step_lv.perimeter = 2 * (W + H);
    h->step_lv.enc = lv->encoding;
    h->step_lv.wide = wide ? 1 : 0;
    memset(h->wide_tiles_host, 0, sizeof h->wide_tiles_host);
    for (int c = 0; c < W * H; ++c) h->wide_tiles_host[c] = lv->tiles[c];
    h->level = *lv;
    h->A = num_agents;
    h->K = K;
    h->max_T = max_T;
    h->device = device;
    h->args = L;
    h->cus = 256;  // MI355X; replaced by the device's own count when there is a device
    if (!host_only) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            h->cus = cus;
        else
            (void)hipGetLastError();
    }
    // planner rollout: the static reachability graph's BFS table (world.py:67-108) and the
    // level's other static tables, one blob per level (oc_rollout.h)
    {
        const int n = ocro::build_roll_level(h->roll, h->roll_blob_host, W, H, lv->tiles, lv->encoding);
        if (n < 0) {
            h->roll.nnodes = -1;
        } else if (!host_only) {
            h->roll_blob_bytes = h->roll.blob_bytes;
            if (hipSetDevice(device) != hipSuccess ||
                hipMalloc(&h->roll_blob, (size_t)h->roll_blob_bytes) != hipSuccess ||
                hipMemcpy(h->roll_blob, h->roll_blob_host.data(), (size_t)h->roll_blob_bytes, hipMemcpyHostToDevice) !=
                    hipSuccess) {
                h->roll_blob = nullptr;  // no device (e.g. a CPU-only build check): rollout unavailable
                (void)hipGetLastError();
            }
        }
    }
    if (h->roll.nnodes >= 0) h->roll_blob_bytes = h->roll.blob_bytes;
    if (wide && !host_only) {
        const size_t tb = (size_t)((W * H + 3) & ~3);
        if (hipSetDevice(device) != hipSuccess || hipMalloc(&h->wide_tiles, tb) != hipSuccess ||
            hipMemcpy(h->wide_tiles, h->wide_tiles_host, tb, hipMemcpyHostToDevice) != hipSuccess) {
            h->wide_tiles = nullptr;  // no device: oc_cpu_step only
            (void)hipGetLastError();
        }
    }
    *out = h;
    return OC_OK;
}

// the node table and the distances, as u8 (oc_reachability) or u16 (oc_reachability16)
static int reachability(const oc_handle* h, int32_t* num_nodes, uint16_t* node_of, int64_t node_of_len, void* dist,
                        int64_t dist_len, int out_bytes) {
    if (h == nullptr || num_nodes == nullptr) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    if (h->roll.nnodes < 0)
        return fail(OC_ELEVEL, "reachability graph exceeds %d nodes (a level of more than %d cells)", ocro::kMaxNodesWide,
                    ocro::kMaxCellsWide);
    const int n = h->roll.nnodes, cells = h->level.width * h->level.height;
    *num_nodes = n;
    if (node_of != nullptr) {
        if (node_of_len < (int64_t)cells * 5) return fail(OC_EINVAL, "node_of needs %d entries", cells * 5);
        memcpy(node_of, h->roll_blob_host.data() + h->roll.node_off, (size_t)cells * 5 * sizeof(uint16_t));
    }
    if (dist != nullptr) {
        if (dist_len < (int64_t)n * n) return fail(OC_EINVAL, "dist needs %d entries", n * n);
        const uint8_t* src = h->roll_blob_host.data() + h->roll.dist_off;
        const size_t nn = (size_t)n * n;
        if (out_bytes == 1) {
            if (h->roll.dist16)
                return fail(OC_ELEVEL, "a BFS distance of 255 or more: the u8 table cannot hold it (oc_reachability16)");
            memcpy(dist, src, nn);
        } else if (h->roll.dist16) {
            memcpy(dist, src, nn * 2);
        } else {
            for (size_t i = 0; i < nn; ++i) ((uint16_t*)dist)[i] = src[i] == ocro::kNone ? (uint16_t)0xFFFF : src[i];
        }
    }
    return OC_OK;
}

int oc_reachability(const oc_handle* h, int32_t* num_nodes, uint16_t* node_of, int64_t node_of_len, uint8_t* dist,
                    int64_t dist_len) {
    return reachability(h, num_nodes, node_of, node_of_len, dist, dist_len, 1);
}

int oc_reachability16(const oc_handle* h, int32_t* num_nodes, uint16_t* node_of, int64_t node_of_len, uint16_t* dist,
                      int64_t dist_len) {
    return reachability(h, num_nodes, node_of, node_of_len, dist, dist_len, 2);
}

int oc_destroy(oc_handle* h) {
    if (h != nullptr && h->roll_blob != nullptr) (void)hipFree(h->roll_blob);
    if (h != nullptr && h->wide_tiles != nullptr) (void)hipFree(h->wide_tiles);
    delete h;
    return OC_OK;
}

int oc_get_layout(const oc_handle* h, int64_t B, oc_layout* out) {
    if (h == nullptr || out == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    const int A = h->A, K = h->K;
    out->pitch = pitch_for(B);
    out->num_agents = A;
    out->num_items = K;
    out->plane_agent_x = 0;
    out->plane_agent_y = A;
    out->plane_agent_hold = 2 * A;
    const int LK = h->wide ? 2 * K : K;  // item cell planes: low bytes, then (wide) high bytes
    out->plane_item_loc = 3 * A;
    out->plane_item_loc_hi = h->wide ? 3 * A + K : -1;
    out->cell_bytes = h->wide ? 2 : 1;
    out->plane_item_mask = 3 * A + LK;
    out->plane_t = 3 * A + LK + K;
    out->plane_flags = 3 * A + LK + K + 2;
    out->num_planes = 3 * A + LK + K + 3;
    out->state_bytes = out->num_planes * out->pitch;
    return OC_OK;
}

#define OC_DISPATCH(A_, K_, LAUNCH)                                                         \
    switch ((A_) * ((K_) >= 10 ? 100 : 10) + (K_)) {                                        \
        case 14: LAUNCH(1, 4); break;                                                       \
        case 24: LAUNCH(2, 4); break;                                                       \
        case 34: LAUNCH(3, 4); break;                                                       \
        case 44: LAUNCH(4, 4); break;                                                       \
        case 18: LAUNCH(1, 8); break;                                                       \
        case 28: LAUNCH(2, 8); break;                                                       \
        case 38: LAUNCH(3, 8); break;                                                       \
        case 48: LAUNCH(4, 8); break;                                                       \
        case 116: LAUNCH(1, 16); break;                                                     \
        case 216: LAUNCH(2, 16); break;                                                     \
        case 316: LAUNCH(3, 16); break;                                                     \
        case 416: LAUNCH(4, 16); break;                                                     \
        default: return fail(OC_EINVAL, "unsupported (A,K)=(%d,%d)", (A_), (K_));           \
    }

// The planner kernels: LAUNCH(A, K, W, GD): narrow (byte cell ids) or wide (u16) rows; the
// distance table in LDS (GD false) or in device memory (GD: every wide level, and a narrow level
// whose graph has more than ocro::kMaxNodes nodes).
#define OC_DISPATCH_PLAN(h_, LAUNCH)                                                        \
    if ((h_)->wide) {                                                                       \
        OC_DISPATCH((h_)->A, (h_)->K, OC_PLAN_WIDE)                                         \
    } else if ((h_)->roll.dist_global) {                                                    \
        OC_DISPATCH((h_)->A, (h_)->K, OC_PLAN_NARROW_GD)                                    \
    } else {                                                                                \
        OC_DISPATCH((h_)->A, (h_)->K, OC_PLAN_NARROW)                                       \
    }

// The render kernel: narrow (byte cell ids) or wide (u16) rows.
#define OC_DISPATCH_W(h_, LAUNCH)                                                           \
    if ((h_)->wide) {                                                                       \
        switch ((h_)->A * ((h_)->K >= 10 ? 100 : 10) + (h_)->K) {                           \
            case 14: LAUNCH(1, 4, true); break;                                             \
            case 24: LAUNCH(2, 4, true); break;                                             \
            case 34: LAUNCH(3, 4, true); break;                                             \
            case 44: LAUNCH(4, 4, true); break;                                             \
            case 18: LAUNCH(1, 8, true); break;                                             \
            case 28: LAUNCH(2, 8, true); break;                                             \
            case 38: LAUNCH(3, 8, true); break;                                             \
            case 48: LAUNCH(4, 8, true); break;                                             \
            case 116: LAUNCH(1, 16, true); break;                                           \
            case 216: LAUNCH(2, 16, true); break;                                           \
            case 316: LAUNCH(3, 16, true); break;                                           \
            case 416: LAUNCH(4, 16, true); break;                                           \
            default: return fail(OC_EINVAL, "unsupported (A,K)=(%d,%d)", (h_)->A, (h_)->K); \
        }                                                                                   \
    } else {                                                                                \
        switch ((h_)->A * ((h_)->K >= 10 ? 100 : 10) + (h_)->K) {                           \
            case 14: LAUNCH(1, 4, false); break;                                            \
            case 24: LAUNCH(2, 4, false); break;                                            \
            case 34: LAUNCH(3, 4, false); break;                                            \
            case 44: LAUNCH(4, 4, false); break;                                            \
            case 18: LAUNCH(1, 8, false); break;                                            \
            case 28: LAUNCH(2, 8, false); break;                                            \
            case 38: LAUNCH(3, 8, false); break;                                            \
            case 48: LAUNCH(4, 8, false); break;                                            \
            case 116: LAUNCH(1, 16, false); break;                                          \
            case 216: LAUNCH(2, 16, false); break;                                          \
            case 316: LAUNCH(3, 16, false); break;                                          \
            case 416: LAUNCH(4, 16, false); break;                                          \
            default: return fail(OC_EINVAL, "unsupported (A,K)=(%d,%d)", (h_)->A, (h_)->K); \
        }                                                                                   \
    }

// The step kernels: 4-slot levels of the common class (H <= 8, W*H <= 128, presence masks:
// every shipped kitchen) take the MODE 0 build of the SWAR step, everything else MODE 1.
#define OC_DISPATCH_STEP(h_, LAUNCH)                                                        \
    if ((h_)->K == 4 && !(h_)->args.sw.tall && !(h_)->args.sw.big && !(h_)->args.sw.counts &&  \
        !(h_)->args.sw.edge) {                                                              \
        switch ((h_)->A) {                                                                  \
            case 1: LAUNCH(1, 4, 0); break;                                                 \
            case 2: LAUNCH(2, 4, 0); break;                                                 \
            case 3: LAUNCH(3, 4, 0); break;                                                 \
            case 4: LAUNCH(4, 4, 0); break;                                                 \
            default: return fail(OC_EINVAL, "unsupported A=%d", (h_)->A);                   \
        }                                                                                   \
    } else {                                                                                \
        switch ((h_)->A * ((h_)->K >= 10 ? 100 : 10) + (h_)->K) {                           \
            case 14: LAUNCH(1, 4, 1); break;                                                \
            case 24: LAUNCH(2, 4, 1); break;                                                \
            case 34: LAUNCH(3, 4, 1); break;                                                \
            case 44: LAUNCH(4, 4, 1); break;                                                \
            case 18: LAUNCH(1, 8, 1); break;                                                \
            case 28: LAUNCH(2, 8, 1); break;                                                \
            case 38: LAUNCH(3, 8, 1); break;                                                \
            case 48: LAUNCH(4, 8, 1); break;                                                \
            case 116: LAUNCH(1, 16, 1); break;                                              \
            case 216: LAUNCH(2, 16, 1); break;                                              \
            case 316: LAUNCH(3, 16, 1); break;                                              \
            case 416: LAUNCH(4, 16, 1); break;                                              \
            default: return fail(OC_EINVAL, "unsupported (A,K)=(%d,%d)", (h_)->A, (h_)->K); \
        }                                                                                   \
    }

// Wide levels: n steps of the scalar kernel (oc_step: n = 1), statistics folded by
// oc_stats_reduce when totals are asked for.
static int step_wide(const oc_handle* h, const void* sin, void* sout, const uint8_t* act, void* traj, uint8_t* ex,
                     uint8_t* coll, uint64_t* stats, uint64_t* totals, int64_t B, int32_t n, void* stream) {
    if (h->wide_tiles == nullptr) return fail(OC_EHIP, "level tables not on the device");
    WideArgs R;
    R.L = h->step_lv;
    R.S = h->step;
    R.sw = h->args.sw;
    R.tile_words = (h->level.width * h->level.height + 3) / 4;
    R.pitch = pitch_for(B);
    R.B = B;
    // one lane per 4 envs; up to 8 blocks per CU (grid-stride past that)
    const int64_t need = ((B + kEPL - 1) / kEPL + kBlock - 1) / kBlock, cap = (int64_t)h->cus * 8;
    const dim3 grid((unsigned)(need < cap ? need : cap));
    const uint32_t rows = (uint32_t)stats_rows(h, B);
    hipStream_t st = (hipStream_t)stream;
    // launches of at most `per` steps, so a launch's buffer offsets (trajectory, actions) stay
    // < 2 GiB; each starts from the previous one's final state (as oc_step_n's narrow path)
    const int64_t NP = 3 * h->A + 3 * h->K + 3, P = R.pitch;
    if (NP * P >= (1ll << 31)) return fail(OC_EINVAL, "batch too large for one launch (state must be < 2 GiB)");
    int64_t per = ((1ll << 31) - 1) / (NP * P);
    if (per > 4096) per = 4096;
    per = (n + (n + per - 1) / per - 1) / ((n + per - 1) / per);  // equal launches
    const uint8_t* last_slot = traj ? (const uint8_t*)traj + (int64_t)(n - 1) * NP * P : nullptr;
    const bool out_is_last = traj != nullptr && (const uint8_t*)sout == last_slot;
    const uint8_t* src = (const uint8_t*)sin;
    for (int64_t r0 = 0; r0 < n; r0 += per) {
        const int m = (int)(n - r0 < per ? n - r0 : per);
        const bool last = r0 + m >= n;
        uint8_t* tr = traj ? (uint8_t*)traj + r0 * NP * P : nullptr;
        uint8_t* so = (traj != nullptr && !last) || (out_is_last && last) ? nullptr : (uint8_t*)sout;
        uint8_t* e_ = ex ? ex + r0 * h->A * P : nullptr;
        uint8_t* c_ = coll ? coll + r0 * P : nullptr;
        const uint8_t* a_ = act + r0 * h->A * P;
#define OC_LAUNCH_WSTEP(A, K)                                                                                  \
    hipLaunchKernelGGL((oc_step_wide_kernel<A, K>), grid, dim3(kBlock), 0, st, R, h->wide_tiles, src, so, a_,  \
                       tr, e_, c_, stats, rows, m)
        OC_DISPATCH(h->A, h->K, OC_LAUNCH_WSTEP)
        if (const int rc = hip_check("oc_step (wide) launch")) return rc;
        src = traj != nullptr ? tr + (int64_t)(m - 1) * NP * P : (const uint8_t*)sout;
    }
    return totals != nullptr ? oc_stats_reduce(h, stats, B, totals, stream) : OC_OK;
}

int oc_reset(const oc_handle* h, void* state, int64_t B, void* stream) {
    if (h == nullptr || state == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (B == 0) return OC_OK;
    if (h->wide) {
        WideArgs R;
        R.L = h->step_lv;
        R.S = h->step;
        R.sw = h->args.sw;
        R.tile_words = 0;
        R.pitch = pitch_for(B);
        R.B = B;
        const dim3 grid((unsigned)(R.pitch / kBlock));
        hipStream_t st = (hipStream_t)stream;
#define OC_LAUNCH_WRESET(A, K) hipLaunchKernelGGL((oc_reset_wide_kernel<A, K>), grid, dim3(kBlock), 0, st, R, (uint8_t*)state)
        OC_DISPATCH(h->A, h->K, OC_LAUNCH_WRESET)
        return hip_check("oc_reset (wide) launch");
    }
    LevelArgs L = h->args;
    L.pitch = pitch_for(B);
    L.B = B;
    const dim3 grid((unsigned)(L.pitch / kEnvsPerBlock));
    hipStream_t s = (hipStream_t)stream;
#define OC_LAUNCH_RESET(A, K) hipLaunchKernelGGL((oc_reset_kernel<A, K>), grid, dim3(kBlock), 0, s, L, (uint8_t*)state)
    OC_DISPATCH(h->A, h->K, OC_LAUNCH_RESET)
    return hip_check("oc_reset launch");
}

int oc_step(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
            uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* stats, int64_t B, void* stream) {
    if (h == nullptr || state_in == nullptr || state_out == nullptr || actions == nullptr || B < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (B == 0) return OC_OK;
    if (((uintptr_t)state_in | (uintptr_t)state_out | (uintptr_t)actions | (uintptr_t)exec_actions |
         (uintptr_t)coll_mask) & 15u)
        return fail(OC_EINVAL, "buffers must be 16-byte aligned");
    if (h->wide) return step_wide(h, state_in, state_out, actions, nullptr, exec_actions, coll_mask, stats, nullptr, B, 1, stream);
    LevelArgs L = h->args;
    L.pitch = pitch_for(B);
    L.B = B;
    if ((int64_t)(3 * h->A + 2 * h->K + 3) * L.pitch >= (1ll << 31))
        return fail(OC_EINVAL, "batch too large for one launch (state must be < 2 GiB)");
    const dim3 grid((unsigned)(L.pitch / kEPL / kStepBlock));  // pitch is a multiple of 4096
    const uint32_t rows = (uint32_t)stats_rows(h, B);
    hipStream_t s = (hipStream_t)stream;
#define OC_LAUNCH_STEP(A, K, MODE)                                                                        \
    hipLaunchKernelGGL((oc_step_kernel<A, K, MODE>), grid, dim3(kStepBlock), 0, s, L, (const uint8_t*)state_in, \
                       (uint8_t*)state_out, actions, exec_actions, coll_mask, stats, rows)
    OC_DISPATCH_STEP(h, OC_LAUNCH_STEP)
    return hip_check("oc_step launch");
}

int oc_cpu_step(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
                uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* totals, int64_t B, int32_t nthreads) {
    if (h == nullptr || state_in == nullptr || state_out == nullptr || actions == nullptr || B < 0 || nthreads < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    if (B == 0) return OC_OK;
    const int64_t P = pitch_for(B), words = (B + kEPL - 1) / kEPL;
    if (nthreads == 0) nthreads = (int32_t)std::thread::hardware_concurrency();
    int64_t nt = nthreads < 1 ? 1 : nthreads;
    if (nt > (words + 4095) / 4096) nt = (words + 4095) / 4096;  // >= 4096 words (16 Ki envs) per thread
    if (nt < 1) nt = 1;
    std::vector<uint64_t> part((size_t)nt * OC_NSTATS, 0);
    auto run = [&](int64_t i) {
        const int64_t g0 = words * i / nt, g1 = words * (i + 1) / nt;
        const uint8_t* si = (const uint8_t*)state_in;
        uint8_t* so = (uint8_t*)state_out;
        uint64_t* st = part.data() + i * OC_NSTATS;
        if (h->wide) {  // the wide SWAR step (step4w), four envs per word as the kernel
#define OC_CPU_WSTEP(A, K) cpu_step_wide<A, K>(h, si, so, actions, exec_actions, coll_mask, B, P, g0, g1, st)
            OC_DISPATCH(h->A, h->K, OC_CPU_WSTEP)
#undef OC_CPU_WSTEP
            return OC_OK;
        }
#define OC_CPU_STEP(A, K, MODE) cpu_step_words<A, K, MODE>(h, si, so, actions, exec_actions, coll_mask, B, P, g0, g1, st)
        OC_DISPATCH_STEP(h, OC_CPU_STEP)
#undef OC_CPU_STEP
        return OC_OK;
    };
    // Every range runs the same (A, K, MODE) dispatch, so it is checked once here, on the calling
    // thread (an unsupported shape fails before any thread starts).  Then ranges 1..nt-1 start on
    // workers and range 0 runs on the calling thread while they work; a worker's failure message
    // is still carried back.  Ranges whose thread cannot be started run here too.
#define OC_CPU_NOP(...) (void)0
    if (h->wide) {
        OC_DISPATCH(h->A, h->K, OC_CPU_NOP)
    } else {
        OC_DISPATCH_STEP(h, OC_CPU_NOP)
    }
#undef OC_CPU_NOP
    std::vector<std::thread> pool;
    std::vector<int> rcs((size_t)nt, OC_OK);
    std::vector<std::string> msgs((size_t)nt);
    int64_t started = 1;
    try {
        for (; started < nt; ++started)
            pool.emplace_back([&, i = started] {
                rcs[(size_t)i] = run(i);
                if (rcs[(size_t)i] != OC_OK) msgs[(size_t)i] = g_last_error;
            });
    } catch (const std::exception&) {  // no more threads: the rest of the ranges run here
    }
    int rc = run(0);
    for (int64_t i = started; i < nt; ++i) {
        rcs[(size_t)i] = run(i);
        if (rcs[(size_t)i] != OC_OK) msgs[(size_t)i] = g_last_error;
    }
    for (auto& t : pool) t.join();
    for (int64_t i = 1; i < nt && rc == OC_OK; ++i)
        if (rcs[(size_t)i] != OC_OK) rc = fail(rcs[(size_t)i], "%s", msgs[(size_t)i].c_str());
    if (rc == OC_OK && totals != nullptr)
        for (int64_t i = 0; i < nt; ++i)
            for (int c = 0; c < OC_NSTATS; ++c) totals[c] += part[(size_t)(i * OC_NSTATS + c)];
    return rc;
}

int oc_step_n(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions, void* traj,
              uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* stats, uint64_t* totals, int64_t B, int32_t n,
              void* stream) {
    if (h == nullptr || state_in == nullptr || state_out == nullptr || actions == nullptr || B < 0 || n < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (totals != nullptr && stats == nullptr) return fail(OC_EINVAL, "totals need the stats buffer");
    if (totals != nullptr && (uintptr_t)totals & 7u) return fail(OC_EINVAL, "totals must be 8-byte aligned");
    if (B == 0 || n == 0) return totals != nullptr && B > 0 ? oc_stats_reduce(h, stats, B, totals, stream) : OC_OK;
    if (((uintptr_t)state_in | (uintptr_t)state_out | (uintptr_t)actions | (uintptr_t)traj | (uintptr_t)exec_actions |
         (uintptr_t)coll_mask) & 15u)
        return fail(OC_EINVAL, "buffers must be 16-byte aligned");
    LevelArgs L = h->args;
    L.pitch = pitch_for(B);
    L.B = B;
    const int64_t NP = 3 * h->A + (h->wide ? 3 : 2) * h->K + 3;
    // state_out may be the trajectory's last state (written once); nothing else may overlap it
    const uint8_t* last_slot = traj ? (const uint8_t*)traj + (int64_t)(n - 1) * NP * L.pitch : nullptr;
    const bool out_is_last = traj != nullptr && (const uint8_t*)state_out == last_slot;
    if (traj != nullptr) {
        const uint8_t *t0 = (const uint8_t*)traj, *t1 = t0 + (int64_t)n * NP * L.pitch;
        auto overlaps = [&](const void* p) {
            const uint8_t* q = (const uint8_t*)p;
            return q + NP * L.pitch > t0 && q < t1;
        };
        if (overlaps(state_in) || (overlaps(state_out) && !out_is_last))
            return fail(OC_EINVAL, "traj must not overlap the state (state_out may be its last state)");
    }
    if (h->wide) return step_wide(h, state_in, state_out, actions, traj, exec_actions, coll_mask, stats, totals, B, n, stream);
    if (NP * L.pitch >= (1ll << 31)) return fail(OC_EINVAL, "batch too large for one launch (state must be < 2 GiB)");
    // steps per launch so every per-launch buffer (trajectory, actions) stays < 2 GiB of offsets
    int64_t per = ((1ll << 31) - 1) / (NP * L.pitch);
    if (per > 4096) per = 4096;
    per = (n + (n + per - 1) / per - 1) / ((n + per - 1) / per);  // equal launches
    // <= 5 waves per SIMD resident: 5 blocks of 4 waves per CU, or 4 of 5 with the loader wave
    const int64_t need = L.pitch / kEnvsPerBlock;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t rows = (uint32_t)stats_rows(h, B);
    const uint8_t* src = (const uint8_t*)state_in;
    for (int64_t r0 = 0; r0 < n; r0 += per) {
        const int m = (int)(n - r0 < per ? n - r0 : per);
        const int64_t off = r0;
        uint8_t* tr = traj ? (uint8_t*)traj + off * NP * L.pitch : nullptr;
        uint8_t* ex = exec_actions ? exec_actions + off * h->A * L.pitch : nullptr;
        uint8_t* cm = coll_mask ? coll_mask + off * L.pitch : nullptr;
        const uint8_t* ac = actions + off * h->A * L.pitch;
        // With a trajectory, a launch's final state is its last trajectory slot: the next launch
        // starts from there, and state_out is written by the last launch only (and not at all
        // when it is the trajectory's last state).  So no launch reads a buffer it also writes.
        const bool last = r0 + m >= n;
        uint8_t* so = (traj != nullptr && !last) || (out_is_last && last) ? nullptr : (uint8_t*)state_out;
#define OC_LAUNCH_STEPN(A, K, MODE)                                                                    \
    {                                                                                                  \
        constexpr bool kLW = use_loader_wave<A, K, MODE>();                                           \
        const int64_t cap = (int64_t)h->cus * (kLW ? 4 : 5);                                           \
        const dim3 grid((unsigned)(need < cap ? need : cap));                                          \
        hipLaunchKernelGGL((oc_step_n_kernel<A, K, kCPnt, 0, MODE>), grid, dim3(kBlock + (kLW ? 64 : 0)), 0, s, L, \
                           src, so, ac, tr, ex, cm, stats, last ? totals : nullptr, rows, m);                 \
    }
        OC_DISPATCH_STEP(h, OC_LAUNCH_STEPN)
        src = traj != nullptr ? tr + (int64_t)(m - 1) * NP * L.pitch : (const uint8_t*)state_out;
        if (const int rc = hip_check("oc_step_n launch")) return rc;
    }
    return OC_OK;
}

// Shared argument block of oc_rollout / oc_nav_likelihood / oc_subtask_bounds: level tables +
// validated subtasks.  rollout: oc_rollout's call (Level-1 configurations allowed; the
// node-to-square table staged only for launches of one round of blocks, below).
static int roll_args(const oc_handle* h, const oc_subtask* subtasks, int32_t num_subtasks, int64_t B, RollArgs& R,
                     bool rollout = false) {
    for (int i = 0; i < num_subtasks && subtasks != nullptr; ++i)
        if (subtasks[i].level != OC_LEVEL0 && !rollout)
            return fail(OC_EINVAL, "subtask %d: only oc_rollout takes OC_LEVEL1", i);
    if (num_subtasks < 1 || num_subtasks > OC_MAX_SUBTASKS) return fail(OC_EINVAL, "num_subtasks %d", num_subtasks);
    if (h->roll.nnodes < 0)
        return fail(OC_ELEVEL, "reachability graph exceeds %d nodes (a level of more than %d cells)", ocro::kMaxNodesWide,
                    ocro::kMaxCellsWide);
    if (h->roll_blob == nullptr) return fail(OC_EHIP, "rollout tables not on the device");
    R.L = h->roll;
    R.nsub = num_subtasks;
    R.blob_words = h->roll.lds_bytes / 4;  // staged in LDS: the whole blob, or the tables before the distances
    if (R.L.sq_off != 0 && rollout && B > (int64_t)h->cus * kRollBlock) {
        // The node-to-square table (the blob's tail) shortens the one-agent Merge bound from ~3.8
        // to 1.1-2.0 us of a wave.  A rollout launch of one round of blocks (the planner's latency
        // shape) gains (9.03 -> 8.87 us at 4096 rows); past that every rollout block stages 40%
        // more table for one row per lane (11.16-11.34 -> 11.35-11.51 us at 2^18: tools/rollx.hip,
        // profiles/r06/pass_i), so larger rollouts search B's approach nodes as before.  The bounds
        // kernel (many configurations per staged table) gains at every size, 96-97 -> 85 us at C5,
        // and the likelihood kernels are unchanged (profiles/r06/pass_w).
        R.blob_words = R.L.sq_off / 4;
        R.L.sq_off = 0;
    }
    R.pitch = pitch_for(B);
    R.B = B;
    for (int i = 0; i < num_subtasks; ++i) {
        const oc_subtask& s = subtasks[i];
        if (s.kind < OC_SUB_NONE || s.kind > OC_SUB_DELIVER) return fail(OC_EINVAL, "subtask %d kind %d", i, s.kind);
        if (s.num_agents < 1 || s.num_agents > 2) return fail(OC_EINVAL, "subtask %d: %d agents", i, s.num_agents);
        for (int q = 0; q < s.num_agents; ++q)
            if (s.agent[q] >= h->A) return fail(OC_EINVAL, "subtask %d: agent %d", i, s.agent[q]);
        if (s.num_agents == 2 && s.agent[0] >= s.agent[1]) return fail(OC_EINVAL, "subtask %d: agents not ascending", i);
        ocro::Sub& d = R.subs[i];
        d.kind = s.kind;
        d.n = s.num_agents;
        d.agent[0] = s.agent[0];
        d.agent[1] = s.num_agents == 2 ? s.agent[1] : s.agent[0];
        d.start[0] = s.start_mask[0];
        d.start[1] = s.start_mask[1];
        if (s.level > OC_LEVEL1) return fail(OC_EINVAL, "subtask %d: level %d", i, s.level);
        d.goal = s.goal_mask;
        d.count = s.goal_count;
        d.level = s.level;
        d.pad = 0;
    }
    return OC_OK;
}

// The planner kernels stage the level's table blob in dynamic LDS.  Past the 64 KB a launch gets
// by default (graphs of more than ~245 nodes) the kernel must be allowed more, up to the CU's
// 160 KB; the kernel's static LDS counts against the same limit.
constexpr int kLdsPerCu = 160 * 1024;
static int allow_dyn_lds(const void* kernel, int dyn) {
    if (dyn <= 48 * 1024) return OC_OK;
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, kernel) != hipSuccess) return hip_check("hipFuncGetAttributes");
    if ((int64_t)fa.sharedSizeBytes + dyn > kLdsPerCu)
        return fail(OC_ELEVEL, "level tables (%d B) and the kernel's LDS (%d B) exceed %d B", dyn,
                    (int)fa.sharedSizeBytes, kLdsPerCu);
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, dyn) != hipSuccess)
        return hip_check("hipFuncSetAttribute");
    return OC_OK;
}

int oc_rollout(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
               const uint8_t* alloc, const oc_subtask* subtasks, int32_t num_subtasks, uint8_t* out_flags,
               float* lower_bound, int64_t B, void* stream) {
    if (h == nullptr || state_in == nullptr || state_out == nullptr || actions == nullptr || subtasks == nullptr ||
        out_flags == nullptr || lower_bound == nullptr || B < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (state_in == state_out) return fail(OC_EINVAL, "oc_rollout is out of place");
    if (((uintptr_t)lower_bound & 3u) || ((uintptr_t)state_in & 1u) || ((uintptr_t)state_out & 1u))
        return fail(OC_EINVAL, "misaligned buffer");
    RollArgs R;
    if (const int rc = roll_args(h, subtasks, num_subtasks, B, R, true)) return rc;
    if (B == 0) return OC_OK;
    const int64_t need = (B + kRollBlock - 1) / kRollBlock, cap = (int64_t)h->cus * 8 * kBlock / kRollBlock;
    const dim3 grid((unsigned)(need < cap ? need : cap));
    hipStream_t st = (hipStream_t)stream;
    if (!h->wide && !h->roll.dist_global && B * kRollGroup <= (int64_t)h->cus * kRollBlock) {
        // one round of blocks with a lane group per row (oc_rollout_group_kernel)
        const dim3 ggrid((unsigned)((B * kRollGroup + kRollBlock - 1) / kRollBlock));
#define OC_LAUNCH_ROLL_GROUP(A, K)                                                                                  \
    if (const int rc = allow_dyn_lds((const void*)oc_rollout_group_kernel<A, K>, R.blob_words * 4)) return rc;        \
    hipLaunchKernelGGL((oc_rollout_group_kernel<A, K>), ggrid, dim3(kRollBlock), R.blob_words * 4, st, R,            \
                       (const uint8_t*)state_in, (uint8_t*)state_out, actions, alloc, h->roll_blob, out_flags, lower_bound)
        OC_DISPATCH(h->A, h->K, OC_LAUNCH_ROLL_GROUP)
#undef OC_LAUNCH_ROLL_GROUP
        return hip_check("oc_rollout launch");
    }
#define OC_LAUNCH_ROLL(A, K, W, GD)                                                                             \
    if (const int rc = allow_dyn_lds((const void*)oc_rollout_kernel<A, K, W, GD>, R.blob_words * 4)) return rc;   \
    hipLaunchKernelGGL((oc_rollout_kernel<A, K, W, GD>), grid, dim3(kRollBlock), R.blob_words * 4, st, R,            \
                       (const uint8_t*)state_in, (uint8_t*)state_out, actions, alloc, h->roll_blob, out_flags,       \
                       lower_bound)
#define OC_PLAN_WIDE(A, K) OC_LAUNCH_ROLL(A, K, true, true)
#define OC_PLAN_NARROW_GD(A, K) OC_LAUNCH_ROLL(A, K, false, true)
#define OC_PLAN_NARROW(A, K) OC_LAUNCH_ROLL(A, K, false, false)
    OC_DISPATCH_PLAN(h, OC_LAUNCH_ROLL)
#undef OC_PLAN_WIDE
#undef OC_PLAN_NARROW_GD
#undef OC_PLAN_NARROW
    return hip_check("oc_rollout launch");
}

int oc_nav_likelihood(const oc_handle* h, const void* state, const uint8_t* taken, const uint8_t* alloc,
                      const oc_subtask* subtasks, int32_t num_subtasks, int32_t self_agent, double beta,
                      double none_action_prob, double* likelihood, uint8_t* out_flags, int64_t B, void* stream) {
    if (h == nullptr || state == nullptr || taken == nullptr || subtasks == nullptr || likelihood == nullptr ||
        out_flags == nullptr || B < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (self_agent < 0 || self_agent >= h->A) return fail(OC_EINVAL, "self_agent %d", self_agent);
    if (((uintptr_t)likelihood & 7u) || ((uintptr_t)state & 1u)) return fail(OC_EINVAL, "misaligned buffer");
    RollArgs R;
    if (const int rc = roll_args(h, subtasks, num_subtasks, B, R)) return rc;
    if (B == 0) return OC_OK;
    bool any_joint = false;  // lanes per row: one per candidate with a two-agent configuration
    for (int i = 0; i < num_subtasks; ++i) any_joint |= subtasks[i].num_agents == 2;
    const int64_t G = any_joint ? 32 : 8;
    // grid: up to 16 blocks per CU with 32-lane groups (5 resident per CU: measured 0.35 vs
    // 0.39 ms per 2^18 C5 rows against 8 per CU), 8 per CU with 8-lane groups (3-4 resident)
    // the compacted form's row slots take up to kLikCompactLds more LDS: a level whose tables
    // leave less than that runs the grouped form (same outputs)
    // (oc_set_likelihood_form(h, OC_LIK_FORM_GROUPED) forces the grouped form: the parity test of that path)
    const bool compact = OC_LIK_COMPACT && h->lik_form == OC_LIK_FORM_AUTO &&
                         h->roll.lds_bytes + kLikCompactLds + (int)sizeof(ocro::Sub) * OC_MAX_SUBTASKS <= kLdsPerCu;
    const int64_t rows_per_block = compact ? (kBlock / 64) * lik_rows_per_round((int)G) : kBlock / G;
    const int64_t need = (B + rows_per_block - 1) / rows_per_block, cap = (int64_t)h->cus * (any_joint ? 16 : 8);
    const dim3 grid((unsigned)(need < cap ? need : cap));
    hipStream_t st = (hipStream_t)stream;
#define OC_LIK_GO(KERN, A, K, GG, W, GD)                                                                             \
    do {                                                                                                             \
        if (const int rc = allow_dyn_lds((const void*)KERN<A, K, GG, W, GD>, R.blob_words * 4)) return rc;          \
        hipLaunchKernelGGL((KERN<A, K, GG, W, GD>), grid, dim3(kBlock), R.blob_words * 4, st, R, (const uint8_t*)state, \
                           taken, alloc, h->roll_blob, self_agent, beta, none_action_prob, likelihood, out_flags);   \
    } while (0)
#define OC_LAUNCH_LIK(A, K, W, GD)                                                                                   \
    if (compact && any_joint)                                                                                        \
        OC_LIK_GO(oc_likelihood_compact_kernel, A, K, 32, W, GD);                                                    \
    else if (compact)                                                                                                \
        OC_LIK_GO(oc_likelihood_compact_kernel, A, K, 8, W, GD);                                                     \
    else if (any_joint)                                                                                              \
        OC_LIK_GO(oc_likelihood_kernel, A, K, 32, W, GD);                                                            \
    else                                                                                                             \
        OC_LIK_GO(oc_likelihood_kernel, A, K, 8, W, GD)
#define OC_PLAN_WIDE(A, K) OC_LAUNCH_LIK(A, K, true, true)
#define OC_PLAN_NARROW_GD(A, K) OC_LAUNCH_LIK(A, K, false, true)
#define OC_PLAN_NARROW(A, K) OC_LAUNCH_LIK(A, K, false, false)
    OC_DISPATCH_PLAN(h, OC_LAUNCH_LIK)
#undef OC_PLAN_WIDE
#undef OC_PLAN_NARROW_GD
#undef OC_PLAN_NARROW
    return hip_check("oc_nav_likelihood launch");
}

// configuration chunks: enough blocks for this many per CU (round 2's sweep, 0.44 ms kernels:
// 64 best; round 5, 0.09 ms kernels with each block staging the tables: 32 at 0.0916-0.0924 ms
// against 0.0925-0.0938 at 64 and 0.0925-0.0931 at 24, profiles/r05/ab/ab_bounds_chunks.jsonl)
#ifndef OC_BOUNDS_BLOCKS_PER_CU
#define OC_BOUNDS_BLOCKS_PER_CU 32
#endif
int oc_subtask_bounds(const oc_handle* h, const void* state, const oc_subtask* subtasks, int32_t num_subtasks,
                      float* lower_bound, uint8_t* doable, int64_t B, void* stream) {
    if (h == nullptr || state == nullptr || subtasks == nullptr || lower_bound == nullptr || doable == nullptr ||
        B < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (((uintptr_t)lower_bound & 3u) || ((uintptr_t)state & 1u)) return fail(OC_EINVAL, "misaligned buffer");
    RollArgs R;
    if (const int rc = roll_args(h, subtasks, num_subtasks, B, R)) return rc;
    if (B == 0) return OC_OK;
    const int64_t need = (B + kBlock - 1) / kBlock, cap = (int64_t)h->cus * 8;
    const int64_t bx = need < cap ? need : cap;
    // configuration chunks: enough blocks for OC_BOUNDS_BLOCKS_PER_CU per CU, at most one
    // configuration per chunk (round 2, C5, 2^18 envs x 64 configurations: 0.75 ms unchunked,
    // 0.53 / 0.46 / 0.44 / 0.44 ms at 16 / 32 / 64 / 128 blocks per CU, 0.47 ms at one
    // configuration per block; profiles/r02/bounds_chunk_sweep.log; round 5: see the macro)
    int64_t chunks = ((int64_t)h->cus * OC_BOUNDS_BLOCKS_PER_CU + bx - 1) / bx;
    if (chunks > R.nsub) chunks = R.nsub;
    if (chunks < 1) chunks = 1;
    const dim3 grid((unsigned)bx, (unsigned)chunks);
    hipStream_t st = (hipStream_t)stream;
#define OC_LAUNCH_BOUNDS(A, K, W, GD)                                                                         \
    if (const int rc = allow_dyn_lds((const void*)oc_bounds_kernel<A, K, W, GD>, R.blob_words * 4)) return rc;  \
    hipLaunchKernelGGL((oc_bounds_kernel<A, K, W, GD>), grid, dim3(kBlock), R.blob_words * 4, st, R,           \
                       (const uint8_t*)state, h->roll_blob, lower_bound, doable)
#define OC_PLAN_WIDE(A, K) OC_LAUNCH_BOUNDS(A, K, true, true)
#define OC_PLAN_NARROW_GD(A, K) OC_LAUNCH_BOUNDS(A, K, false, true)
#define OC_PLAN_NARROW(A, K) OC_LAUNCH_BOUNDS(A, K, false, false)
    OC_DISPATCH_PLAN(h, OC_LAUNCH_BOUNDS)
#undef OC_PLAN_WIDE
#undef OC_PLAN_NARROW_GD
#undef OC_PLAN_NARROW
    return hip_check("oc_subtask_bounds launch");
}

int oc_render(const oc_handle* h, const void* state, const uint32_t* atlas, const uint32_t* background,
              const oc_render_desc* desc, uint8_t* out, int64_t B, void* stream) {
    return oc_render_ordered(h, state, nullptr, atlas, background, desc, out, B, stream);
}

int oc_render_ordered(const oc_handle* h, const void* state, const uint8_t* draw_rank, const uint32_t* atlas,
                      const uint32_t* background, const oc_render_desc* desc, uint8_t* out, int64_t B,
                      void* stream) {
    if (h == nullptr || state == nullptr || atlas == nullptr || background == nullptr || desc == nullptr ||
        out == nullptr || B < 0)
        return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    const int W = h->level.width, H = h->level.height;
    if (W > kRenderMaxW) return fail(OC_ELEVEL, "render: width %d > %d", W, kRenderMaxW);  // oc_create caps it at 255
    if (desc->tile < kRenderPx || desc->tile % kRenderPx != 0 || desc->tile > 1024)
        return fail(OC_EINVAL, "render: tile %d (a multiple of %d)", desc->tile, kRenderPx);
    for (int c = 0; c < OC_RENDER_SIZES; ++c)
        if (desc->size[c] < 0 || desc->offset[c] < 0 || desc->size[c] + desc->offset[c] > desc->tile)
            return fail(OC_EINVAL, "render: size class %d (%d at %d) leaves the %d-px cell", c, desc->size[c],
                        desc->offset[c], desc->tile);
    for (int q = 0; q < 3; ++q)
        if (((desc->chan_map >> (8 * q)) & 0xFFu) > 3u) return fail(OC_EINVAL, "render: chan_map 0x%x", desc->chan_map);
    if (((uintptr_t)atlas | (uintptr_t)background | (uintptr_t)out) & 15u) return fail(OC_EINVAL, "misaligned buffer");
    if (B == 0) return OC_OK;
    if (B * H * 2 > 0x7FFFFFFFll) return fail(OC_EINVAL, "render: batch too large");
    RenderArgs R;
    R.W = W;
    R.H = H;
    R.tile = desc->tile;
    for (int c = 0; c < OC_RENDER_SIZES; ++c) {
        R.size[c] = desc->size[c];
        R.offset[c] = desc->offset[c];
        R.food_base[c] = desc->food_base[c];
    }
    R.plate_off[0] = desc->plate_off[0];
    R.plate_off[1] = desc->plate_off[1];
    for (int a = 0; a < OC_MAX_AGENTS; ++a) R.agent_off[a] = desc->agent_off[a];
    R.chan_map = desc->chan_map;
    R.counts = h->level.encoding == OC_ENC_COUNTS;
    R.pitch = pitch_for(B);
    for (int m = 0; m < 128; ++m) R.food_sprite[m] = desc->food_sprite[m];
    R.parts = 2;  // two blocks per (env, cell row): 0.198 vs 0.214 ms per 1,024 images (3 or 4: 0.211-0.213)
    const dim3 grid((unsigned)(B * H * R.parts));
    hipStream_t st = (hipStream_t)stream;
#define OC_LAUNCH_RENDER(A, K, WD)                                                                               \
    hipLaunchKernelGGL((oc_render_kernel<A, K, WD>), grid, dim3(kBlock), 0, st, R, (const uint8_t*)state, draw_rank, \
                       atlas, background, out)
    OC_DISPATCH_W(h, OC_LAUNCH_RENDER)
    return hip_check("oc_render launch");
}

int oc_gen_actions(const oc_handle* h, uint8_t* actions, int64_t B, int64_t env_offset, int64_t step,
                   uint64_t seed, void* stream) {
    if (h == nullptr || actions == nullptr || B < 0 || env_offset < 0 || step < 0) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    if (B == 0) return OC_OK;
    const int64_t P = pitch_for(B);
    hipLaunchKernelGGL(oc_gen_actions_kernel, dim3((unsigned)(P / kBlock)), dim3(kBlock), 0, (hipStream_t)stream,
                       actions, h->A, B, P, env_offset, (uint64_t)step, seed);
    return hip_check("oc_gen_actions launch");
}

int oc_state_checksum(const oc_handle* h, const void* state, int64_t B, uint64_t* out, void* stream) {
    if (h == nullptr || state == nullptr || out == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(out, 0, sizeof(uint64_t), s) != hipSuccess) return hip_check("oc_state_checksum memset");
    if (B == 0) return OC_OK;
    const int64_t P = pitch_for(B);
    const int np = 3 * h->A + (h->wide ? 3 : 2) * h->K + 3;
    const dim3 grid((unsigned)(P / kEnvsPerBlock));
#define OC_CK(NP) hipLaunchKernelGGL((oc_checksum_kernel<NP>), grid, dim3(kBlock), 0, s, (const uint8_t*)state, P, B, (unsigned long long*)out)
    switch (np) {
        case 17: OC_CK(17); break;   // A=2 K=4
        case 14: OC_CK(14); break;   // A=1 K=4
        case 20: OC_CK(20); break;   // A=3 K=4
        case 23: OC_CK(23); break;   // A=4 K=4
        case 22: OC_CK(22); break;   // A=1 K=8
        case 25: OC_CK(25); break;   // A=2 K=8
        case 28: OC_CK(28); break;   // A=3 K=8
        case 31: OC_CK(31); break;   // A=4 K=8
        case 38: OC_CK(38); break;   // A=1 K=16
        case 41: OC_CK(41); break;   // A=2 K=16
        case 44: OC_CK(44); break;   // A=3 K=16
        case 47: OC_CK(47); break;   // A=4 K=16
        case 18: OC_CK(18); break;   // wide: A=1 K=4
        case 21: OC_CK(21); break;   // wide: A=2 K=4
        case 24: OC_CK(24); break;   // wide: A=3 K=4
        case 27: OC_CK(27); break;   // wide: A=4 K=4
        case 30: OC_CK(30); break;   // wide: A=1 K=8
        case 33: OC_CK(33); break;   // wide: A=2 K=8
        case 36: OC_CK(36); break;   // wide: A=3 K=8
        case 39: OC_CK(39); break;   // wide: A=4 K=8
        case 54: OC_CK(54); break;   // wide: A=1 K=16
        case 57: OC_CK(57); break;   // wide: A=2 K=16
        case 60: OC_CK(60); break;   // wide: A=3 K=16
        case 63: OC_CK(63); break;   // wide: A=4 K=16
        default: return fail(OC_EINVAL, "unsupported plane count %d", np);
    }
    return hip_check("oc_state_checksum launch");
}

int oc_stats_size(const oc_handle* h, int64_t B, int64_t* nbytes) {
    if (h == nullptr || nbytes == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    const int64_t groups = ((int64_t)h->cus * 5 + kTicketGroup - 1) / kTicketGroup;  // oc_step_n's grid <= 5 blocks per CU
    *nbytes = (ticket_base(stats_rows(h, B)) + (1 + groups) * kTicketStride) * (int64_t)sizeof(uint64_t);
    return OC_OK;
}

int oc_stats_reduce(const oc_handle* h, const uint64_t* stats, int64_t B, uint64_t* totals, void* stream) {
    if (h == nullptr || stats == nullptr || totals == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    ErrScope es_(h);
    OC_NEED_DEVICE(h);
    const int64_t rows = stats_rows(h, B);
    hipLaunchKernelGGL(oc_stats_reduce_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, stats, rows, totals);
    return hip_check("oc_stats_reduce launch");
}

}  // extern "C"
