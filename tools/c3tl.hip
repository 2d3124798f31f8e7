// tools/c3tl.hip -- a per-wave timeline of the C3 multi-step kernel (round 5):
// where do the last ~0.9 us/step between oc_step_n<3,4> with its loader wave and the no-load
// floor go?  Includes the engine TU.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o tools/c3tl tools/c3tl.hip
// Workload: bench.py's C3 -- full-divider_tl, 3 agents, 2^20 envs, 100-step launches, every
// step's state, executed actions and collision mask written (nt stores), mid-run start state.
// Variants (a copy of oc_step_n_kernel's stepping loop with s_memrealtime stamps, 100 MHz):
//   lw      the product's loader-wave form (a fifth wave loads the action words 4 steps at a time
//           into an LDS ring; an LDS barrier every 4 steps hands a ring half over)
//   noload  the actions hashed in-kernel: no load and no barrier in the loop (the floor)
//   lw_nostamp / noload_nostamp: the same without the stamps, to see what the stamps cost
// Per sampled stepping wave and step: the step's start (after the ring read; after the barrier
// on every 4th step), its compute end (step4 returned) and its store-issue end.  Printed:
// per-step time split (barrier wait, compute, store issue) over waves and steps, and the spread
// of the waves' progress (how far apart the waves of a block and of the grid run).
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <algorithm>
#include <type_traits>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

constexpr int kSample = 8;      // every 8th stepping wave of the grid is recorded
constexpr int kMaxSteps = 100;

__device__ __forceinline__ uint64_t now() { return wall_clock64(); }

template <int A, int K, int MODE, bool LW, bool NOLOAD, bool STAMP, int SW = 4, int LB = 5>
__global__ __launch_bounds__(SW * 64 + (LW ? 64 : 0), LW ? LB : 1) void stepn_tl(LevelArgs L, const uint8_t* __restrict__ sin,
                                                                             uint8_t* __restrict__ sout,
                                                                             const uint8_t* __restrict__ actions,
                                                                             uint8_t* __restrict__ traj,
                                                                             uint8_t* __restrict__ exec_out,
                                                                             uint8_t* __restrict__ coll_out, int n,
                                                                             uint64_t* __restrict__ tl) {
    constexpr int CP = kCPnt, LCP = 0;
    __shared__ uint32_t tbl4[64];
    constexpr int kBS = SW * 64;  // stepping lanes per block
    __shared__ uint32_t ring[LW ? 2 * kLwSteps * SW * A * 64 : 1];
    if (threadIdx.x < 64u) tbl4[threadIdx.x] = L.cls4[threadIdx.x];
    __syncthreads();
    const bool loader = LW && threadIdx.x >= (uint32_t)kBS;
    const uint32_t lane = threadIdx.x & 63u;
    const uint8_t* tbl = (const uint8_t*)tbl4;
    const uint32_t P = (uint32_t)L.pitch, nlanes = P / kEPL, stride = gridDim.x * (uint32_t)kBS;
    constexpr int NP = 3 * A + 2 * K + 3;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    auto cls_of = [&](uint32_t cells) -> uint32_t {
        const uint32_t b0 = tbl[cells & 0xFFu], b1 = tbl[(cells >> 8) & 0xFFu], b2 = tbl[(cells >> 16) & 0xFFu],
                       b3 = tbl[cells >> 24];
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    };
    Bufs b;
    b.sin = make_rsrc(sin, (int64_t)NP * P);
    b.sout = make_rsrc(sout, (int64_t)NP * P);
    b.act = make_rsrc(actions, (int64_t)n * A * P);
    const __amdgpu_buffer_rsrc_t tr = make_rsrc(traj, (int64_t)n * NP * P);
    b.ex = make_rsrc(exec_out, (int64_t)n * A * P);
    b.coll = make_rsrc(coll_out, (int64_t)n * P);
    StepStats st;
    const uint32_t gwave = (blockIdx.x * (uint32_t)kBS + threadIdx.x) / 64u;  // stepping waves
    const bool rec = STAMP && !loader && (gwave % kSample) == 0u && lane == 0u;
    uint64_t* out = tl + (uint64_t)(gwave / kSample) * (3 * kMaxSteps + 3);
    if (rec) out[0] = now();
    typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
    for (uint32_t gb = blockIdx.x * (uint32_t)kBS; gb < nlanes; gb += stride) {
        if (loader) {
            auto fill = [&](int r0, int h) {
                uint32_t w[kLwSteps][SW][A];
#pragma unroll
                for (int q = 0; q < kLwSteps; ++q)
#pragma unroll
                    for (int v = 0; v < SW; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            w[q][v][a] = r0 + q < n ? bld32<LCP>(b.act, (gb + 64u * v + lane) * 4u,
                                                                 (uint32_t)((r0 + q) * A + a) * P)
                                                    : 0u;
#pragma unroll
                for (int q = 0; q < kLwSteps; ++q)
#pragma unroll
                    for (int v = 0; v < SW; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            ring[(((h * kLwSteps + q) * SW + v) * A + a) * 64 + lane] = w[q][v][a];
            };
            fill(0, 0);
            for (int r0 = 0; r0 < n; r0 += kLwSteps) {
                lds_barrier();
                if (r0 + kLwSteps < n) fill(r0 + kLwSteps, ((r0 / kLwSteps) & 1) ^ 1);
            }
            lds_barrier();
            continue;
        }
        const uint32_t g = gb + threadIdx.x;
        const bool live = g < nlanes;
        Chunk<A, K> c;
        load_chunk<A, K, false>(c, b, P, g);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        if (rec) out[1] = now();
        const uint32_t vo = g * 4u;
        uint32_t T0 = c.wt.x, T1 = c.wt.y;
        uint32_t pending = ocsw::at_done80<K, MODE>(L.sw, c.wl);
        const int64_t rem = L.B - (int64_t)g * kEPL;
        const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (1u << (8 * (uint32_t)rem)) - 1u);
        for (int r = 0; r < n; ++r) {
            uint32_t act[A], ex[A], cm;
            if (NOLOAD) {
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    uint32_t h = g * 0x9E3779B1u ^ (uint32_t)r * 0x85EBCA6Bu ^ (uint32_t)(a + 1) * 0xC2B2AE35u;
                    h ^= h >> 15;
                    h *= 0x2C1B3C6Du;
                    h ^= h >> 12;
                    act[a] = ((h & 0xFFu) % 5u) | (((h >> 8) & 0xFFu) % 5u) << 8 | (((h >> 16) & 0xFFu) % 5u) << 16 |
                             ((h >> 24) % 5u) << 24;
                }
            } else {
                const int q = r % kLwSteps;
                if (q == 0) lds_barrier();
                const int h = (r / kLwSteps) & 1;
#pragma unroll
                for (int a = 0; a < A; ++a)
                    act[a] = ring[(((h * kLwSteps + q) * SW + (threadIdx.x >> 6)) * A + a) * 64 + lane];
            }
            if (rec) {
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the ring words have landed
                out[2 + 3 * r] = now();
            }
            const uint32_t f_in = c.wf;
            const bool full = ocsw::step4<A, K, MODE>(L.sw, c.wx, c.wy, c.wh, c.wl, c.wm, T0, T1, c.wf, act, ex,
                                                      cm, cls_of, WaveAny{}, pending);
            st.coll += __popc(cm & vmask);
            if (full) {
                const uint32_t ended = (c.wf & ~f_in & vmask) & ocsw::k01;
                st.eps += __popc(ended);
            }
            if (rec) out[3 + 3 * r] = now();
            const uint32_t base = live ? (uint32_t)r * NP * P : 0x7FFFFFFFu;  // past num_records: dropped
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
            for (int a = 0; a < A; ++a) bst32<CP>(b.ex, ex[a], vo, live ? (uint32_t)(r * A + a) * P : 0x7FFFFFFFu);
            bst32<CP>(b.coll, cm, vo, live ? (uint32_t)r * P : 0x7FFFFFFFu);
            if (rec) out[4 + 3 * r] = now();
        }
        if (LW) lds_barrier();
        if (!live) continue;
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
    if (rec) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        out[2 + 3 * kMaxSteps] = now();  // every store acknowledged
    }
    if (st.coll == 0xFFFFFFFFu) tl[0] = st.eps;  // keep the statistics live
}


// Round 6: the loader-wave form with the work handed out dynamically.  A work
// item is (chunk of the block's 1,024 envs, segment of SEG steps); items are taken from a
// per-launch atomic queue in segment-major order by a grid of co-resident blocks, so a block
// that finishes early takes more work and no block starts in a second residency round.  A
// chunk's segment k > 0 continues from the state its segment k - 1 left in the trajectory
// slot k*SEG - 1: that step's stores are sc1 (write-through), the producing block's waves wait
// vmcnt(0), meet at a barrier, and one lane stores the chunk's flag (sc1); the consuming
// block's thread 0 polls the flag with sc1 loads, the block meets at a barrier and loads the
// state with sc1 loads (MI355X_MICROARCH.md "Valid forms", row 1).  The last segment resets
// the flag, the last block out resets the queue, so every launch starts from zeros.
template <int A, int K, int MODE, int SEG>
__global__ __launch_bounds__(5 * 64, 5) void stepn_seg(LevelArgs L, const uint8_t* __restrict__ sin,
                                                        uint8_t* __restrict__ sout,
                                                        const uint8_t* __restrict__ actions,
                                                        uint8_t* __restrict__ traj,
                                                        uint8_t* __restrict__ exec_out,
                                                        uint8_t* __restrict__ coll_out, int n,
                                                        uint32_t* __restrict__ q, uint32_t* __restrict__ flags) {
    constexpr int CP = kCPnt, SW = 4, kBS = SW * 64;
    __shared__ uint32_t tbl4[64];
    __shared__ uint32_t ring[2 * kLwSteps * SW * A * 64];
    __shared__ uint32_t item_s;
    if (threadIdx.x < 64u) tbl4[threadIdx.x] = L.cls4[threadIdx.x];
    __syncthreads();
    const bool loader = threadIdx.x >= (uint32_t)kBS;
    const uint32_t lane = threadIdx.x & 63u;
    const uint8_t* tbl = (const uint8_t*)tbl4;
    const uint32_t P = (uint32_t)L.pitch, nlanes = P / kEPL;
    constexpr int NP = 3 * A + 2 * K + 3;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    auto cls_of = [&](uint32_t cells) -> uint32_t {
        const uint32_t b0 = tbl[cells & 0xFFu], b1 = tbl[(cells >> 8) & 0xFFu], b2 = tbl[(cells >> 16) & 0xFFu],
                       b3 = tbl[cells >> 24];
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    };
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(sin, (int64_t)NP * P), rout = make_rsrc(sout, (int64_t)NP * P);
    const __amdgpu_buffer_rsrc_t ract = make_rsrc(actions, (int64_t)n * A * P);
    const __amdgpu_buffer_rsrc_t tr = make_rsrc(traj, (int64_t)n * NP * P);
    const __amdgpu_buffer_rsrc_t rex = make_rsrc(exec_out, (int64_t)n * A * P), rco = make_rsrc(coll_out, (int64_t)n * P);
    const uint32_t nchunks = nlanes / (uint32_t)kBS, nseg = (uint32_t)((n + SEG - 1) / SEG), total = nchunks * nseg;
    StepStats st;
    typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
    for (;;) {
        if (threadIdx.x == 0u) {
            const uint32_t it = atomicAdd(q, 1u);
            if (it < total && it >= nchunks) {  // segment k > 0: wait for the chunk's segment k - 1
                const uint32_t c = it % nchunks, k = it / nchunks;
                while (__hip_atomic_load(flags + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != k)
                    __builtin_amdgcn_s_sleep(2);
            }
            item_s = it;
        }
        lds_barrier();
        const uint32_t it = item_s;
        if (it >= total) break;
        const uint32_t c = it % nchunks, k = it / nchunks;
        const int r0 = (int)k * SEG, r1 = min(n, r0 + SEG);
        const uint32_t gb = c * (uint32_t)kBS;
        if (loader) {
            auto fill = [&](int rb, int h) {
                uint32_t w[kLwSteps][SW][A];
#pragma unroll
                for (int qq = 0; qq < kLwSteps; ++qq)
#pragma unroll
                    for (int v = 0; v < SW; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            w[qq][v][a] = rb + qq < r1 ? bld32<0>(ract, (gb + 64u * v + lane) * 4u,
                                                                   (uint32_t)((rb + qq) * A + a) * P)
                                                       : 0u;
#pragma unroll
                for (int qq = 0; qq < kLwSteps; ++qq)
#pragma unroll
                    for (int v = 0; v < SW; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            ring[(((h * kLwSteps + qq) * SW + v) * A + a) * 64 + lane] = w[qq][v][a];
            };
            fill(r0, 0);
            for (int rb = r0; rb < r1; rb += kLwSteps) {
                lds_barrier();
                if (rb + kLwSteps < r1) fill(rb + kLwSteps, (((rb - r0) / kLwSteps) & 1) ^ 1);
            }
            lds_barrier();  // the item's last batch has been read
            lds_barrier();  // the stepping waves' stores drained (segment end)
            continue;
        }
        const uint32_t g = gb + threadIdx.x, vo = g * 4u;
        // the state: the batch's input (segment 0) or the slot segment k - 1 left (sc1 loads)
        Chunk<A, K> ch;
        {
            const __amdgpu_buffer_rsrc_t rs = k == 0u ? rin : tr;
            const uint32_t base = k == 0u ? 0u : (uint32_t)(r0 - 1) * NP * P;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                ch.wx[a] = bld32<kCPsc1>(rs, vo, base + a * P);
                ch.wy[a] = bld32<kCPsc1>(rs, vo, base + (kPY + a) * P);
                ch.wh[a] = bld32<kCPsc1>(rs, vo, base + (kPH + a) * P);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                ch.wl[j] = bld32<kCPsc1>(rs, vo, base + (kPL + j) * P);
                ch.wm[j] = bld32<kCPsc1>(rs, vo, base + (kPM + j) * P);
            }
            const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(g * 8u), (int)(base + kPT * P), kCPsc1);
            ch.wt = make_uint2(t[0], t[1]);
            ch.wf = bld32<kCPsc1>(rs, vo, base + kPF * P);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        uint32_t T0 = ch.wt.x, T1 = ch.wt.y;
        uint32_t pending = ocsw::at_done80<K, MODE>(L.sw, ch.wl);
        const int64_t rem = L.B - (int64_t)g * kEPL;
        const uint32_t vmask = rem >= kEPL ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (1u << (8 * (uint32_t)rem)) - 1u);
        for (int r = r0; r < r1; ++r) {
            uint32_t act[A], ex[A], cm;
            const int qq = (r - r0) % kLwSteps;
            if (qq == 0) lds_barrier();
            const int h = ((r - r0) / kLwSteps) & 1;
#pragma unroll
            for (int a = 0; a < A; ++a) act[a] = ring[(((h * kLwSteps + qq) * SW + (threadIdx.x >> 6)) * A + a) * 64 + lane];
            const uint32_t f_in = ch.wf;
            const bool full = ocsw::step4<A, K, MODE>(L.sw, ch.wx, ch.wy, ch.wh, ch.wl, ch.wm, T0, T1, ch.wf, act, ex,
                                                      cm, cls_of, WaveAny{}, pending);
            st.coll += __popc(cm & vmask);
            if (full) {
                const uint32_t ended = (ch.wf & ~f_in & vmask) & ocsw::k01;
                st.eps += __popc(ended);
            }
            const uint32_t base = (uint32_t)r * NP * P;
            auto store_state = [&](auto pol) {
                constexpr int PC = decltype(pol)::value;
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    bst32<PC>(tr, ch.wx[a], vo, base + a * P);
                    bst32<PC>(tr, ch.wy[a], vo, base + (kPY + a) * P);
                    bst32<PC>(tr, ch.wh[a], vo, base + (kPH + a) * P);
                }
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    bst32<PC>(tr, ch.wl[j], vo, base + (kPL + j) * P);
                    bst32<PC>(tr, ch.wm[j], vo, base + (kPM + j) * P);
                }
                const u32x2 tw = {T0, T1};
                __builtin_amdgcn_raw_buffer_store_b64(tw, tr, (int)(g * 8u), (int)(base + kPT * P), PC);
                bst32<PC>(tr, ch.wf, vo, base + kPF * P);
            };
            if (r + 1 == r1 && r1 < n) store_state(std::integral_constant<int, kCPsc1>{});  // the hand-off slot
            else store_state(std::integral_constant<int, CP>{});
#pragma unroll
            for (int a = 0; a < A; ++a) bst32<CP>(rex, ex[a], vo, (uint32_t)(r * A + a) * P);
            bst32<CP>(rco, cm, vo, (uint32_t)r * P);
        }
        lds_barrier();  // pairs with the loader's end-of-item barrier
        if (r1 == n) {
#pragma unroll
            for (int a = 0; a < A; ++a) {
                bst32<CP>(rout, ch.wx[a], vo, a * P);
                bst32<CP>(rout, ch.wy[a], vo, (kPY + a) * P);
                bst32<CP>(rout, ch.wh[a], vo, (kPH + a) * P);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                bst32<CP>(rout, ch.wl[j], vo, (kPL + j) * P);
                bst32<CP>(rout, ch.wm[j], vo, (kPM + j) * P);
            }
            const u32x2 tw = {T0, T1};
            __builtin_amdgcn_raw_buffer_store_b64(tw, rout, (int)(g * 8u), (int)(kPT * P), CP);
            bst32<CP>(rout, ch.wf, vo, kPF * P);
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's hand-off stores are done
        }
        lds_barrier();  // every stepping wave's stores drained
        if (threadIdx.x == 0u)
            __hip_atomic_store(flags + c, r1 == n ? 0u : k + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the last block out resets the queue for the next launch
    if (threadIdx.x == 0u && atomicAdd(q + 1, 1u) == gridDim.x - 1u) {
        __hip_atomic_store(q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (st.coll == 0xFFFFFFFFu) flags[0] = st.eps;  // keep the statistics live
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t B = 1 << 20;
    const int n = kMaxSteps;
    // full-divider_tl's oc_level_desc, written by capi.level_desc (tools/gpu_r5*.sh)
    oc_level_desc lv{};
    FILE* f = fopen(argc > 1 ? argv[1] : "gpurun_out/c3_level.bin", "rb");
    if (f == nullptr || fread(&lv, sizeof lv, 1, f) != 1) { printf("level file\n"); return 1; }
    fclose(f);
    oc_handle* h;
    if (oc_create(&lv, 3, 100, 0, &h) != 0) { printf("create: %s\n", oc_last_error()); return 1; }
    oc_layout lay;
    oc_get_layout(h, B, &lay);
    const int64_t S = lay.state_bytes, P = lay.pitch;
    uint8_t *s0, *acts, *traj, *ex, *coll, *sout;
    uint64_t* tl;
    const int64_t nlanes = P / kEPL, nstep_waves = nlanes / 64, nrec = nstep_waves / kSample;
    const int64_t rec_words = 3 * kMaxSteps + 3;
    CK(hipMalloc(&s0, S)); CK(hipMalloc(&sout, S)); CK(hipMalloc(&acts, (int64_t)n * 3 * P));
    CK(hipMalloc(&traj, (int64_t)n * S)); CK(hipMalloc(&ex, (int64_t)n * 3 * P)); CK(hipMalloc(&coll, (int64_t)n * P));
    CK(hipMalloc(&tl, (nrec + 8) * rec_words * 8));
    // mid-run start state: 1,050 steps from a reset
    uint8_t* s1;
    CK(hipMalloc(&s1, S));
    oc_reset(h, s0, B, nullptr);
    for (int r = 0; r < 1050; ++r) {
        oc_gen_actions(h, acts, B, 0, r, 3, nullptr);
        oc_step(h, r & 1 ? s1 : s0, r & 1 ? s0 : s1, acts, nullptr, nullptr, nullptr, B, nullptr);
    }
    for (int r = 0; r < n; ++r) oc_gen_actions(h, acts + (int64_t)r * 3 * P, B, 0, 5000 + r, 3, nullptr);
    CK(hipDeviceSynchronize());
    LevelArgs L = h->args;
    L.pitch = P;
    L.B = B;
    const int64_t need = P / kEnvsPerBlock;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto launch = [&](auto kern, bool lw, int sw = 4, int per_cu = 0) {
        const int64_t lanes_pb = 64 * sw, blocks = (nlanes + lanes_pb - 1) / lanes_pb;
        const int64_t cap = (int64_t)h->cus * (per_cu ? per_cu : (lw ? 4 : 5));
        hipLaunchKernelGGL(kern, dim3((unsigned)(blocks < cap ? blocks : cap)), dim3(64 * sw + (lw ? 64 : 0)), 0, nullptr,
                           L, s0, sout, acts, traj, ex, coll, n, tl);
    };
    auto time = [&](const char* name, auto kern, bool lw, int sw = 4, int per_cu = 0) {
        for (int i = 0; i < 3; ++i) launch(kern, lw, sw, per_cu);
        CK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) launch(kern, lw, sw, per_cu);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.3f us/step  (%.1f us per 100-step launch)\n", name, ms * 1e3 / 10 / n, ms * 1e3 / 10);
    };
    auto report = [&](const char* name) {
        std::vector<uint64_t> v(nrec * rec_words);
        CK(hipMemcpy(v.data(), tl, v.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull;
        for (int64_t w = 0; w < nrec; ++w) t0 = std::min(t0, v[w * rec_words]);
        std::vector<double> start, loaded, wait, comp, store, total, end, at50;
        for (int64_t w = 0; w < nrec; ++w) {
            const uint64_t* o = v.data() + w * rec_words;
            start.push_back((o[0] - t0) * 0.01);
            loaded.push_back((o[1] - o[0]) * 0.01);
            for (int r = 0; r < n; ++r) {
                const uint64_t s = o[2 + 3 * r], c = o[3 + 3 * r], st = o[4 + 3 * r];
                const uint64_t prev = r == 0 ? o[1] : o[4 + 3 * (r - 1)];
                wait.push_back((s - prev) * 0.01);
                comp.push_back((c - s) * 0.01);
                store.push_back((st - c) * 0.01);
            }
            total.push_back((o[4 + 3 * (n - 1)] - o[1]) * 0.01 / n);
            end.push_back((o[2 + 3 * kMaxSteps] - t0) * 0.01);
            at50.push_back((o[2 + 3 * 50] - t0) * 0.01);
        }
        auto pr = [](const char* what, std::vector<double>& x) {
            std::sort(x.begin(), x.end());
            double sum = 0;
            for (double d : x) sum += d;
            printf("    %-34s mean %7.3f  p10 %7.3f  p50 %7.3f  p90 %7.3f  max %7.3f\n", what, sum / x.size(),
                   x[x.size() / 10], x[x.size() / 2], x[x.size() * 9 / 10], x.back());
        };
        printf("  timeline %s: %lld sampled waves (us; 100 MHz wall clock)\n", name, (long long)nrec);
        pr("wave start (from the first)", start);
        pr("state loads landed", loaded);
        pr("per step: wait before compute", wait);
        pr("per step: compute (step4)", comp);
        pr("per step: store issue", store);
        pr("per step: all (loop / n)", total);
        pr("step 50 start (from the first wave)", at50);
        pr("all stores acked (from the first)", end);
    };
    time("lw (product form)", stepn_tl<3, 4, 0, true, false, false>, true);
    time("lw + stamps", stepn_tl<3, 4, 0, true, false, true>, true);
    report("lw");
    CK(hipMemset(tl, 0, nrec * rec_words * 8));
    time("lw, 3 stepping waves + loader per block", stepn_tl<3, 4, 0, true, false, false, 3, 5>, true, 3, 5);
    time("lw3 + stamps", stepn_tl<3, 4, 0, true, false, true, 3, 5>, true, 3, 5);
    report("lw3");
    time("lw, launch bounds 6 waves per SIMD", stepn_tl<3, 4, 0, true, false, false, 4, 6>, true);
    time("lw6 + stamps", stepn_tl<3, 4, 0, true, false, true, 4, 6>, true);
    report("lw6");
    time("noload (no loads, no barrier)", stepn_tl<3, 4, 0, false, true, false>, false);
    time("noload + stamps", stepn_tl<3, 4, 0, false, true, true>, false);
    report("noload");
    // round 6: the dynamic (chunk, segment) queue; outputs compared with the product form's
    uint32_t* qf;
    CK(hipMalloc(&qf, (2 + nlanes / 256) * 4));
    CK(hipMemset(qf, 0, (2 + nlanes / 256) * 4));
    std::vector<uint8_t> ref_traj((size_t)n * S), got((size_t)n * S), ref_ex((size_t)n * 3 * P), got_ex((size_t)n * 3 * P);
    launch(stepn_tl<3, 4, 0, true, false, false>, true);
    CK(hipMemcpy(ref_traj.data(), traj, ref_traj.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref_ex.data(), ex, ref_ex.size(), hipMemcpyDeviceToHost));
    auto seg = [&](const char* name, auto kern, int per_cu) {
        auto go = [&]() {
            hipLaunchKernelGGL(kern, dim3((unsigned)(h->cus * per_cu)), dim3(320), 0, nullptr, L, s0, sout, acts, traj, ex,
                               coll, n, qf, qf + 2);
        };
        CK(hipMemset(traj, 0, (size_t)n * S));
        go();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), traj, got.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(got_ex.data(), ex, got_ex.size(), hipMemcpyDeviceToHost));
        const bool same = got == ref_traj && got_ex == ref_ex;
        for (int i = 0; i < 3; ++i) go();
        CK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) go();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(got.data(), traj, got.size(), hipMemcpyDeviceToHost));
        const bool same2 = got == ref_traj;
        printf("%-44s %8.3f us/step  outputs %s\n", name, ms * 1e3 / 10 / n,
               same && same2 ? "identical to lw" : "DIFFER from lw");
    };
    if (getenv("C3TL_SEG")) {  // pass A of round 6 (profiles/r06/pass_a/c3tl.log)
        seg("seg 20 steps, 3 blocks/CU", stepn_seg<3, 4, 0, 20>, 3);
        seg("seg 20 steps, 4 blocks/CU", stepn_seg<3, 4, 0, 20>, 4);
        seg("seg 10 steps, 3 blocks/CU", stepn_seg<3, 4, 0, 10>, 3);
        seg("seg 25 steps, 3 blocks/CU", stepn_seg<3, 4, 0, 25>, 3);
        seg("seg 50 steps, 3 blocks/CU", stepn_seg<3, 4, 0, 50>, 3);
        seg("seg 100 steps (queue only), 3 blocks/CU", stepn_seg<3, 4, 0, 100>, 3);
    }
    // round 6, pass C: blocks of more stepping waves per loader (fewer loader waves, and at 8
    // stepping waves every block of a 2^20-env launch is resident at once: 512 blocks of 9 waves,
    // two per CU), against the product form, alternating
    for (int rep = 0; rep < 3; ++rep) {
        time("lw (product form)", stepn_tl<3, 4, 0, true, false, false>, true);
        time("lw, 8 stepping waves + loader, 2 blocks/CU", stepn_tl<3, 4, 0, true, false, false, 8, 2>, true, 8, 2);
        time("lw, 6 stepping waves + loader, 3 blocks/CU", stepn_tl<3, 4, 0, true, false, false, 6, 3>, true, 6, 3);
        time("lw, launch bounds 6 waves per SIMD", stepn_tl<3, 4, 0, true, false, false, 4, 6>, true);
    }
    time("lw8 + stamps", stepn_tl<3, 4, 0, true, false, true, 8, 2>, true, 8, 2);
    report("lw8");
    // the product launch, for reference (C-ABI, with the statistics)
    uint64_t* stats;
    int64_t nb;
    oc_stats_size(h, B, &nb);
    CK(hipMalloc(&stats, nb));
    CK(hipMemset(stats, 0, nb));
    for (int i = 0; i < 3; ++i) oc_step_n(h, s0, traj + (int64_t)(n - 1) * S, acts, traj, ex, coll, stats, nullptr, B, n, nullptr);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) oc_step_n(h, s0, traj + (int64_t)(n - 1) * S, acts, traj, ex, coll, stats, nullptr, B, n, nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s %8.3f us/step\n", "product oc_step_n (C-ABI)", ms * 1e3 / 10 / n);
    return 0;
}
