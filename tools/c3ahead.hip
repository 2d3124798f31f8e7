// tools/c3ahead.hip -- round 6: can C3's stepping waves prefetch their own action words without
// the loader wave?    Standalone: it includes only the
// SWAR step (oc_swar.h), so it builds in seconds, not the engine's minutes.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o tools/c3ahead tools/c3ahead.hip
// Run:   tools/c3ahead LEVEL.bin   (full-divider_tl's oc_level_desc, written by capi.level_desc)
// Workload: bench.py's C3 -- 3 agents, 2^20 envs, 100-step launches, every step's state,
// executed actions and collision mask written with nt stores, from a mid-run state.
// Variants of oc_step_n_kernel's stepping loop, outputs compared byte for byte with the first:
//   lw         the product's form: a fifth wave per block loads 4 steps of actions into an LDS
//              ring, an LDS barrier every 4 steps
//   ahead_c<D> each stepping wave loads its action words D steps ahead (compiler-visible loads:
//              the compiler's waitcnt pass places the wait)
//   ahead_a<D> the same with inline-asm loads and a hand-counted s_waitcnt vmcnt((D-1) x (the
//              step's 23 stores + 3 loads)): loads and stores share vmcnt in issue order, so the
//              wait covers exactly the words needed and the stores older than them
//   noload     actions hashed in-kernel: no action load at all (a floor)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/oc_engine.h"
#include "../gym-cooking_amd/csrc/oc_swar.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

constexpr int A = 3, K = 4, NP = 3 * A + 2 * K + 3, kEPL = 4;
constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
constexpr int kStores = 4 * A + 2 * K + 3;  // per step: state planes (t as one b64), exec, coll
constexpr int kLw = 4;

struct Args {
    ocsw::SwarLevel sw;
    uint32_t cls4[64];
    uint32_t P;
    int n;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, (int)so, 0);
}
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t vo, uint32_t so) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)vo, (int)so, 2 /* nt */);
}
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
struct WaveAny {
    __device__ __forceinline__ bool operator()(uint32_t v) const { return __ballot(v != 0u) != 0ull; }
};

struct State {
    uint32_t x[A], y[A], h[A], l[K], m[K], t0, t1, f;
};

__device__ __forceinline__ void load_state(State& s, __amdgpu_buffer_rsrc_t r, uint32_t P, uint32_t g) {
    const uint32_t vo = g * 4u;
#pragma unroll
    for (int a = 0; a < A; ++a) {
        s.x[a] = ld(r, vo, a * P);
        s.y[a] = ld(r, vo, (kPY + a) * P);
        s.h[a] = ld(r, vo, (kPH + a) * P);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        s.l[j] = ld(r, vo, (kPL + j) * P);
        s.m[j] = ld(r, vo, (kPM + j) * P);
    }
    const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(g * 8u), (int)(kPT * P), 0);
    s.t0 = t[0];
    s.t1 = t[1];
    s.f = ld(r, vo, kPF * P);
}

// one step of the lane's chunk and its kStores stores
template <class ClsOf>
__device__ __forceinline__ void step_store(const Args& R, State& s, const uint32_t (&act)[A], uint32_t& pending,
                                           ClsOf cls_of, __amdgpu_buffer_rsrc_t tr, __amdgpu_buffer_rsrc_t ex,
                                           __amdgpu_buffer_rsrc_t co, uint32_t g, int r) {
    typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
    const uint32_t P = R.P, vo = g * 4u;
    uint32_t e[A], cm;
    ocsw::step4<A, K, 0>(R.sw, s.x, s.y, s.h, s.l, s.m, s.t0, s.t1, s.f, act, e, cm, cls_of, WaveAny{}, pending);
    const uint32_t base = (uint32_t)r * NP * P;
#pragma unroll
    for (int a = 0; a < A; ++a) {
        st(tr, s.x[a], vo, base + a * P);
        st(tr, s.y[a], vo, base + (kPY + a) * P);
        st(tr, s.h[a], vo, base + (kPH + a) * P);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        st(tr, s.l[j], vo, base + (kPL + j) * P);
        st(tr, s.m[j], vo, base + (kPM + j) * P);
    }
    const u32x2 tw = {s.t0, s.t1};
    __builtin_amdgcn_raw_buffer_store_b64(tw, tr, (int)(g * 8u), (int)(base + kPT * P), 2);
    st(tr, s.f, vo, base + kPF * P);
#pragma unroll
    for (int a = 0; a < A; ++a) st(ex, e[a], vo, (uint32_t)(r * A + a) * P);
    st(co, cm, vo, (uint32_t)r * P);
}

#define TABLE_SETUP                                                                                 \
    __shared__ uint32_t tbl4[64];                                                                   \
    if (threadIdx.x < 64u) tbl4[threadIdx.x] = R.cls4[threadIdx.x];                                 \
    __syncthreads();                                                                                \
    const uint8_t* tbl = (const uint8_t*)tbl4;                                                      \
    auto cls_of = [&](uint32_t c) -> uint32_t {                                                     \
        return (uint32_t)tbl[c & 0xFFu] | ((uint32_t)tbl[(c >> 8) & 0xFFu] << 8) |                  \
               ((uint32_t)tbl[(c >> 16) & 0xFFu] << 16) | ((uint32_t)tbl[c >> 24] << 24);           \
    };                                                                                              \
    const uint32_t P = R.P, nlanes = P / kEPL;                                                      \
    const int n = R.n;                                                                              \
    const auto rin = rsrc(sin, (int64_t)NP * P), ra = rsrc(acts, (int64_t)n * A * P);               \
    const auto tr = rsrc(traj, (int64_t)n * NP * P), rex = rsrc(exo, (int64_t)n * A * P);           \
    const auto rco = rsrc(coll, (int64_t)n * P);

// the product's loader-wave form (oc_step_n_kernel with LW), 4 stepping waves + 1 loader
__global__ __launch_bounds__(320, 5) void k_lw(Args R, const uint8_t* sin, const uint8_t* acts, uint8_t* traj,
                                               uint8_t* exo, uint8_t* coll) {
    TABLE_SETUP
    __shared__ uint32_t ring[2 * kLw * 4 * A * 64];
    const bool loader = threadIdx.x >= 256u;
    const uint32_t lane = threadIdx.x & 63u, stride = gridDim.x * 256u;
    for (uint32_t gb = blockIdx.x * 256u; gb < nlanes; gb += stride) {
        if (loader) {
            auto fill = [&](int r0, int hh) {
                uint32_t w[kLw][4][A];
#pragma unroll
                for (int q = 0; q < kLw; ++q)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a)
                            w[q][v][a] = r0 + q < n ? ld(ra, (gb + 64u * v + lane) * 4u, (uint32_t)((r0 + q) * A + a) * P) : 0u;
#pragma unroll
                for (int q = 0; q < kLw; ++q)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
#pragma unroll
                        for (int a = 0; a < A; ++a) ring[(((hh * kLw + q) * 4 + v) * A + a) * 64 + lane] = w[q][v][a];
            };
            fill(0, 0);
            for (int r0 = 0; r0 < n; r0 += kLw) {
                lds_barrier();
                if (r0 + kLw < n) fill(r0 + kLw, ((r0 / kLw) & 1) ^ 1);
            }
            lds_barrier();
            continue;
        }
        const uint32_t g = gb + threadIdx.x;
        State s;
        load_state(s, rin, P, g);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        uint32_t pending = ocsw::at_done80<K, 0>(R.sw, s.l);
        for (int r = 0; r < n; ++r) {
            const int q = r % kLw;
            if (q == 0) lds_barrier();
            const int hh = (r / kLw) & 1;
            uint32_t act[A];
#pragma unroll
            for (int a = 0; a < A; ++a) act[a] = ring[(((hh * kLw + q) * 4 + (threadIdx.x >> 6)) * A + a) * 64 + lane];
            step_store(R, s, act, pending, cls_of, tr, rex, rco, g, r);
        }
        lds_barrier();
    }
}

// compiler-visible prefetch, D steps ahead (a register ring rotated every step)
template <int D>
__global__ __launch_bounds__(256, 1) void k_ahead_c(Args R, const uint8_t* sin, const uint8_t* acts, uint8_t* traj,
                                                    uint8_t* exo, uint8_t* coll) {
    TABLE_SETUP
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nlanes; g += stride) {
        const uint32_t vo = g * 4u;
        State s;
        load_state(s, rin, P, g);
        uint32_t ringv[D][A];
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int a = 0; a < A; ++a) ringv[d][a] = ld(ra, vo, (uint32_t)(min(d, n - 1) * A + a) * P);
        uint32_t pending = ocsw::at_done80<K, 0>(R.sw, s.l);
        for (int r = 0; r < n; ++r) {
            uint32_t act[A];
#pragma unroll
            for (int a = 0; a < A; ++a) act[a] = ringv[0][a];
#pragma unroll
            for (int d = 0; d + 1 < D; ++d)
#pragma unroll
                for (int a = 0; a < A; ++a) ringv[d][a] = ringv[d + 1][a];
            const int rn = min(r + D, n - 1);
#pragma unroll
            for (int a = 0; a < A; ++a) ringv[D - 1][a] = ld(ra, vo, (uint32_t)(rn * A + a) * P);
            step_store(R, s, act, pending, cls_of, tr, rex, rco, g, r);
        }
    }
}

// inline-asm prefetch, D steps ahead: the loop is unrolled by D so that ring slot u is always
// the same variable (a register the asm load writes asynchronously; nothing reads it before the
// hand-counted wait, which names it as an operand)
template <int D>
__global__ __launch_bounds__(256, 1) void k_ahead_a(Args R, const uint8_t* sin, const uint8_t* acts, uint8_t* traj,
                                                    uint8_t* exo, uint8_t* coll) {
    TABLE_SETUP
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nlanes; g += stride) {
        const uint32_t vo = g * 4u;
        State s;
        load_state(s, rin, P, g);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // the state (compiler-visible loads) before the asm loads
        uint32_t ringv[D][A];
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int a = 0; a < A; ++a) {
                const uint32_t so = (uint32_t)(min(d, n - 1) * A + a) * P;
                asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(ringv[d][a]) : "v"(vo), "s"(ra), "s"(so) : "memory");
            }
        uint32_t pending = ocsw::at_done80<K, 0>(R.sw, s.l);
        for (int r0 = 0; r0 < n; r0 += D) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
                const int r = r0 + u;
                if (r >= n) break;  // n is a multiple of D in this harness
                // slot u's A loads were issued D steps ago; younger: (D - 1) steps of stores + loads
                static_assert((D - 1) * (kStores + A) <= 63, "vmcnt holds 63");
                if constexpr (A == 3)
                    asm volatile("s_waitcnt vmcnt(%3)" : "+v"(ringv[u][0]), "+v"(ringv[u][1]), "+v"(ringv[u][2])
                                 : "n"((D - 1) * (kStores + A)) : "memory");
                uint32_t act[A];
#pragma unroll
                for (int a = 0; a < A; ++a) act[a] = ringv[u][a];
                step_store(R, s, act, pending, cls_of, tr, rex, rco, g, r);
                const int rn = min(r + D, n - 1);
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    const uint32_t so = (uint32_t)(rn * A + a) * P;
                    asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(ringv[u][a]) : "v"(vo), "s"(ra), "s"(so) : "memory");
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last prefetches land before the registers are reused
    }
}

__global__ __launch_bounds__(256, 1) void k_noload(Args R, const uint8_t* sin, const uint8_t* acts, uint8_t* traj,
                                                   uint8_t* exo, uint8_t* coll) {
    TABLE_SETUP
    (void)ra;
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < nlanes; g += stride) {
        State s;
        load_state(s, rin, P, g);
        uint32_t pending = ocsw::at_done80<K, 0>(R.sw, s.l);
        for (int r = 0; r < n; ++r) {
            uint32_t act[A];
#pragma unroll
            for (int a = 0; a < A; ++a) {
                uint32_t h = g * 0x9E3779B1u ^ (uint32_t)r * 0x85EBCA6Bu ^ (uint32_t)(a + 1) * 0xC2B2AE35u;
                h ^= h >> 15;
                h *= 0x2C1B3C6Du;
                h ^= h >> 12;
                act[a] = h & 0x03030303u;
            }
            step_store(R, s, act, pending, cls_of, tr, rex, rco, g, r);
        }
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t B = 1 << 20, P = B;
    const int n = 96;  // a multiple of 2, 3 and 4
    oc_level_desc lv{};
    FILE* f = fopen(argc > 1 ? argv[1] : "gpurun_out/c3_level.bin", "rb");
    if (f == nullptr || fread(&lv, sizeof lv, 1, f) != 1) { printf("level file\n"); return 1; }
    fclose(f);
    const int W = lv.width, H = lv.height;
    Args R{};
    uint8_t cell[16], mask[16];
    for (int j = 0; j < 16; ++j) {
        cell[j] = j < lv.num_items ? (uint8_t)lv.item_cell[j] : 0xFF;
        mask[j] = j < lv.num_items ? lv.item_mask[j] : 0;
    }
    int done_cell = -1;
    for (int c = 0; c < W * H; ++c) {
        R.cls4[c >> 2] |= (uint32_t)ocsw::tile_class(lv.tiles[c]) << (8 * (c & 3));
        if (lv.tiles[c] == OC_TILE_DELIVERY && done_cell < 0) done_cell = c;
    }
    ocsw::build_swar_level(R.sw, W, H, done_cell, lv.goal_mask, lv.num_goals, 100, lv.spawn_x, lv.spawn_y, A, cell,
                           mask, lv.encoding, lv.tiles);
    R.P = (uint32_t)P;
    R.n = n;
    // the template state, then 1,050 steps of the lw form from it (a mid-run state)
    std::vector<uint8_t> s0((size_t)NP * P, 0);
    for (int a = 0; a < A; ++a) {
        memset(&s0[(size_t)a * P], lv.spawn_x[a], P);
        memset(&s0[(size_t)(kPY + a) * P], lv.spawn_y[a], P);
        memset(&s0[(size_t)(kPH + a) * P], 0xFF, P);
    }
    for (int j = 0; j < K; ++j) {
        memset(&s0[(size_t)(kPL + j) * P], cell[j], P);
        memset(&s0[(size_t)(kPM + j) * P], mask[j], P);
    }
    std::vector<uint8_t> ah((size_t)n * A * P);
    uint64_t x = 88172645463325252ull;
    for (auto& v : ah) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = (uint8_t)(x % 5);
    }
    uint8_t *sin, *acts, *traj, *exo, *coll;
    CK(hipMalloc(&sin, (size_t)NP * P)); CK(hipMalloc(&acts, ah.size()));
    CK(hipMalloc(&traj, (size_t)n * NP * P)); CK(hipMalloc(&exo, (size_t)n * A * P)); CK(hipMalloc(&coll, (size_t)n * P));
    CK(hipMemcpy(sin, s0.data(), s0.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(acts, ah.data(), ah.size(), hipMemcpyHostToDevice));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned blocks = (unsigned)(P / kEPL / 256);
    for (int i = 0; i < 11; ++i) {  // mid-run: 11 x 96 steps from the template
        hipLaunchKernelGGL(k_lw, dim3(std::min<unsigned>(blocks, cus * 4)), dim3(320), 0, nullptr, R, sin, acts, traj, exo, coll);
        CK(hipMemcpy(sin, traj + (size_t)(n - 1) * NP * P, (size_t)NP * P, hipMemcpyDeviceToDevice));
    }
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> ref_t((size_t)n * NP * P), ref_e((size_t)n * A * P), got_t(ref_t.size()), got_e(ref_e.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kern, unsigned grid, unsigned threads, bool reference) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, nullptr, R, sin, acts, traj, exo, coll);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got_t.data(), traj, got_t.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(got_e.data(), exo, got_e.size(), hipMemcpyDeviceToHost));
        if (reference) { ref_t = got_t; ref_e = got_e; }
        const bool same = got_t == ref_t && got_e == ref_e;
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, nullptr, R, sin, acts, traj, exo, coll);
        CK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, nullptr, R, sin, acts, traj, exo, coll);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 10 / n, bytes = (double)NP / n + NP + 2 * A + 1;
        printf("%-40s %7.3f us/step  frac %.3f  outputs %s\n", name, us, bytes * B / (us * 1e-6) / 8e12,
               reference ? "(reference)" : same ? "identical" : "DIFFER");
        fflush(stdout);
    };
    const unsigned lwg = std::min<unsigned>(blocks, cus * 4), g5 = std::min<unsigned>(blocks, cus * 5);
    for (int rep = 0; rep < 3; ++rep) {
        run("lw (product form)", k_lw, lwg, 320, rep == 0);
        run("ahead_c<2> (compiler waits)", k_ahead_c<2>, g5, 256, false);
        run("ahead_c<3>", k_ahead_c<3>, g5, 256, false);
        run("ahead_a<2> (asm loads, vmcnt(26))", k_ahead_a<2>, g5, 256, false);
        run("ahead_a<3> (asm loads, vmcnt(52))", k_ahead_a<3>, g5, 256, false);
        run("noload (actions hashed: a floor)", k_noload, g5, 256, false);
    }
    return 0;
}
