// tools/stepnexp.hip -- oc_step_n launch-shape experiment (includes the engine TU).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o stepnexp tools/stepnexp.hip
// Run:   stepnexp N_STEPS [A]   (A = 2 or 3; partial-divider_salad, B = 2^20, every step's state /
//        executed actions / collision mask written, stats on)
// Variants, timed interleaved (7 rounds x 20 launches each, min and median per variant):
//   product  oc_step_n_kernel: 4 envs per lane, one dword per plane per instruction (256 B per
//            wave store instruction); alone, with its in-launch totals fold, or followed by an
//            oc_stats_reduce launch
//   x2       8 envs per lane as two SWAR words, b64 loads and stores (512 B per wave store
//            instruction, half the store instructions), persistent grid of <= 5 blocks per CU
// Every variant's trajectory, exec, coll and final state are compared with the product's.
// Results (profiles/r02/stepnexp_*.log): on different boxes x2 ran 4-6 % faster than the
// product at A = 2 without the statistics fold, ~4 % slower with it, slower at A = 3 (156 VGPRs,
// 2 waves per SIMD), and at 100 steps per launch 6 % faster on one box and 8 % slower on
// another; the product stayed.
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
typedef unsigned int u32x4 __attribute__((__vector_size__(4 * sizeof(unsigned int))));

__device__ __forceinline__ u32x2 bld64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
}
template <int CP>
__device__ __forceinline__ void bst64(__amdgpu_buffer_rsrc_t r, uint32_t lo, uint32_t hi, uint32_t voff, uint32_t soff) {
    const u32x2 v = {lo, hi};
    __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)voff, (int)soff, CP);
}

template <int A, int K, int CP>
__global__ __launch_bounds__(kBlock) void step_n_x2(LevelArgs L, const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                                    const uint8_t* __restrict__ actions, uint8_t* __restrict__ traj,
                                                    uint8_t* __restrict__ exec_out, uint8_t* __restrict__ coll_out,
                                                    uint64_t* __restrict__ stats, uint32_t stat_rows, int n) {
    __shared__ uint32_t tbl4[64];
    if (threadIdx.x < 64u) tbl4[threadIdx.x] = L.cls4[threadIdx.x];
    __syncthreads();
    const uint8_t* tbl = (const uint8_t*)tbl4;
    const uint32_t P = (uint32_t)L.pitch, nlanes = P / 8u, stride = gridDim.x * (uint32_t)kBlock;
    constexpr int NP = 3 * A + 2 * K + 3;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    auto cls_of = [&](uint32_t cells) -> uint32_t {
        const uint32_t b0 = tbl[cells & 0xFFu], b1 = tbl[(cells >> 8) & 0xFFu], b2 = tbl[(cells >> 16) & 0xFFu],
                       b3 = tbl[cells >> 24];
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    };
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(sin, (int64_t)NP * P), ro = make_rsrc(sout, (int64_t)NP * P),
                                 ra = make_rsrc(actions, (int64_t)n * A * P), rt = make_rsrc(traj, (int64_t)n * NP * P),
                                 re = make_rsrc(exec_out, (int64_t)n * A * P), rc = make_rsrc(coll_out, (int64_t)n * P);
    StepStats st;
    for (uint32_t g = blockIdx.x * (uint32_t)kBlock + threadIdx.x; g < nlanes; g += stride) {
        const uint32_t vo = g * 8u;
        Chunk<A, K> c[2];
#pragma unroll
        for (int a = 0; a < A; ++a) {
            u32x2 v = bld64(rs, vo, a * P);
            c[0].wx[a] = v[0]; c[1].wx[a] = v[1];
            v = bld64(rs, vo, (kPY + a) * P);
            c[0].wy[a] = v[0]; c[1].wy[a] = v[1];
            v = bld64(rs, vo, (kPH + a) * P);
            c[0].wh[a] = v[0]; c[1].wh[a] = v[1];
            v = bld64(ra, vo, a * P);
            c[0].wa[a] = v[0]; c[1].wa[a] = v[1];
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            u32x2 v = bld64(rs, vo, (kPL + j) * P);
            c[0].wl[j] = v[0]; c[1].wl[j] = v[1];
            v = bld64(rs, vo, (kPM + j) * P);
            c[0].wm[j] = v[0]; c[1].wm[j] = v[1];
        }
        const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(g * 16u), (int)(kPT * P), 0);
        uint32_t T0[2] = {t[0], t[2]}, T1[2] = {t[1], t[3]};
        {
            const u32x2 v = bld64(rs, vo, kPF * P);
            c[0].wf = v[0]; c[1].wf = v[1];
        }
        uint32_t nxt[2][A];
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const u32x2 v = n > 1 ? bld64(ra, vo, (uint32_t)(A + a) * P) : u32x2{0u, 0u};
            nxt[0][a] = v[0]; nxt[1][a] = v[1];
        }
        const int64_t rem0 = L.B - (int64_t)g * 8;
        for (int r = 0; r < n; ++r) {
            uint32_t act[2][A], ex[2][A], cm[2];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    act[h][a] = c[h].wa[a];
                    c[h].wa[a] = nxt[h][a];
                }
            if (r + 2 < n) {
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    const u32x2 v = bld64(ra, vo, (uint32_t)((r + 2) * A + a) * P);
                    nxt[0][a] = v[0]; nxt[1][a] = v[1];
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t rem = rem0 - 4 * h;
                const uint32_t vmask = rem >= 4 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (1u << (8 * (uint32_t)rem)) - 1u);
                const uint32_t f_in = c[h].wf;
                ocsw::step4<A, K>(L.sw, c[h].wx, c[h].wy, c[h].wh, c[h].wl, c[h].wm, T0[h], T1[h], c[h].wf, act[h], ex[h],
                                  cm[h], cls_of);
                const uint32_t ended = (c[h].wf & ~f_in & vmask) & ocsw::k01;
                st.eps += __popc(ended);
                st.succ += __popc(c[h].wf & (ended << 1));
                st.err += __popc(c[h].wf & (ended << 2));
                st.coll += __popc(cm[h] & vmask);
                const uint32_t efull = (0x80808080u - ended) ^ 0x80808080u;
                const uint32_t sa = T0[h] & __builtin_amdgcn_perm(0u, efull, 0x01010000u);
                const uint32_t sb2 = T1[h] & __builtin_amdgcn_perm(0u, efull, 0x03030202u);
                st.steps += (sa & 0xFFFFu) + (sa >> 16) + (sb2 & 0xFFFFu) + (sb2 >> 16);
            }
            const uint32_t base = (uint32_t)r * NP * P;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                bst64<CP>(rt, c[0].wx[a], c[1].wx[a], vo, base + a * P);
                bst64<CP>(rt, c[0].wy[a], c[1].wy[a], vo, base + (kPY + a) * P);
                bst64<CP>(rt, c[0].wh[a], c[1].wh[a], vo, base + (kPH + a) * P);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                bst64<CP>(rt, c[0].wl[j], c[1].wl[j], vo, base + (kPL + j) * P);
                bst64<CP>(rt, c[0].wm[j], c[1].wm[j], vo, base + (kPM + j) * P);
            }
            const u32x4 tw = {T0[0], T1[0], T0[1], T1[1]};
            __builtin_amdgcn_raw_buffer_store_b128(tw, rt, (int)(g * 16u), (int)(base + kPT * P), CP);
            bst64<CP>(rt, c[0].wf, c[1].wf, vo, base + kPF * P);
#pragma unroll
            for (int a = 0; a < A; ++a) bst64<CP>(re, ex[0][a], ex[1][a], vo, (uint32_t)(r * A + a) * P);
            bst64<CP>(rc, cm[0], cm[1], vo, (uint32_t)r * P);
        }
#pragma unroll
        for (int a = 0; a < A; ++a) {
            bst64<CP>(ro, c[0].wx[a], c[1].wx[a], vo, a * P);
            bst64<CP>(ro, c[0].wy[a], c[1].wy[a], vo, (kPY + a) * P);
            bst64<CP>(ro, c[0].wh[a], c[1].wh[a], vo, (kPH + a) * P);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bst64<CP>(ro, c[0].wl[j], c[1].wl[j], vo, (kPL + j) * P);
            bst64<CP>(ro, c[0].wm[j], c[1].wm[j], vo, (kPM + j) * P);
        }
        const u32x4 tw = {T0[0], T1[0], T0[1], T1[1]};
        __builtin_amdgcn_raw_buffer_store_b128(tw, ro, (int)(g * 16u), (int)(kPT * P), CP);
        bst64<CP>(ro, c[0].wf, c[1].wf, vo, kPF * P);
    }
    if (stats != nullptr) {
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

}  // namespace

int main(int argc, char** argv) {
    const int64_t B = 1 << 20;
    const int n = argc > 1 ? atoi(argv[1]) : 20;
    const int A = argc > 2 ? atoi(argv[2]) : 2;  // 2 or 3 agents
    // partial-divider_salad (levels.py builtin): 7x7
    const char* rows[7] = {"-----t-", "/     l", "/  -  -", "*  -  -", "-  -  -", "-     p", "-----p-"};
    oc_level_desc lv{};
    lv.width = 7; lv.height = 7; lv.num_spawns = 4; lv.num_goals = 1;
    int ni = 0;
    for (int y = 0; y < 7; ++y)
        for (int x = 0; x < 7; ++x) {
            const char ch = rows[y][x];
            int t = ch == ' ' ? OC_TILE_FLOOR : ch == '/' ? OC_TILE_CUTBOARD : ch == '*' ? OC_TILE_DELIVERY : OC_TILE_COUNTER;
            lv.tiles[y * 7 + x] = (uint8_t)t;
            if (ch == 't' || ch == 'l' || ch == 'p') {
                lv.item_cell[ni] = (uint8_t)(y * 7 + x);
                lv.item_mask[ni++] = ch == 't' ? OC_M_TOMATO : ch == 'l' ? OC_M_LETTUCE : OC_M_PLATE;
            }
        }
    lv.num_items = ni;
    const uint8_t sx[4] = {2, 4, 4, 2}, sy[4] = {1, 1, 4, 4};
    for (int a = 0; a < 4; ++a) { lv.spawn_x[a] = sx[a]; lv.spawn_y[a] = sy[a]; }
    lv.goal_mask[0] = 0x3B;
    oc_handle* h;
    if (oc_create(&lv, A, 100, 0, &h) != 0) { printf("create: %s\n", oc_last_error()); return 1; }
    oc_layout lay;
    oc_get_layout(h, B, &lay);
    const int64_t S = lay.state_bytes, P = lay.pitch;
    uint8_t *s0, *s1, *acts, *tr[2], *ex[2], *co[2], *fin[2];
    uint64_t *stats, *totals;
    int64_t sb = 0;
    oc_stats_size(h, B, &sb);
    CK(hipMalloc(&s0, S)); CK(hipMalloc(&s1, S)); CK(hipMalloc(&acts, (int64_t)n * A * P));
    CK(hipMalloc(&stats, sb + 64)); CK(hipMalloc(&totals, 64));
    for (int v = 0; v < 2; ++v) {
        CK(hipMalloc(&tr[v], n * S)); CK(hipMalloc(&ex[v], (int64_t)n * A * P)); CK(hipMalloc(&co[v], (int64_t)n * P));
        CK(hipMalloc(&fin[v], S));
    }
    CK(hipMemset(stats, 0, sb + 64));
    oc_reset(h, s0, B, nullptr);
    for (int r = 0; r < n; ++r) oc_gen_actions(h, acts + (int64_t)r * A * P, B, 0, r, 7, nullptr);
    // a mid-episode start state: 37 product steps
    {
        uint8_t* a1;
        CK(hipMalloc(&a1, A * P));
        for (int r = 0; r < 37; ++r) {
            oc_gen_actions(h, a1, B, 0, 1000 + r, 3, nullptr);
            oc_step(h, r & 1 ? s1 : s0, r & 1 ? s0 : s1, a1, nullptr, nullptr, nullptr, B, nullptr);
        }
        CK(hipMemcpy(s0, s1, S, hipMemcpyDeviceToDevice));
    }
    CK(hipDeviceSynchronize());
    LevelArgs L = h->args;
    L.pitch = P;
    L.B = B;
    const uint32_t srows = (uint32_t)stats_rows(h, B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    // variants are timed interleaved: 7 rounds over all of them, 20 launches each, so that clock
    // and box drift hit every variant alike; min and median per variant are printed
    std::vector<std::pair<std::string, std::function<void(int)>>> vs;
    uint64_t* tot;
    CK(hipMalloc(&tot, 64));
    vs.push_back({"product oc_step_n (4 envs/lane, dword)", [&](int v) {
        oc_step_n(h, s0, fin[v], acts, tr[v], ex[v], co[v], stats, nullptr, B, n, nullptr);
    }});
    vs.push_back({"product, in-launch totals fold", [&](int v) {
        oc_step_n(h, s0, fin[v], acts, tr[v], ex[v], co[v], stats, tot, B, n, nullptr);
    }});
    vs.push_back({"product + oc_stats_reduce launch", [&](int v) {
        oc_step_n(h, s0, fin[v], acts, tr[v], ex[v], co[v], stats, nullptr, B, n, nullptr);
        oc_stats_reduce(h, stats, B, tot, nullptr);
    }});
    const int cus = h->cus;
    {
        const uint32_t need = (uint32_t)(P / 8 / kBlock), cap = (uint32_t)(cus * 5);
        const dim3 grid(need < cap ? need : cap);
        for (int red = 0; red < 2; ++red)
            vs.push_back({red ? "x2 (8 envs/lane, b64) + oc_stats_reduce launch" : "x2 (8 envs/lane, b64)",
                          [&, grid, red](int v) {
                              if (A == 2)
                                  hipLaunchKernelGGL((step_n_x2<2, 4, kCPnt>), grid, dim3(kBlock), 0, nullptr, L, s0, fin[v],
                                                     acts, tr[v], ex[v], co[v], stats, srows, n);
                              else
                                  hipLaunchKernelGGL((step_n_x2<3, 4, kCPnt>), grid, dim3(kBlock), 0, nullptr, L, s0, fin[v],
                                                     acts, tr[v], ex[v], co[v], stats, srows, n);
                              if (red) oc_stats_reduce(h, stats, B, tot, nullptr);
                          }});
    }
    std::vector<std::vector<double>> us(vs.size());
    for (auto& v : vs)
        for (int i = 0; i < 5; ++i) v.second(i & 1);
    for (int round = 0; round < 7; ++round)
        for (size_t k = 0; k < vs.size(); ++k) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < 20; ++i) vs[k].second(i & 1);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us[k].push_back(ms * 1e3 / 20);
        }
    const double bytes = (double)((3 * A + 11) + n * (3 * A + 11 + 2 * A + 1)) * B;
    for (size_t k = 0; k < vs.size(); ++k) {
        std::sort(us[k].begin(), us[k].end());
        printf("%-40s min %7.2f  median %7.2f us/launch  (%5.2f us/step, %4.2f TB/s at the median)\n", vs[k].first.c_str(),
               us[k][0], us[k][3], us[k][3] / n, bytes / (us[k][3] * 1e-6) / 1e12);
    }
    // outputs of every variant against the product's
    vs[0].second(0);  // the product: the reference outputs
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> ref_tr(n * S), ref_ex((size_t)n * A * P), ref_co((size_t)n * P), ref_f(S);
    CK(hipMemcpy(ref_tr.data(), tr[0], n * S, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref_ex.data(), ex[0], ref_ex.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref_co.data(), co[0], ref_co.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref_f.data(), fin[0], S, hipMemcpyDeviceToHost));
    bool all_same = true;
    for (size_t k = 1; k < vs.size(); ++k) {
        vs[k].second(1);
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> t2(n * S), e2(ref_ex.size()), c2(ref_co.size()), f2(S);
        CK(hipMemcpy(t2.data(), tr[1], n * S, hipMemcpyDeviceToHost));
        CK(hipMemcpy(e2.data(), ex[1], e2.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(c2.data(), co[1], c2.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(f2.data(), fin[1], S, hipMemcpyDeviceToHost));
        const bool same = t2 == ref_tr && e2 == ref_ex && c2 == ref_co && f2 == ref_f;
        all_same &= same;
        if (!same) printf("    %s: outputs DIFFER\n", vs[k].first.c_str());
    }
    printf("outputs %s\n", all_same ? "identical for every variant" : "differ");
    return 0;
}
