// tools/rolltl.hip -- where oc_rollout_kernel's time goes (round 5), and variants of its launch
// phases.  Includes the engine TU.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o tools/rolltl tools/rolltl.hip
// Workload: bench.py's C5 rows -- full-divider_salad, 4 agents, random-play states (37 steps),
// 64 Salad configurations, configuration-major allocation ids, random joint actions; 2^18 rows
// (bench) and 4,096 rows (the planner's launch size).
// Variants (all compared with the product's outputs):
//   product   oc_rollout (the C-ABI call)
//   tl        the product kernel with a per-wave s_memrealtime timeline: start, tables staged
//             (after the barrier), row loads landed, row computed, stores acknowledged
//   pre       the row's loads (state, t, flags, alloc, all A action planes) issued before the
//             table staging, so their latency overlaps it
//   pre_tl    pre with the timeline
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <algorithm>
#include <random>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

__device__ __forceinline__ uint64_t stamp(bool drain) {
    if (drain) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    return wall_clock64();
}

template <int A, int K, bool PRE, bool TL, bool UNI = false, bool TWICE = false>
__global__ __launch_bounds__(kBlock) void roll_var(RollArgs R, const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                                  const uint8_t* __restrict__ act, const uint8_t* __restrict__ alloc,
                                                  const uint8_t* __restrict__ blob_g, uint8_t* __restrict__ out_flags,
                                                  float* __restrict__ lb, uint64_t* __restrict__ tl) {
    extern __shared__ uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    uint64_t ts[6];
    if (TL) ts[0] = stamp(false);
    const int64_t P = R.pitch;
    using PL = Planes<A, K, false>;
    const int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x;  // one row per lane (grid covers B)
    const bool live = e < R.B;
    const int64_t ee = live ? e : 0;
    ocro::RowT<K, false> r;
    uint16_t t = 0;
    uint8_t fl_in = 0;
    int ai = 0;
    uint8_t ac[A];
    if (PRE) {
        r = load_row<A, K, false>(sin, P, ee);
        t = ((const uint16_t*)(sin + PL::T * P))[ee];
        fl_in = sin[PL::F * P + ee];
        ai = alloc != nullptr ? alloc[ee] : 0;
#pragma unroll
        for (int a = 0; a < A; ++a) ac[a] = act[a * P + ee];
    }
    stage_roll_tables(R, blob_g, blob_w, subs);
    if (TL) ts[1] = stamp(false);
    const uint8_t* blob = (const uint8_t*)blob_w;
    if (!PRE) {
        r = load_row<A, K, false>(sin, P, ee);
        t = ((const uint16_t*)(sin + PL::T * P))[ee];
        fl_in = sin[PL::F * P + ee];
        ai = alloc != nullptr ? alloc[ee] : 0;
#pragma unroll
        for (int a = 0; a < A; ++a) ac[a] = act[a * P + ee];
    }
    if (TL) ts[2] = stamp(true);
    float bound = 0.0f;
    int f = OC_ROLL_BADALLOC;
    uint32_t aw = 0;
#pragma unroll
    for (int a = 0; a < A; ++a) aw |= (uint32_t)ac[a] << (8 * a);
    auto go = [&](const ocro::Sub& s) {
        const int c0 = (aw >> (8 * s.agent[0])) & 0xFF, c1 = s.n == 2 ? (aw >> (8 * s.agent[1])) & 0xFF : ocro::kNoop;
        ocro::RowOps<A, K, false> ops(R.L, blob, blob + R.L.dist_off);
        f = ops.run(r, s, c0, c1, bound);
    };
    if (TWICE) {  // the same row computed once before, discarded: the second pass runs from a warm
                  // instruction cache (and the same LDS lines)
        if (ai < R.nsub) {
            ocro::RowT<K, false> r2 = r;
            float b2 = 0.0f;
            const ocro::Sub& s = subs[ai];
            const int c0 = (aw >> (8 * s.agent[0])) & 0xFF, c1 = s.n == 2 ? (aw >> (8 * s.agent[1])) & 0xFF : ocro::kNoop;
            ocro::RowOps<A, K, false> ops(R.L, blob, blob + R.L.dist_off);
            const int f2 = ops.run(r2, s, c0, c1, b2);
            asm volatile("" :: "v"(f2), "v"(b2), "v"(r2.x));
        }
        if (TL) ts[5] = stamp(true);
    }
    if (ai < R.nsub) {
        if (UNI) {
            const int a0 = __builtin_amdgcn_readfirstlane(ai);
            if (__ballot(ai != a0) == 0ull) {  // one configuration in the wave: its fields in SGPRs
                const uint32_t* sw = (const uint32_t*)&subs[a0];
                ocro::Sub su;
                su.kind = __builtin_amdgcn_readfirstlane((int)sw[0]);
                su.n = __builtin_amdgcn_readfirstlane((int)sw[1]);
                const uint32_t w2 = __builtin_amdgcn_readfirstlane(sw[2]), w3 = __builtin_amdgcn_readfirstlane(sw[3]);
                su.agent[0] = w2 & 0xFF; su.agent[1] = (w2 >> 8) & 0xFF; su.start[0] = (w2 >> 16) & 0xFF;
                su.start[1] = w2 >> 24; su.goal = w3 & 0xFF; su.count = (w3 >> 8) & 0xFF;
                su.level = (w3 >> 16) & 0xFF; su.pad = 0;
                go(su);
            } else {
                go(subs[ai]);
            }
        } else {
            go(subs[ai]);
        }
    }
    if (TL) ts[3] = stamp(true);
    if (live) {
        store_row<A, K, false>(sout, P, e, r);
        ((uint16_t*)(sout + PL::T * P))[e] = t;
        sout[PL::F * P + e] = fl_in;
        out_flags[e] = (uint8_t)f;
        lb[e] = bound;
    }
    if (TL) {
        ts[4] = stamp(true);
        if ((threadIdx.x & 63) == 0) {
            const int64_t w = (blockIdx.x * (int64_t)kBlock + threadIdx.x) / 64;
#pragma unroll
            for (int k = 0; k < 5; ++k) tl[w * 8 + k] = ts[k];
            if (TWICE) tl[w * 8 + 5] = ts[5];
        }
    }
}

// The product row (RowOps::run) split into its phases, a stamp after each (lane 0 of every wave
// records; the drains make each phase's LDS reads land inside it)
template <int A, int K>
__global__ __launch_bounds__(kBlock) void roll_phases(RollArgs R, const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                                     const uint8_t* __restrict__ act, const uint8_t* __restrict__ alloc,
                                                     const uint8_t* __restrict__ blob_g, uint8_t* __restrict__ out_flags,
                                                     float* __restrict__ lb, uint64_t* __restrict__ tl) {
    extern __shared__ uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    const int64_t P = R.pitch;
    using PL = Planes<A, K, false>;
    const int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    const bool live = e < R.B;
    const int64_t ee = live ? e : 0;
    ocro::RowT<K, false> r = load_row<A, K, false>(sin, P, ee);
    const uint32_t t = ((const uint16_t*)(sin + PL::T * P))[ee], fl_in = sin[PL::F * P + ee];
    const int ai = alloc[ee];
    uint32_t aw = 0;
#pragma unroll
    for (int a = 0; a < A; ++a) aw |= (uint32_t)act[a * P + ee] << (8 * a);
    stage_roll_tables(R, blob_g, blob_w, subs);
    const uint8_t* blob = (const uint8_t*)blob_w;
    uint64_t ts[7];
    ts[0] = stamp(true);
    float bound = 0.0f;
    int f = OC_ROLL_BADALLOC;
    if (ai < R.nsub) {
        const ocro::Sub& s = subs[ai];
        int c0 = (aw >> (8 * s.agent[0])) & 0xFF, c1 = s.n == 2 ? (aw >> (8 * s.agent[1])) & 0xFF : ocro::kNoop;
        ocro::RowOps<A, K, false> ops(R.L, blob, blob + R.L.dist_off);
        const ocro::RowT<K, false> r_in = r;
        const bool raised = ops.level0(r, s);
        ts[1] = stamp(true);
        if (raised) {
            r = r_in;
            f = 8;
            ts[2] = ts[3] = ts[4] = ts[5] = stamp(true);
        } else {
            if (s.kind == 0) c0 = c1 = ocro::kNoop;
            c0 = c0 > ocro::kNoop ? ocro::kNoop : c0;
            c1 = c1 > ocro::kNoop ? ocro::kNoop : c1;
            // as RowOps::run: the agents' target squares read once, the legality without branches
            const auto g0 = ops.target(r, s.agent[0], c0), g1 = s.n == 2 ? ops.target(r, s.agent[1], c1) : g0;
            int fl = ops.action_legal(r, s, c0, c1, g0, g1) ? 1 : 0;
            ts[2] = stamp(true);
            ops.interact(r, s.agent[0], c0, g0);
            if (s.n == 2) ops.interact(r, s.agent[1], c1, g1);
            ts[3] = stamp(true);
            const bool asserted = s.n == 2 && ops.agent_cell(r, s.agent[0]) == ops.agent_cell(r, s.agent[1]);
            if (asserted) fl |= 4;
            else if (ops.is_goal(r, s)) fl |= 2;
            ts[4] = stamp(true);
            bound = ops.lower_bound(r, s);
            ts[5] = stamp(true);
            f = fl;
        }
    } else {
        ts[1] = ts[2] = ts[3] = ts[4] = ts[5] = stamp(true);
    }
    if (live) {
        store_row<A, K, false>(sout, P, e, r);
        ((uint16_t*)(sout + PL::T * P))[e] = (uint16_t)t;
        sout[PL::F * P + e] = (uint8_t)fl_in;
        out_flags[e] = (uint8_t)f;
        lb[e] = bound;
    }
    ts[6] = stamp(true);
    if ((threadIdx.x & 63) == 0) {
        const int64_t w = (blockIdx.x * (int64_t)kBlock + threadIdx.x) / 64;
#pragma unroll
        for (int k = 0; k < 7; ++k) tl[w * 8 + k] = ts[k];
        tl[w * 8 + 7] = (uint64_t)ai;
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t Bmax = 1 << 18;
    const char* rows[7] = {"-----t-", "/  -  l", "/  -  -", "*  -  -", "-  -  -", "-  -  p", "-----p-"};
    oc_level_desc lv{};
    lv.width = 7; lv.height = 7; lv.num_spawns = 4; lv.num_goals = 1;
    int ni = 0;
    for (int y = 0; y < 7; ++y)
        for (int x = 0; x < 7; ++x) {
            const char ch = rows[y][x];
            int tt = ch == ' ' ? OC_TILE_FLOOR : ch == '/' ? OC_TILE_CUTBOARD : ch == '*' ? OC_TILE_DELIVERY : OC_TILE_COUNTER;
            lv.tiles[y * 7 + x] = (uint8_t)tt;
            if (ch == 't' || ch == 'l' || ch == 'p') {
                lv.item_cell[ni] = (uint16_t)(y * 7 + x);
                lv.item_mask[ni++] = ch == 't' ? OC_M_TOMATO : ch == 'l' ? OC_M_LETTUCE : OC_M_PLATE;
            }
        }
    lv.num_items = ni;
    const uint8_t sx[4] = {2, 4, 4, 2}, sy[4] = {1, 1, 4, 4};
    for (int a = 0; a < 4; ++a) { lv.spawn_x[a] = sx[a]; lv.spawn_y[a] = sy[a]; }
    lv.goal_mask[0] = 0x3B;
    oc_handle* h;
    if (oc_create(&lv, 4, 100, 0, &h) != 0) { printf("create: %s\n", oc_last_error()); return 1; }
    const int kinds[9] = {1, 1, 2, 2, 2, 2, 2, 2, 3};
    const uint8_t st0[9] = {0x01, 0x02, 0x11, 0x11, 0x22, 0x33, 0x19, 0x2A, 0x3B}, st1[9] = {0, 0, 0x22, 0x08, 0x08, 0x08, 0x22, 0x11, 0};
    const uint8_t goal[9] = {0x11, 0x22, 0x33, 0x19, 0x2A, 0x3B, 0x3B, 0x3B, 0x3B};
    std::vector<oc_subtask> subs;
    const int sets[10][2] = {{0, -1}, {1, -1}, {2, -1}, {3, -1}, {0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
    for (int k = 0; k < 9 && (int)subs.size() < 64; ++k)
        for (int a = 0; a < 10 && (int)subs.size() < 64; ++a) {
            oc_subtask st{};
            st.kind = kinds[k]; st.num_agents = sets[a][1] < 0 ? 1 : 2;
            st.agent[0] = (uint8_t)sets[a][0]; st.agent[1] = (uint8_t)(sets[a][1] < 0 ? 0 : sets[a][1]);
            st.start_mask[0] = st0[k]; st.start_mask[1] = st1[k]; st.goal_mask = goal[k];
            subs.push_back(st);
        }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (const int64_t B : {Bmax, (int64_t)4096}) {
        oc_layout lay;
        oc_get_layout(h, B, &lay);
        const int64_t S = lay.state_bytes, P = lay.pitch;
        uint8_t *s0, *s1, *acts, *alloc, *out[2], *fl[2];
        float* lbd[2];
        uint64_t* tl;
        const int64_t nwaves = (B + 63) / 64;
        CK(hipMalloc(&s0, S)); CK(hipMalloc(&s1, S)); CK(hipMalloc(&acts, 4 * P)); CK(hipMalloc(&alloc, P));
        CK(hipMalloc(&tl, nwaves * 8 * sizeof(uint64_t)));
        for (int v = 0; v < 2; ++v) { CK(hipMalloc(&out[v], S)); CK(hipMalloc(&fl[v], P)); CK(hipMalloc(&lbd[v], 4 * P)); }
        oc_reset(h, s0, B, nullptr);
        for (int r = 0; r < 37; ++r) {
            oc_gen_actions(h, acts, B, 0, r, 11, nullptr);
            oc_step(h, r & 1 ? s1 : s0, r & 1 ? s0 : s1, acts, nullptr, nullptr, nullptr, B, nullptr);
        }
        CK(hipMemcpy(s0, s1, S, hipMemcpyDeviceToDevice));
        oc_gen_actions(h, acts, B, 0, 99, 12, nullptr);
        std::vector<uint8_t> al(P, 0);
        {
            std::mt19937 g(5);
            for (int64_t e = 0; e < B; ++e) al[e] = (uint8_t)(g() % subs.size());
            std::sort(al.begin(), al.begin() + B);
        }
        CK(hipMemcpy(alloc, al.data(), P, hipMemcpyHostToDevice));
        RollArgs R;
        if (roll_args(h, subs.data(), (int)subs.size(), B, R, true)) { printf("args: %s\n", oc_last_error()); return 1; }
        const int reps = B > 4096 ? 200 : 1000;
        auto time = [&](const char* name, auto&& fn) {
            for (int i = 0; i < 5; ++i) fn(0);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) fn(0);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("B=%-7lld %-40s %8.2f us/launch\n", (long long)B, name, ms * 1e3 / reps);
        };
        auto product = [&](int v) {
            oc_rollout(h, s0, out[v], acts, alloc, subs.data(), (int)subs.size(), fl[v], lbd[v], B, nullptr);
        };
        const dim3 grid((unsigned)((B + kBlock - 1) / kBlock));
        const int lds = h->roll.lds_bytes;
#define VAR(PRE, TL)                                                                                         \
    [&](int v) {                                                                                             \
        hipLaunchKernelGGL((roll_var<4, 4, PRE, TL>), grid, dim3(kBlock), lds, nullptr, R, s0, out[v], acts, \
                           alloc, h->roll_blob, fl[v], lbd[v], tl);                                           \
    }
#define VAR3(PRE, TL, UNI)                                                                                     \
    [&](int v) {                                                                                                   \
        hipLaunchKernelGGL((roll_var<4, 4, PRE, TL, UNI>), grid, dim3(kBlock), lds, nullptr, R, s0, out[v], acts, \
                           alloc, h->roll_blob, fl[v], lbd[v], tl);                                                 \
    }
        std::vector<uint8_t> o0(S), o1(S), f0(B), f1(B);
        std::vector<float> l0(B), l1(B);
        auto same = [&]() {
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(o0.data(), out[0], S, hipMemcpyDeviceToHost)); CK(hipMemcpy(o1.data(), out[1], S, hipMemcpyDeviceToHost));
            CK(hipMemcpy(f0.data(), fl[0], B, hipMemcpyDeviceToHost)); CK(hipMemcpy(f1.data(), fl[1], B, hipMemcpyDeviceToHost));
            CK(hipMemcpy(l0.data(), lbd[0], 4 * B, hipMemcpyDeviceToHost)); CK(hipMemcpy(l1.data(), lbd[1], 4 * B, hipMemcpyDeviceToHost));
            return o0 == o1 && f0 == f1 && l0 == l1;
        };
        auto timeline = [&](const char* name) {
            std::vector<uint64_t> h_tl(nwaves * 8);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h_tl.data(), tl, h_tl.size() * 8, hipMemcpyDeviceToHost));
            uint64_t t0 = ~0ull, tend = 0;
            for (int64_t w = 0; w < nwaves; ++w) { t0 = std::min(t0, h_tl[w * 8]); tend = std::max(tend, h_tl[w * 8 + 4]); }
            const char* ph[5] = {"start", "staged", "loaded", "computed", "stored"};
            printf("  timeline %s (wall_clock64 100 MHz, us from the first wave's start; whole %.2f us)\n", name,
                   (tend - t0) * 0.01);
            for (int k = 0; k < 5; ++k) {
                std::vector<double> v;
                for (int64_t w = 0; w < nwaves; ++w) v.push_back((h_tl[w * 8 + k] - t0) * 0.01);
                std::sort(v.begin(), v.end());
                printf("    %-9s min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f\n", ph[k], v[0], v[v.size() / 10],
                       v[v.size() / 2], v[v.size() * 9 / 10], v.back());
            }
            for (int k = 1; k < 5; ++k) {
                std::vector<double> v;
                for (int64_t w = 0; w < nwaves; ++w) v.push_back((h_tl[w * 8 + k] - h_tl[w * 8 + k - 1]) * 0.01);
                std::sort(v.begin(), v.end());
                printf("    d(%s-%s) p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f\n", ph[k], ph[k - 1], v[v.size() / 10],
                       v[v.size() / 2], v[v.size() * 9 / 10], v.back());
            }
        };
        time("product (oc_rollout)", product);
        auto v_pre = VAR(true, false);
        time("pre: row loads before the staging", v_pre);
        product(0); v_pre(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        auto v_tl = VAR(false, true);
        time("tl: product kernel + timeline", v_tl);
        product(0); v_tl(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        timeline("product");
        auto v_ptl = VAR(true, true);
        time("pre_tl: pre + timeline", v_ptl);
        product(0); v_ptl(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        timeline("pre");
        {
            auto v_tw = [&](int v) {
                hipLaunchKernelGGL((roll_var<4, 4, true, true, false, true>), grid, dim3(kBlock), lds, nullptr, R, s0,
                                   out[v], acts, alloc, h->roll_blob, fl[v], lbd[v], tl);
            };
            time("twice: pre + the row computed twice (timeline)", v_tw);
            product(0); v_tw(1);
            printf("  outputs %s\n", same() ? "identical" : "DIFFER");
            std::vector<uint64_t> h_tl(nwaves * 8);
            CK(hipMemcpy(h_tl.data(), tl, h_tl.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> d1, d2;
            for (int64_t w = 0; w < nwaves; ++w) {
                d1.push_back((h_tl[w * 8 + 5] - h_tl[w * 8 + 2]) * 0.01);  // first pass (cold)
                d2.push_back((h_tl[w * 8 + 3] - h_tl[w * 8 + 5]) * 0.01);  // second pass (warm)
            }
            std::sort(d1.begin(), d1.end());
            std::sort(d2.begin(), d2.end());
            printf("  first pass  p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", d1[d1.size() / 10], d1[d1.size() / 2],
                   d1[d1.size() * 9 / 10], d1.back());
            printf("  second pass p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", d2[d2.size() / 10], d2[d2.size() / 2],
                   d2[d2.size() * 9 / 10], d2.back());
        }
        auto v_uni = VAR3(true, false, true);
        time("uni: pre + wave-uniform configuration in SGPRs", v_uni);
        product(0); v_uni(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        auto v_utl = VAR3(true, true, true);
        time("uni_tl", v_utl);
        timeline("uni");
        {  // the row's phases, per wave; waves grouped by their first row's configuration kind
            auto v_ph = [&](int v) {
                hipLaunchKernelGGL((roll_phases<4, 4>), grid, dim3(kBlock), lds, nullptr, R, s0, out[v], acts, alloc,
                                   h->roll_blob, fl[v], lbd[v], tl);
            };
            time("phases: the row's phases stamped", v_ph);
            product(0); v_ph(1);
            printf("  outputs %s\n", same() ? "identical" : "DIFFER");
            std::vector<uint64_t> h_tl(nwaves * 8);
            CK(hipMemcpy(h_tl.data(), tl, h_tl.size() * 8, hipMemcpyDeviceToHost));
            const char* nm[6] = {"level0", "legal", "interact", "goal", "bound", "store"};
            for (int grpk = 0; grpk < 4; ++grpk) {  // 0: Chop 1 agent, 1: Chop 2, 2: Merge 1, 3: Merge 2
                printf("  phases, waves of %s %s agent(s), us (p50 / p90):", grpk < 2 ? "Chop" : "Merge", grpk % 2 ? "2" : "1");
                for (int k = 1; k < 7; ++k) {
                    std::vector<double> d;
                    for (int64_t w = 0; w < nwaves; ++w) {
                        const int ai = (int)h_tl[w * 8 + 7];
                        if (ai >= (int)subs.size()) continue;
                        const int kind = subs[ai].kind, na = subs[ai].num_agents;
                        if (kind == 3 || (kind == 1) != (grpk < 2) || (na == 2) != (grpk % 2 == 1)) continue;
                        d.push_back((h_tl[w * 8 + k] - h_tl[w * 8 + k - 1]) * 0.01);
                    }
                    if (d.empty()) continue;
                    std::sort(d.begin(), d.end());
                    printf("  %s %.2f/%.2f", nm[k - 1], d[d.size() / 2], d[d.size() * 9 / 10]);
                }
                printf("\n");
            }
        }
        if (B > 4096 && argc > 1) {  // every row of one configuration: the cost of each configuration's path
            std::vector<uint8_t> one(P, 0);
            for (int c = 0; c < (int)subs.size(); ++c) {
                std::fill(one.begin(), one.begin() + B, (uint8_t)c);
                CK(hipMemcpy(alloc, one.data(), P, hipMemcpyHostToDevice));
                char name[96];
                snprintf(name, sizeof name, "config %2d kind %d agents %d,%d", c, subs[c].kind, subs[c].agent[0],
                         subs[c].num_agents == 2 ? subs[c].agent[1] : -1);
                time(name, product);
                time("   uni", v_uni);
            }
            CK(hipMemcpy(alloc, al.data(), P, hipMemcpyHostToDevice));
        }
        CK(hipFree(s0)); CK(hipFree(s1)); CK(hipFree(acts)); CK(hipFree(alloc)); CK(hipFree(tl));
        for (int v = 0; v < 2; ++v) { CK(hipFree(out[v])); CK(hipFree(fl[v])); CK(hipFree(lbd[v])); }
    }
    oc_destroy(h);
    return 0;
}
