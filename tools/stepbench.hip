// tools/stepbench.hip -- ablations of the step kernel (includes the engine TU for its internals).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o tools/stepbench tools/stepbench.hip
// Workload: partial-divider_salad, 2 agents, B = 2^20 (the bench config).
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

// E2: memory only (identity step), same loads/stores/pipelining as the product kernel.
template <int A, int K>
__global__ __launch_bounds__(kBlock) void mem_only(LevelArgs L, const uint8_t* sin, uint8_t* sout, const uint8_t* actions,
                                                   uint8_t* exec_out, uint8_t* coll_out) {
    const uint32_t P = (uint32_t)L.pitch, nlanes = P / kEPL, stride = gridDim.x * (uint32_t)kBlock;
    constexpr int NP = 3 * A + 2 * K + 3;
    Bufs b;
    b.sin = make_rsrc(sin, (int64_t)NP * P);
    b.sout = make_rsrc(sout, (int64_t)NP * P);
    b.act = make_rsrc(actions, (int64_t)A * P);
    b.ex = make_rsrc(exec_out, (int64_t)A * P);
    b.coll = make_rsrc(coll_out, (int64_t)P);
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    for (uint32_t g = blockIdx.x * (uint32_t)kBlock + threadIdx.x; g < nlanes; g += stride) {
        Chunk<A, K> c;
        load_chunk<A, K>(c, b, P, g);
        const uint32_t vo = g * 4u;
        for (int a = 0; a < A; ++a) {
            bst32(b.sout, c.wx[a], vo, a * P);
            bst32(b.sout, c.wy[a], vo, (kPY + a) * P);
            bst32(b.sout, c.wh[a], vo, (kPH + a) * P);
            bst32(b.ex, c.wa[a], vo, a * P);
        }
        for (int j = 0; j < K; ++j) {
            bst32(b.sout, c.wl[j], vo, (kPL + j) * P);
            bst32(b.sout, c.wm[j], vo, (kPM + j) * P);
        }
        typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
        const u32x2 tw = {c.wt.x, c.wt.y};
        __builtin_amdgcn_raw_buffer_store_b64(tw, b.sout, (int)(g * 8u), (int)(kPT * P), 0);
        bst32(b.sout, c.wf, vo, kPF * P);
        bst32(b.coll, c.wf, vo, 0u);
    }
}

// E3/E4: R fused steps per launch; state stays in registers; per step the actions are read
// (actions + r * A * P) and, if traj != nullptr, the full state + exec + coll are written.
template <int A, int K>
__global__ __launch_bounds__(kBlock) void fused(LevelArgs L, const uint8_t* sin, uint8_t* sout, const uint8_t* actions,
                                                uint8_t* traj, int R) {
    __shared__ uint8_t tbl[256];
    tbl[threadIdx.x] = ocsw::tile_class(L.floor_mask, L.deliv_mask, L.cut_mask, threadIdx.x);
    __syncthreads();
    const uint32_t P = (uint32_t)L.pitch, nlanes = P / kEPL, stride = gridDim.x * (uint32_t)kBlock;
    constexpr int NP = 3 * A + 2 * K + 3;
    auto cls_of = [&](uint32_t cells) -> uint32_t {
        const uint32_t b0 = tbl[cells & 0xFFu], b1 = tbl[(cells >> 8) & 0xFFu], b2 = tbl[(cells >> 16) & 0xFFu], b3 = tbl[cells >> 24];
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    };
    Bufs b;
    b.sin = make_rsrc(sin, (int64_t)NP * P);
    b.sout = make_rsrc(sout, (int64_t)NP * P);
    b.act = make_rsrc(actions, (int64_t)R * A * P);
    __amdgpu_buffer_rsrc_t tr = make_rsrc(traj ? traj : sout, traj ? (int64_t)R * (NP + A + 1) * P : 0);
    for (uint32_t g = blockIdx.x * (uint32_t)kBlock + threadIdx.x; g < nlanes; g += stride) {
        Chunk<A, K> c;
        load_chunk<A, K>(c, b, P, g);
        uint32_t T0 = c.wt.x, T1 = c.wt.y;
        const uint32_t vo = g * 4u;
        uint32_t nxt[A];
        for (int a = 0; a < A; ++a) nxt[a] = bld32(b.act, vo, (uint32_t)(R > 1 ? A + a : a) * P);
        for (int r = 0; r < R; ++r) {
            uint32_t act[A], ex[A], cm;
            for (int a = 0; a < A; ++a) act[a] = c.wa[a];
            if (r + 1 < R)  // prefetch next step's actions
                for (int a = 0; a < A; ++a) c.wa[a] = nxt[a];
            if (r + 2 < R)
                for (int a = 0; a < A; ++a) nxt[a] = bld32(b.act, vo, (uint32_t)((r + 2) * A + a) * P);
            ocsw::step4<A, K>(L.sw, c.wx, c.wy, c.wh, c.wl, c.wm, T0, T1, c.wf, act, ex, cm, cls_of);
            if (traj != nullptr) {
                const uint32_t base = (uint32_t)r * (NP + A + 1) * P;
                for (int a = 0; a < A; ++a) {
                    bst32(tr, c.wx[a], vo, base + a * P);
                    bst32(tr, c.wy[a], vo, base + (A + a) * P);
                    bst32(tr, c.wh[a], vo, base + (2 * A + a) * P);
                    bst32(tr, ex[a], vo, base + (NP + a) * P);
                }
                for (int j = 0; j < K; ++j) {
                    bst32(tr, c.wl[j], vo, base + (3 * A + j) * P);
                    bst32(tr, c.wm[j], vo, base + (3 * A + K + j) * P);
                }
                typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
                const u32x2 tw = {T0, T1};
                __builtin_amdgcn_raw_buffer_store_b64(tw, tr, (int)(g * 8u), (int)(base + (3 * A + 2 * K) * P), 0);
                bst32(tr, c.wf, vo, base + (NP - 1) * P);
                bst32(tr, cm, vo, base + (NP + A) * P);
            }
        }
        // final state
        constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
        for (int a = 0; a < A; ++a) {
            bst32(b.sout, c.wx[a], vo, a * P);
            bst32(b.sout, c.wy[a], vo, (kPY + a) * P);
            bst32(b.sout, c.wh[a], vo, (kPH + a) * P);
        }
        for (int j = 0; j < K; ++j) {
            bst32(b.sout, c.wl[j], vo, (kPL + j) * P);
            bst32(b.sout, c.wm[j], vo, (kPM + j) * P);
        }
        typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
        const u32x2 tw = {T0, T1};
        __builtin_amdgcn_raw_buffer_store_b64(tw, b.sout, (int)(g * 8u), (int)(kPT * P), 0);
        bst32(b.sout, c.wf, vo, kPF * P);
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? atoll(argv[1]) : (1ll << 20);
    const int A = 2, K = 4;
    oc_level_desc lv{};
    const char* rows[7] = {"-----t-", "/  -  l", "/  -  -", "*  -  -", "-  -  -", "-     p", "-----p-"};
    lv.width = 7;
    lv.height = 7;
    int ni = 0;
    for (int y = 0; y < 7; ++y)
        for (int x = 0; x < 7; ++x) {
            const char ch = rows[y][x];
            const int c = y * 7 + x;
            lv.tiles[c] = ch == ' ' ? 0 : ch == '/' ? 2 : ch == '*' ? 3 : 1;
            if (ch == 't' || ch == 'l' || ch == 'p') {
                lv.item_cell[ni] = (uint8_t)c;
                lv.item_mask[ni++] = ch == 't' ? 1 : ch == 'l' ? 2 : 8;
            }
        }
    lv.num_items = ni;
    lv.num_spawns = 4;
    const uint8_t sx[4] = {2, 4, 4, 2}, sy[4] = {1, 1, 4, 4};
    for (int a = 0; a < 4; ++a) { lv.spawn_x[a] = sx[a]; lv.spawn_y[a] = sy[a]; }
    lv.num_goals = 1;
    lv.goal_mask[0] = 0x3B;
    oc_handle* h;
    if (oc_create(&lv, A, 100, 0, &h) != 0) { printf("create: %s\n", oc_last_error()); return 1; }
    oc_layout lay;
    oc_get_layout(h, B, &lay);
    const int64_t P = lay.pitch, NP = lay.num_planes;
    const int R = 16;
    uint8_t *sa, *sb, *act, *ex, *coll, *traj;
    CK(hipMalloc(&sa, NP * P));
    CK(hipMalloc(&sb, NP * P));
    CK(hipMalloc(&act, (int64_t)R * A * P));
    CK(hipMalloc(&ex, A * P));
    CK(hipMalloc(&coll, P));
    CK(hipMalloc(&traj, (int64_t)R * (NP + A + 1) * P));
    oc_reset(h, sa, B, nullptr);
    for (int r = 0; r < R; ++r) oc_gen_actions(h, act + (int64_t)r * A * P, B, 0, r, 1, nullptr);
    CK(hipDeviceSynchronize());
    LevelArgs L = h->args;
    L.pitch = P;
    L.B = B;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto f, int reps) {
        for (int i = 0; i < 3; ++i) f();
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1000.0 / reps;
    };
    const double bytes = 39.0 * B;
    printf("B=%lld  algorithmic %.1f MB/step\n", (long long)B, bytes / 1e6);
    for (int bpc : {1, 2, 4}) {
        h->blocks_per_cu = bpc;
        const double us = timeit([&] { oc_step(h, sa, sb, act, ex, coll, nullptr, B, nullptr); }, 50);
        printf("E1 product oc_step        bpc %d: %7.2f us/step  %6.2f TB/s alg\n", bpc, us, bytes / us / 1e6);
    }
    uint64_t* stats;
    CK(hipMalloc(&stats, 1 << 20));
    CK(hipMemset(stats, 0, 1 << 20));
    for (int bpc : {2}) {
        h->blocks_per_cu = bpc;
        const double us = timeit([&] { oc_step(h, sa, sb, act, ex, coll, stats, B, nullptr); }, 50);
        printf("E1b product + stats       bpc %d: %7.2f us/step\n", bpc, us);
        int k = 0;
        const double us2 = timeit([&] { oc_step(h, (k & 1) ? sb : sa, (k & 1) ? sa : sb, act + (int64_t)(k % R) * A * P, ex, coll, stats, B, nullptr); ++k; }, 50);
        printf("E1c ping-pong + stats     bpc %d: %7.2f us/step\n", bpc, us2);
        // hipGraph of 16 ping-pong steps
        hipStream_t s;
        CK(hipStreamCreate(&s));
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 16; ++i) oc_step(h, (i & 1) ? sb : sa, (i & 1) ? sa : sb, act + (int64_t)i * A * P, ex, coll, stats, B, s);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        hipEvent_t a0, a1;
        CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1));
        for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(a0, s));
        for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(a1, s));
        CK(hipEventSynchronize(a1));
        float ms; CK(hipEventElapsedTime(&ms, a0, a1));
        printf("E1d hipGraph 16 steps     bpc %d: %7.2f us/step\n", bpc, ms * 1000.0 / 160);
    }
    {  // E5: two half-batch chains on two streams (independent env ranges), as a graph
        h->blocks_per_cu = 2;
        for (int nsplit : {1, 2, 4}) {
            hipStream_t s0, sx[4];
            CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
            for (int i = 0; i < nsplit; ++i) CK(hipStreamCreateWithFlags(&sx[i], hipStreamNonBlocking));
            hipEvent_t fork, join[4];
            CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
            for (int i = 0; i < nsplit; ++i) CK(hipEventCreateWithFlags(&join[i], hipEventDisableTiming));
            const int64_t Bh = B / nsplit;  // multiple of 4096: byte offsets stay 16-B aligned
            oc_handle* hh;
            oc_create(&lv, A, 100, 0, &hh);
            hh->blocks_per_cu = 2;
            oc_layout lh;
            oc_get_layout(hh, Bh, &lh);
            std::vector<uint8_t*> ha(nsplit), hb(nsplit), hact(nsplit), hex(nsplit), hco(nsplit);
            for (int i = 0; i < nsplit; ++i) {
                CK(hipMalloc(&ha[i], lh.state_bytes)); CK(hipMalloc(&hb[i], lh.state_bytes));
                CK(hipMalloc(&hact[i], (int64_t)16 * A * lh.pitch)); CK(hipMalloc(&hex[i], A * lh.pitch));
                CK(hipMalloc(&hco[i], lh.pitch));
                oc_reset(hh, ha[i], Bh, nullptr);
                for (int r = 0; r < 16; ++r) oc_gen_actions(hh, hact[i] + (int64_t)r * A * lh.pitch, Bh, i * Bh, r, 1, nullptr);
            }
            CK(hipDeviceSynchronize());
            hipGraph_t gr;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
            CK(hipEventRecord(fork, s0));
            for (int i = 0; i < nsplit; ++i) {
                CK(hipStreamWaitEvent(sx[i], fork, 0));
                for (int k = 0; k < 16; ++k)
                    oc_step(hh, (k & 1) ? hb[i] : ha[i], (k & 1) ? ha[i] : hb[i], hact[i] + (int64_t)k * A * lh.pitch, hex[i],
                            hco[i], stats, Bh, sx[i]);
                CK(hipEventRecord(join[i], sx[i]));
                CK(hipStreamWaitEvent(s0, join[i], 0));
            }
            CK(hipStreamEndCapture(s0, &gr));
            CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
            hipEvent_t a0, a1;
            CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1));
            for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s0));
            CK(hipEventRecord(a0, s0));
            for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s0));
            CK(hipEventRecord(a1, s0));
            CK(hipEventSynchronize(a1));
            float ms; CK(hipEventElapsedTime(&ms, a0, a1));
            printf("E5 graph, %d parallel chains of B/%d: %7.2f us/step (whole batch)\n", nsplit, nsplit, ms * 1000.0 / 160);
            // eager: round-robin launches over the split streams
            const double us = timeit([&] {
                for (int k = 0; k < 16; ++k)
                    for (int i = 0; i < nsplit; ++i)
                        oc_step(hh, (k & 1) ? hb[i] : ha[i], (k & 1) ? ha[i] : hb[i], hact[i] + (int64_t)k * A * lh.pitch,
                                hex[i], hco[i], stats, Bh, sx[i]);
            }, 5) / 16;
            printf("E5e eager, %d streams of B/%d:        %7.2f us/step (whole batch)\n", nsplit, nsplit, us);
            CK(hipDeviceSynchronize());
            for (int i = 0; i < nsplit; ++i) { hipFree(ha[i]); hipFree(hb[i]); hipFree(hact[i]); hipFree(hex[i]); hipFree(hco[i]); }
            oc_destroy(hh);
        }
    }
    {  // E6: product oc_step_n, 100 steps per launch, full trajectory + exec + coll + stats
        const int N6 = 100;
        uint8_t *act6, *traj6, *ex6, *co6;
        CK(hipMalloc(&act6, (int64_t)N6 * A * P));
        CK(hipMalloc(&traj6, (int64_t)N6 * NP * P));
        CK(hipMalloc(&ex6, (int64_t)N6 * A * P));
        CK(hipMalloc(&co6, (int64_t)N6 * P));
        for (int r = 0; r < N6; ++r) oc_gen_actions(h, act6 + (int64_t)r * A * P, B, 0, r, 1, nullptr);
        const double us = timeit([&] { oc_step_n(h, sa, sb, act6, traj6, ex6, co6, stats, B, N6, nullptr); }, 5) / N6;
        printf("E6 product oc_step_n x%d + traj      : %7.2f us/step\n", N6, us);
        const double us2 = timeit([&] { oc_step_n(h, sa, sb, act6, nullptr, nullptr, nullptr, nullptr, B, N6, nullptr); }, 5) / N6;
        printf("E6b oc_step_n x%d, no outputs        : %7.2f us/step\n", N6, us2);
        hipFree(act6); hipFree(traj6); hipFree(ex6); hipFree(co6);
    }
    for (int grid : {256, 512, 1024}) {
        const double us = timeit([&] { hipLaunchKernelGGL((mem_only<2, 4>), dim3(grid), dim3(kBlock), 0, 0, L, sa, sb, act, ex, coll); }, 50);
        printf("E2 memory only           grid %4d: %7.2f us\n", grid, us);
    }
    for (int grid : {256, 512, 768, 1024}) {
        const double us = timeit([&] { hipLaunchKernelGGL((fused<2, 4>), dim3(grid), dim3(kBlock), 0, 0, L, sa, sb, act, nullptr, R); }, 20) / R;
        printf("E3 fused x%d, no traj     grid %4d: %7.2f us/step\n", R, grid, us);
    }
    for (int grid : {256, 512, 768, 1024}) {
        const double us = timeit([&] { hipLaunchKernelGGL((fused<2, 4>), dim3(grid), dim3(kBlock), 0, 0, L, sa, sb, act, traj, R); }, 20) / R;
        const double fb = (double)B * (17.0 + 2 + 2 + 1) + 17.0 * B / R;
        printf("E4 fused x%d + trajectory grid %4d: %7.2f us/step  (%.1f B/env-step actual, %6.2f TB/s)\n", R, grid, us,
               fb / B, fb / us / 1e6);
    }
    return 0;
}
