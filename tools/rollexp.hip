// tools/rollexp.hip -- oc_rollout load-width experiment (includes the engine TU).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o tools/rollexp tools/rollexp.hip
// Workload: bench.py's C5 rows -- full-divider_salad, 4 agents, 2^18 rows of random-play states,
// 64 Salad configurations, configuration-major allocation ids, random joint actions.
// Variants:
//   product  oc_rollout_kernel: one row per lane, one u8 load per state plane (64 B per wave
//            load instruction)
//   rpl4     4 consecutive rows per lane: one dword load per plane (256 B per wave instruction),
//            the rows run one after another, outputs gathered into dwords and stored once
// The variant's next states, flags and bounds are compared with the product's.
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

template <int A, int K>
__global__ __launch_bounds__(kBlock) void rollout_rpl4(RollArgs R, const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                                       const uint8_t* __restrict__ act, const uint8_t* __restrict__ alloc,
                                                       const uint8_t* __restrict__ blob_g, uint8_t* __restrict__ out_flags,
                                                       float* __restrict__ lb) {
    extern __shared__ uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    stage_roll_tables(R, blob_g, blob_w, subs);
    const uint8_t* blob = (const uint8_t*)blob_w;
    const int64_t P = R.pitch;
    constexpr int NP = 3 * A + 2 * K + 3;
    const int64_t nq = (R.B + 3) / 4;
    for (int64_t g = blockIdx.x * (int64_t)kBlock + threadIdx.x; g < nq; g += (int64_t)gridDim.x * kBlock) {
        uint32_t w[NP - 3], wa[A], o[NP - 3];
        for (int p = 0; p < NP - 3; ++p) w[p] = ((const uint32_t*)(sin + p * P))[g];
        for (int a = 0; a < A; ++a) wa[a] = ((const uint32_t*)(act + a * P))[g];
        const uint32_t wal = ((const uint32_t*)alloc)[g];
        uint32_t fl4 = 0;
        float b4[4];
        for (int q = 0; q < 4; ++q) {
            ocro::Row r;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                r.x |= ((w[a] >> (8 * q)) & 0xFFu) << (8 * a);
                r.y |= ((w[A + a] >> (8 * q)) & 0xFFu) << (8 * a);
                r.h |= ((w[2 * A + a] >> (8 * q)) & 0xFFu) << (8 * a);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                r.loc |= (uint64_t)((w[3 * A + j] >> (8 * q)) & 0xFFu) << (8 * j);
                r.mask |= (uint64_t)((w[3 * A + K + j] >> (8 * q)) & 0xFFu) << (8 * j);
            }
            const int ai = (int)((wal >> (8 * q)) & 0xFFu);
            float bound = 0.0f;
            int f = OC_ROLL_BADALLOC;
            if (ai < R.nsub) {
                const ocro::Sub& s = subs[ai];
                const int c0 = (int)((wa[s.agent[0]] >> (8 * q)) & 0xFFu);
                const int c1 = s.n == 2 ? (int)((wa[s.agent[1]] >> (8 * q)) & 0xFFu) : ocro::kNoop;
                ocro::RowOps<A, K> ops(R.L, blob);
                f = ops.run(r, s, c0, c1, bound);
            }
            const uint32_t keep = ~(0xFFu << (8 * q));
#pragma unroll
            for (int a = 0; a < A; ++a) {
                o[a] = (q ? o[a] & keep : 0u) | ((uint32_t)r.ax(a) << (8 * q));
                o[A + a] = (q ? o[A + a] & keep : 0u) | ((uint32_t)r.ay(a) << (8 * q));
                o[2 * A + a] = (q ? o[2 * A + a] & keep : 0u) | ((uint32_t)r.ah(a) << (8 * q));
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                o[3 * A + j] = (q ? o[3 * A + j] & keep : 0u) | ((uint32_t)r.il(j) << (8 * q));
                o[3 * A + K + j] = (q ? o[3 * A + K + j] & keep : 0u) | ((uint32_t)r.im(j) << (8 * q));
            }
            fl4 |= (uint32_t)f << (8 * q);
            b4[q] = bound;
        }
        for (int p = 0; p < NP - 3; ++p) ((uint32_t*)(sout + p * P))[g] = o[p];
        ((uint2*)(sout + (NP - 3) * P))[g] = ((const uint2*)(sin + (NP - 3) * P))[g];  // t (u16 x 4)
        ((uint32_t*)(sout + (NP - 1) * P))[g] = ((const uint32_t*)(sin + (NP - 1) * P))[g];
        ((uint32_t*)out_flags)[g] = fl4;
        ((float4*)lb)[g] = make_float4(b4[0], b4[1], b4[2], b4[3]);
    }
}

}  // namespace

int main() {
    const int64_t B = 1 << 18;
    // full-divider_salad (levels.py builtin): 7x7, 4 agents
    const char* rows[7] = {"-----t-", "/  -  l", "/  -  -", "*  -  -", "-  -  -", "-  -  p", "-----p-"};
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
    if (oc_create(&lv, 4, 100, 0, &h) != 0) { printf("create: %s\n", oc_last_error()); return 1; }
    oc_layout lay;
    oc_get_layout(h, B, &lay);
    const int64_t S = lay.state_bytes, P = lay.pitch;
    uint8_t *s0, *s1, *acts, *alloc, *out[2], *fl[2];
    float* lbd[2];
    CK(hipMalloc(&s0, S)); CK(hipMalloc(&s1, S)); CK(hipMalloc(&acts, 4 * P)); CK(hipMalloc(&alloc, P));
    for (int v = 0; v < 2; ++v) { CK(hipMalloc(&out[v], S)); CK(hipMalloc(&fl[v], P)); CK(hipMalloc(&lbd[v], 4 * P)); }
    oc_reset(h, s0, B, nullptr);
    for (int r = 0; r < 37; ++r) {
        oc_gen_actions(h, acts, B, 0, r, 11, nullptr);
        oc_step(h, r & 1 ? s1 : s0, r & 1 ? s0 : s1, acts, nullptr, nullptr, nullptr, B, nullptr);
    }
    CK(hipMemcpy(s0, s1, S, hipMemcpyDeviceToDevice));
    oc_gen_actions(h, acts, B, 0, 99, 12, nullptr);
    // 64 Salad configurations (bench.py SALAD_SUBTASKS x agent sets), configuration-major rows
    const int kinds[9] = {1, 1, 2, 2, 2, 2, 2, 2, 3};
    const uint8_t st0[9] = {0x01, 0x02, 0x11, 0x11, 0x22, 0x33, 0x19, 0x2A, 0x3B}, st1[9] = {0, 0, 0x22, 0x08, 0x08, 0x08, 0x22, 0x11, 0};
    const uint8_t goal[9] = {0x11, 0x22, 0x33, 0x19, 0x2A, 0x3B, 0x3B, 0x3B, 0x3B};
    std::vector<oc_subtask> subs;
    const int sets[10][2] = {{0, -1}, {1, -1}, {2, -1}, {3, -1}, {0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
    for (int k = 0; k < 9 && (int)subs.size() < 64; ++k)
        for (int a = 0; a < 10 && (int)subs.size() < 64; ++a) {
            oc_subtask t{};
            t.kind = kinds[k]; t.num_agents = sets[a][1] < 0 ? 1 : 2;
            t.agent[0] = (uint8_t)sets[a][0]; t.agent[1] = (uint8_t)(sets[a][1] < 0 ? 0 : sets[a][1]);
            t.start_mask[0] = st0[k]; t.start_mask[1] = st1[k]; t.goal_mask = goal[k];
            subs.push_back(t);
        }
    std::vector<uint8_t> al(P, 0);
    for (int64_t e = 0; e < B; ++e) al[e] = (uint8_t)(e * (int64_t)subs.size() / B);
    CK(hipMemcpy(alloc, al.data(), P, hipMemcpyHostToDevice));
    RollArgs R;
    if (roll_args(h, subs.data(), (int)subs.size(), B, R, true)) { printf("args: %s\n", oc_last_error()); return 1; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto time = [&](const char* name, auto&& fn) {
        for (int i = 0; i < 3; ++i) fn(0);
        CK(hipEventRecord(e0));
        for (int i = 0; i < 50; ++i) fn(0);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.2f us/launch\n", name, ms * 1e3 / 50);
    };
    auto product = [&](int v) {
        oc_rollout(h, s0, out[v], acts, alloc, subs.data(), (int)subs.size(), fl[v], lbd[v], B, nullptr);
    };
    time("product (row per lane, u8 plane loads)", product);
    for (int bpc : {1, 2, 4, 8}) {
        const int64_t need = (B / 4 + kBlock - 1) / kBlock, cap = (int64_t)h->cus * bpc;
        const dim3 grid((unsigned)(need < cap ? need : cap));
        char name[80];
        snprintf(name, sizeof name, "rpl4 (4 rows per lane, dword loads), <= %d/CU", bpc);
        auto v4 = [&](int v) {
            hipLaunchKernelGGL((rollout_rpl4<4, 4>), grid, dim3(kBlock), h->roll_blob_bytes, nullptr, R, s0, out[1], acts,
                               alloc, h->roll_blob, fl[1], lbd[1]);
        };
        time(name, v4);
    }
    product(0);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> o0(S), o1(S), f0(B), f1(B);
    std::vector<float> l0(B), l1(B);
    CK(hipMemcpy(o0.data(), out[0], S, hipMemcpyDeviceToHost)); CK(hipMemcpy(o1.data(), out[1], S, hipMemcpyDeviceToHost));
    CK(hipMemcpy(f0.data(), fl[0], B, hipMemcpyDeviceToHost)); CK(hipMemcpy(f1.data(), fl[1], B, hipMemcpyDeviceToHost));
    CK(hipMemcpy(l0.data(), lbd[0], 4 * B, hipMemcpyDeviceToHost)); CK(hipMemcpy(l1.data(), lbd[1], 4 * B, hipMemcpyDeviceToHost));
    printf("outputs %s\n", (o0 == o1 && f0 == f1 && l0 == l1) ? "identical" : "DIFFER");
    return 0;
}
