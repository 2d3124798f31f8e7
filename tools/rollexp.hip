// tools/rollexp.hip -- oc_rollout load-width and row-order experiments (includes the engine TU).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o tools/rollexp tools/rollexp.hip
// Workload: bench.py's C5 rows -- full-divider_salad, 4 agents, 2^18 rows of random-play states,
// 64 Salad configurations, configuration-major (then shuffled) allocation ids, random joint actions.
// Variants:
//   product  oc_rollout_kernel: one row per lane, one u8 load per state plane (64 B per wave
//            load instruction)
//   rpl4     4 consecutive rows per lane: one dword load per plane (256 B per wave instruction),
//            the rows run one after another, outputs gathered into dwords and stored once
//   sorted NT  rows reordered by configuration inside blocks of NT threads (counting sort of the
//              block's alloc ids in LDS), timed on configuration-major and on shuffled alloc ids
// The variant's next states, flags and bounds are compared with the product's.
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <random>
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

// Rows reordered by configuration inside each block of NT threads: a counting sort of the
// tile's NT alloc ids in LDS, then lane t runs the tile's t-th row in configuration order, so a
// wave's rows share few configurations whatever the caller's row order.  Row i's outputs still
// go to row i: results identical to the product's.
template <int A, int K, int NT>
__global__ __launch_bounds__(NT) void rollout_sorted(RollArgs R, const uint8_t* __restrict__ sin, uint8_t* __restrict__ sout,
                                                     const uint8_t* __restrict__ act, const uint8_t* __restrict__ alloc,
                                                     const uint8_t* __restrict__ blob_g, uint8_t* __restrict__ out_flags,
                                                     float* __restrict__ lb) {
    extern __shared__ uint32_t blob_w[];
    __shared__ ocro::Sub subs[OC_MAX_SUBTASKS];
    __shared__ uint32_t hist[OC_MAX_SUBTASKS + 2];
    __shared__ uint16_t order[NT];
    for (int i = threadIdx.x; i < R.blob_words; i += NT) blob_w[i] = ((const uint32_t*)blob_g)[i];
    constexpr int kSubWords = (int)(sizeof(ocro::Sub) / 4);
    for (int i = threadIdx.x; i < R.nsub * kSubWords; i += NT) ((uint32_t*)subs)[i] = ((const uint32_t*)R.subs)[i];
    const uint8_t* blob = (const uint8_t*)blob_w;
    const int64_t P = R.pitch;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    const int nb = R.nsub + 2;  // buckets: configurations, bad alloc ids, rows past B
    for (int64_t tile = (int64_t)blockIdx.x * NT; tile < R.B; tile += (int64_t)gridDim.x * NT) {
        if ((int)threadIdx.x < nb) hist[threadIdx.x] = 0u;
        __syncthreads();
        const int64_t e0 = tile + threadIdx.x;
        const int b = e0 >= R.B ? nb - 1 : min(alloc != nullptr ? (int)alloc[e0] : 0, R.nsub);
        const uint32_t rank = atomicAdd(&hist[b], 1u);
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of <= 66 buckets by one wave: 2 per lane
            const int l = threadIdx.x;
            const uint32_t c0 = 2 * l < nb ? hist[2 * l] : 0u, c1 = 2 * l + 1 < nb ? hist[2 * l + 1] : 0u;
            uint32_t inc = c0 + c1;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t o = __shfl_up(inc, off);
                if (l >= off) inc += o;
            }
            const uint32_t ex = inc - c0 - c1;
            if (2 * l < nb) hist[2 * l] = ex;
            if (2 * l + 1 < nb) hist[2 * l + 1] = ex + c0;
        }
        __syncthreads();
        order[hist[b] + rank] = (uint16_t)threadIdx.x;
        __syncthreads();
        const int64_t e = tile + order[threadIdx.x];
        if (e < R.B) {
            ocro::Row r = load_row<A, K>(sin, P, e);
            const uint16_t t = ((const uint16_t*)(sin + kPT * P))[e];
            const uint8_t fl_in = sin[kPF * P + e];
            const int ai = alloc != nullptr ? alloc[e] : 0;
            float bound = 0.0f;
            int f = OC_ROLL_BADALLOC;
            if (ai < R.nsub) {
                const ocro::Sub& sb = subs[ai];
                const int c0 = act[sb.agent[0] * P + e], c1 = sb.n == 2 ? act[sb.agent[1] * P + e] : ocro::kNoop;
                ocro::RowOps<A, K> ops(R.L, blob);
                f = ops.run(r, sb, c0, c1, bound);
            }
#pragma unroll
            for (int a = 0; a < A; ++a) {
                sout[a * P + e] = (uint8_t)r.ax(a);
                sout[(kPY + a) * P + e] = (uint8_t)r.ay(a);
                sout[(kPH + a) * P + e] = (uint8_t)r.ah(a);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                sout[(kPL + j) * P + e] = (uint8_t)r.il(j);
                sout[(kPM + j) * P + e] = (uint8_t)r.im(j);
            }
            ((uint16_t*)(sout + kPT * P))[e] = t;
            sout[kPF * P + e] = fl_in;
            out_flags[e] = (uint8_t)f;
            lb[e] = bound;
        }
        __syncthreads();
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
    auto time = [&](const char* name, auto&& fn) {  // fn(0): the timed launch
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
    std::vector<uint8_t> o0(S), o1(S), f0(B), f1(B);
    std::vector<float> l0(B), l1(B);
    auto same = [&]() {
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(o0.data(), out[0], S, hipMemcpyDeviceToHost)); CK(hipMemcpy(o1.data(), out[1], S, hipMemcpyDeviceToHost));
        CK(hipMemcpy(f0.data(), fl[0], B, hipMemcpyDeviceToHost)); CK(hipMemcpy(f1.data(), fl[1], B, hipMemcpyDeviceToHost));
        CK(hipMemcpy(l0.data(), lbd[0], 4 * B, hipMemcpyDeviceToHost)); CK(hipMemcpy(l1.data(), lbd[1], 4 * B, hipMemcpyDeviceToHost));
        return o0 == o1 && f0 == f1 && l0 == l1;
    };
    std::vector<uint8_t> al_rnd(al);
    {
        std::mt19937 g(7);
        for (int64_t e = B - 1; e > 0; --e) std::swap(al_rnd[e], al_rnd[g() % (e + 1)]);
    }
    for (int order_i = 0; order_i < 2; ++order_i) {
        CK(hipMemcpy(alloc, order_i ? al_rnd.data() : al.data(), P, hipMemcpyHostToDevice));
        const char* on = order_i ? "random order" : "configuration-major";
        char name[96];
        snprintf(name, sizeof name, "product (row per lane), %s", on);
        time(name, product);
        auto s256 = [&](int v) {
            hipLaunchKernelGGL((rollout_sorted<4, 4, 256>), dim3((unsigned)((B + 255) / 256)), dim3(256), h->roll_blob_bytes,
                               nullptr, R, s0, out[v], acts, alloc, h->roll_blob, fl[v], lbd[v]);
        };
        auto s1024 = [&](int v) {
            hipLaunchKernelGGL((rollout_sorted<4, 4, 1024>), dim3((unsigned)((B + 1023) / 1024)), dim3(1024),
                               h->roll_blob_bytes, nullptr, R, s0, out[v], acts, alloc, h->roll_blob, fl[v], lbd[v]);
        };
        {
            const int64_t need = (B / 4 + kBlock - 1) / kBlock, cap = (int64_t)h->cus * 4;
            auto v4 = [&](int v) {
                hipLaunchKernelGGL((rollout_rpl4<4, 4>), dim3((unsigned)(need < cap ? need : cap)), dim3(kBlock),
                                   h->roll_blob_bytes, nullptr, R, s0, out[v], acts, alloc, h->roll_blob, fl[v], lbd[v]);
            };
            snprintf(name, sizeof name, "rpl4 (4 rows per lane, dword loads), %s", on);
            time(name, v4);
            product(0); v4(1);
            printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        }
        snprintf(name, sizeof name, "sorted in 256-row blocks, %s", on);
        time(name, s256);
        product(0); s256(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        auto s512 = [&](int v) {
            hipLaunchKernelGGL((rollout_sorted<4, 4, 512>), dim3((unsigned)((B + 511) / 512)), dim3(512),
                               h->roll_blob_bytes, nullptr, R, s0, out[v], acts, alloc, h->roll_blob, fl[v], lbd[v]);
        };
        snprintf(name, sizeof name, "sorted in 512-row blocks, %s", on);
        time(name, s512);
        product(0); s512(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
        snprintf(name, sizeof name, "sorted in 1024-row blocks, %s", on);
        time(name, s1024);
        product(0); s1024(1);
        printf("  outputs %s\n", same() ? "identical" : "DIFFER");
    }
    return 0;
}
