// TEST INFRASTRUCTURE: host build of the device rollout row (gym-cooking_amd/csrc/oc_rollout.h)
// so its logic can be checked against the CPU oracle and the reference rows without a GPU.
// The loop mirrors oc_rollout_kernel's plane loads and stores; the product library never
// contains this file.
#include <vector>
#include <math.h>
#include <stdint.h>

#define __device__
#define __host__

#include "../../gym-cooking_amd/csrc/oc_rollout.h"
#include "../../include/oc_engine.h"

// the planes of oc_layout (a wide level: the item cells' high bytes in K planes after the low)
template <int A, int K, bool W>
struct PL {
    static constexpr int Y = A, H = 2 * A, L = 3 * A, LH = 3 * A + K, M = 3 * A + (W ? 2 : 1) * K, T = M + K, F = T + 2;
};

template <int A, int K, bool W>
static ocro::RowT<K, W> load(const uint8_t* sin, int64_t P, int64_t e) {
    using Pl = PL<A, K, W>;
    ocro::RowT<K, W> r;
    for (int a = 0; a < A; ++a) {
        r.x |= (uint32_t)sin[a * P + e] << (8 * a);
        r.y |= (uint32_t)sin[(Pl::Y + a) * P + e] << (8 * a);
        r.h |= (uint32_t)sin[(Pl::H + a) * P + e] << (8 * a);
    }
    for (int j = 0; j < K; ++j) {
        r.set_loc(j, (uint32_t)sin[(Pl::L + j) * P + e] | (W ? (uint32_t)sin[(Pl::LH + j) * P + e] << 8 : 0u));
        r.set_mask(j, sin[(Pl::M + j) * P + e]);
    }
    return r;
}

template <int A, int K, bool W>
static void run(const oc_level_desc* lv, const uint8_t* sin, uint8_t* sout, const uint8_t* act, const uint8_t* alloc,
                const oc_subtask* subs, int nsub, uint8_t* flags, float* lb, int64_t B, int64_t P) {
    std::vector<uint8_t> blob_v;
    ocro::RollLevel L;
    if (ocro::build_roll_level(L, blob_v, lv->width, lv->height, lv->tiles, lv->encoding) < 0) return;
    const uint8_t* blob = blob_v.data();
    using Pl = PL<A, K, W>;
    for (int64_t e = 0; e < B; ++e) {
        ocro::RowT<K, W> r = load<A, K, W>(sin, P, e);
        const int ai = alloc ? alloc[e] : 0;
        float bound = 0.0f;
        int f = OC_ROLL_BADALLOC;
        if (ai < nsub) {
            const oc_subtask& o = subs[ai];
            ocro::Sub s{o.kind, o.num_agents, {o.agent[0], (uint8_t)(o.num_agents == 2 ? o.agent[1] : o.agent[0])},
                        {o.start_mask[0], o.start_mask[1]}, o.goal_mask, o.goal_count, o.level, 0};
            const int c0 = act[s.agent[0] * P + e], c1 = s.n == 2 ? act[s.agent[1] * P + e] : ocro::kNoop;
            ocro::RowOps<A, K, W, false, true> ops(L, blob);
            ops.PT = L.pair_off ? (const uint32_t*)(blob + L.pair_off) : nullptr;  // the agent-pair table
            f = ops.run(r, s, c0, c1, bound);
        }
        for (int a = 0; a < A; ++a) {
            sout[a * P + e] = (uint8_t)r.ax(a);
            sout[(Pl::Y + a) * P + e] = (uint8_t)r.ay(a);
            sout[(Pl::H + a) * P + e] = (uint8_t)r.ah(a);
        }
        for (int j = 0; j < K; ++j) {
            sout[(Pl::L + j) * P + e] = (uint8_t)r.il(j);
            if (W) sout[(Pl::LH + j) * P + e] = (uint8_t)(r.il(j) >> 8);
            sout[(Pl::M + j) * P + e] = (uint8_t)r.im(j);
        }
        sout[Pl::T * P + 2 * e] = sin[Pl::T * P + 2 * e];
        sout[Pl::T * P + 2 * e + 1] = sin[Pl::T * P + 2 * e + 1];
        sout[Pl::F * P + e] = sin[Pl::F * P + e];
        flags[e] = (uint8_t)f;
        lb[e] = bound;
    }
}

template <int A, int K, bool W>
static void lik(const oc_level_desc* lv, const uint8_t* sin, const uint8_t* taken_p, const uint8_t* alloc,
                const oc_subtask* subs, int nsub, int self_agent, double beta, double nap, double* out, uint8_t* flags,
                int64_t B, int64_t P) {
    std::vector<uint8_t> blob_v;
    ocro::RollLevel L;
    if (ocro::build_roll_level(L, blob_v, lv->width, lv->height, lv->tiles, lv->encoding) < 0) return;
    const uint8_t* blob = blob_v.data();
    for (int64_t e = 0; e < B; ++e) {
        const int ai = alloc ? alloc[e] : 0;
        double v = 0.0;
        int f = OC_LIK_BADALLOC;
        if (ai < nsub) {
            ocro::RowT<K, W> r = load<A, K, W>(sin, P, e);
            uint32_t taken = 0;
            for (int a = 0; a < A; ++a) taken |= (uint32_t)taken_p[a * P + e] << (8 * a);
            const oc_subtask& o = subs[ai];
            ocro::Sub s{o.kind, o.num_agents, {o.agent[0], (uint8_t)(o.num_agents == 2 ? o.agent[1] : o.agent[0])},
                        {o.start_mask[0], o.start_mask[1]}, o.goal_mask, o.goal_count, o.level, 0};
            ocro::RowOps<A, K, W, true, true> ops(L, blob);  // the likelihood kernels' lean flavour
            ops.PT = L.pair_off ? (const uint32_t*)(blob + L.pair_off) : nullptr;
            f = ops.likelihood(r, s, taken, self_agent, beta, nap, v);
        }
        out[e] = f == OC_LIK_OK ? v : 0.0;
        flags[e] = (uint8_t)f;
    }
}

extern "C" int lik_host(const oc_level_desc* lv, int A, int K, const uint8_t* sin, const uint8_t* taken,
                        const uint8_t* alloc, const oc_subtask* subs, int nsub, int self_agent, double beta, double nap,
                        double* out, uint8_t* flags, int64_t B, int64_t P) {
    const bool wide = lv->width * lv->height > OC_MAX_NARROW_CELLS;
#define L_(a, k)                                                                                                   \
    if (A == a && K == k) {                                                                                       \
        if (wide) lik<a, k, true>(lv, sin, taken, alloc, subs, nsub, self_agent, beta, nap, out, flags, B, P);    \
        else lik<a, k, false>(lv, sin, taken, alloc, subs, nsub, self_agent, beta, nap, out, flags, B, P);        \
        return 0;                                                                                                 \
    }
    L_(1, 4) L_(2, 4) L_(3, 4) L_(4, 4) L_(1, 8) L_(2, 8) L_(3, 8) L_(4, 8) L_(1, 16) L_(2, 16) L_(3, 16) L_(4, 16)
#undef L_
    return -1;
}

extern "C" int roll_host(const oc_level_desc* lv, int A, int K, const uint8_t* sin, uint8_t* sout, const uint8_t* act,
                         const uint8_t* alloc, const oc_subtask* subs, int nsub, uint8_t* flags, float* lb, int64_t B,
                         int64_t P) {
    const bool wide = lv->width * lv->height > OC_MAX_NARROW_CELLS;
#define R_(a, k)                                                                                 \
    if (A == a && K == k) {                                                                     \
        if (wide) run<a, k, true>(lv, sin, sout, act, alloc, subs, nsub, flags, lb, B, P);     \
        else run<a, k, false>(lv, sin, sout, act, alloc, subs, nsub, flags, lb, B, P);         \
        return 0;                                                                               \
    }
    R_(1, 4) R_(2, 4) R_(3, 4) R_(4, 4) R_(1, 8) R_(2, 8) R_(3, 8) R_(4, 8) R_(1, 16) R_(2, 16) R_(3, 16) R_(4, 16)
#undef R_
    return -1;
}

// oc_bounds_kernel's loop: every env x every configuration, [subtask][pitch] outputs
template <int A, int K, bool W>
static void bounds(const oc_level_desc* lv, const uint8_t* sin, const oc_subtask* subs, int nsub, float* lb,
                   uint8_t* doable, int64_t B, int64_t P) {
    std::vector<uint8_t> blob_v;
    ocro::RollLevel L;
    if (ocro::build_roll_level(L, blob_v, lv->width, lv->height, lv->tiles, lv->encoding) < 0) return;
    const uint8_t* blob = blob_v.data();
    for (int64_t e = 0; e < B; ++e) {
        const ocro::RowT<K, W> r = load<A, K, W>(sin, P, e);
        ocro::RowOps<A, K, W, false, true> ops(L, blob);
            ops.PT = L.pair_off ? (const uint32_t*)(blob + L.pair_off) : nullptr;  // the agent-pair table
        const auto br = ops.template bound_row<true>(r);  // as the kernel: once per row
        for (int i = 0; i < nsub; ++i) {
            const oc_subtask& o = subs[i];
            ocro::Sub s{o.kind, o.num_agents, {o.agent[0], (uint8_t)(o.num_agents == 2 ? o.agent[1] : o.agent[0])},
                        {o.start_mask[0], o.start_mask[1]}, o.goal_mask, o.goal_count, o.level, 0};
            float v;
            doable[i * P + e] = ops.full_bound(br, r, s, v) ? 1 : 0;
            lb[i * P + e] = v;
        }
    }
}

extern "C" int bounds_host(const oc_level_desc* lv, int A, int K, const uint8_t* sin, const oc_subtask* subs, int nsub,
                           float* lb, uint8_t* doable, int64_t B, int64_t P) {
    const bool wide = lv->width * lv->height > OC_MAX_NARROW_CELLS;
#define B_(a, k)                                                                          \
    if (A == a && K == k) {                                                              \
        if (wide) bounds<a, k, true>(lv, sin, subs, nsub, lb, doable, B, P);             \
        else bounds<a, k, false>(lv, sin, subs, nsub, lb, doable, B, P);                 \
        return 0;                                                                        \
    }
    B_(1, 4) B_(2, 4) B_(3, 4) B_(4, 4) B_(1, 8) B_(2, 8) B_(3, 8) B_(4, 8) B_(1, 16) B_(2, 16) B_(3, 16) B_(4, 16)
#undef B_
    return -1;
}
