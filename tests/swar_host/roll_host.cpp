// TEST INFRASTRUCTURE: host build of the device rollout row (gym-cooking_amd/csrc/oc_rollout.h)
// so its logic can be checked against the CPU oracle and the reference rows without a GPU.
// The loop mirrors oc_rollout_kernel's plane loads and stores; the product library never
// contains this file.
#include <math.h>
#include <stdint.h>

#define __device__
#define __host__

#include "../../gym-cooking_amd/csrc/oc_rollout.h"
#include "../../include/oc_engine.h"

template <int A, int K>
static void run(const oc_level_desc* lv, const uint8_t* sin, uint8_t* sout, const uint8_t* act, const uint8_t* alloc,
                const oc_subtask* subs, int nsub, uint8_t* flags, float* lb, int64_t B, int64_t P) {
    static uint8_t blob[ocro::kBlobMax];
    ocro::RollLevel L;
    if (ocro::build_roll_level(L, blob, lv->width, lv->height, lv->tiles, lv->encoding) < 0) return;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K, kPF = kPT + 2;
    for (int64_t e = 0; e < B; ++e) {
        ocro::RowT<K> r;
        for (int a = 0; a < A; ++a) {
            r.x |= (uint32_t)sin[a * P + e] << (8 * a);
            r.y |= (uint32_t)sin[(kPY + a) * P + e] << (8 * a);
            r.h |= (uint32_t)sin[(kPH + a) * P + e] << (8 * a);
        }
        for (int j = 0; j < K; ++j) {
            r.loc[j >> 3] |= (uint64_t)sin[(kPL + j) * P + e] << (8 * (j & 7));
            r.mask[j >> 3] |= (uint64_t)sin[(kPM + j) * P + e] << (8 * (j & 7));
        }
        const int ai = alloc ? alloc[e] : 0;
        float bound = 0.0f;
        int f = OC_ROLL_BADALLOC;
        if (ai < nsub) {
            const oc_subtask& o = subs[ai];
            ocro::Sub s{o.kind, o.num_agents, {o.agent[0], (uint8_t)(o.num_agents == 2 ? o.agent[1] : o.agent[0])},
                        {o.start_mask[0], o.start_mask[1]}, o.goal_mask, o.goal_count, o.level, 0};
            const int c0 = act[s.agent[0] * P + e], c1 = s.n == 2 ? act[s.agent[1] * P + e] : ocro::kNoop;
            ocro::RowOps<A, K> ops(L, blob);
            f = ops.run(r, s, c0, c1, bound);
        }
        for (int a = 0; a < A; ++a) {
            sout[a * P + e] = (uint8_t)r.ax(a);
            sout[(kPY + a) * P + e] = (uint8_t)r.ay(a);
            sout[(kPH + a) * P + e] = (uint8_t)r.ah(a);
        }
        for (int j = 0; j < K; ++j) {
            sout[(kPL + j) * P + e] = (uint8_t)r.il(j);
            sout[(kPM + j) * P + e] = (uint8_t)r.im(j);
        }
        sout[kPT * P + 2 * e] = sin[kPT * P + 2 * e];
        sout[kPT * P + 2 * e + 1] = sin[kPT * P + 2 * e + 1];
        sout[kPF * P + e] = sin[kPF * P + e];
        flags[e] = (uint8_t)f;
        lb[e] = bound;
    }
}

template <int A, int K>
static void lik(const oc_level_desc* lv, const uint8_t* sin, const uint8_t* taken_p, const uint8_t* alloc,
                const oc_subtask* subs, int nsub, int self_agent, double beta, double nap, double* out, uint8_t* flags,
                int64_t B, int64_t P) {
    static uint8_t blob[ocro::kBlobMax];
    ocro::RollLevel L;
    if (ocro::build_roll_level(L, blob, lv->width, lv->height, lv->tiles, lv->encoding) < 0) return;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K;
    for (int64_t e = 0; e < B; ++e) {
        const int ai = alloc ? alloc[e] : 0;
        double v = 0.0;
        int f = OC_LIK_BADALLOC;
        if (ai < nsub) {
            ocro::RowT<K> r;
            for (int a = 0; a < A; ++a) {
                r.x |= (uint32_t)sin[a * P + e] << (8 * a);
                r.y |= (uint32_t)sin[(kPY + a) * P + e] << (8 * a);
                r.h |= (uint32_t)sin[(kPH + a) * P + e] << (8 * a);
            }
            for (int j = 0; j < K; ++j) {
                r.loc[j >> 3] |= (uint64_t)sin[(kPL + j) * P + e] << (8 * (j & 7));
                r.mask[j >> 3] |= (uint64_t)sin[(kPM + j) * P + e] << (8 * (j & 7));
            }
            uint32_t taken = 0;
            for (int a = 0; a < A; ++a) taken |= (uint32_t)taken_p[a * P + e] << (8 * a);
            const oc_subtask& o = subs[ai];
            ocro::Sub s{o.kind, o.num_agents, {o.agent[0], (uint8_t)(o.num_agents == 2 ? o.agent[1] : o.agent[0])},
                        {o.start_mask[0], o.start_mask[1]}, o.goal_mask, o.goal_count, o.level, 0};
            ocro::RowOps<A, K> ops(L, blob);
            f = ops.likelihood(r, s, taken, self_agent, beta, nap, v);
        }
        out[e] = f == OC_LIK_OK ? v : 0.0;
        flags[e] = (uint8_t)f;
    }
}

extern "C" int lik_host(const oc_level_desc* lv, int A, int K, const uint8_t* sin, const uint8_t* taken,
                        const uint8_t* alloc, const oc_subtask* subs, int nsub, int self_agent, double beta, double nap,
                        double* out, uint8_t* flags, int64_t B, int64_t P) {
#define L_(a, k) \
    if (A == a && K == k) { lik<a, k>(lv, sin, taken, alloc, subs, nsub, self_agent, beta, nap, out, flags, B, P); return 0; }
    L_(1, 4) L_(2, 4) L_(3, 4) L_(4, 4) L_(1, 8) L_(2, 8) L_(3, 8) L_(4, 8) L_(1, 16) L_(2, 16) L_(3, 16) L_(4, 16)
#undef L_
    return -1;
}

extern "C" int roll_host(const oc_level_desc* lv, int A, int K, const uint8_t* sin, uint8_t* sout, const uint8_t* act,
                         const uint8_t* alloc, const oc_subtask* subs, int nsub, uint8_t* flags, float* lb, int64_t B,
                         int64_t P) {
#define R_(a, k) \
    if (A == a && K == k) { run<a, k>(lv, sin, sout, act, alloc, subs, nsub, flags, lb, B, P); return 0; }
    R_(1, 4) R_(2, 4) R_(3, 4) R_(4, 4) R_(1, 8) R_(2, 8) R_(3, 8) R_(4, 8) R_(1, 16) R_(2, 16) R_(3, 16) R_(4, 16)
#undef R_
    return -1;
}

// oc_bounds_kernel's loop: every env x every configuration, [subtask][pitch] outputs
template <int A, int K>
static void bounds(const oc_level_desc* lv, const uint8_t* sin, const oc_subtask* subs, int nsub, float* lb,
                   uint8_t* doable, int64_t B, int64_t P) {
    static uint8_t blob[ocro::kBlobMax];
    ocro::RollLevel L;
    if (ocro::build_roll_level(L, blob, lv->width, lv->height, lv->tiles, lv->encoding) < 0) return;
    constexpr int kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K;
    for (int64_t e = 0; e < B; ++e) {
        ocro::RowT<K> r;
        for (int a = 0; a < A; ++a) {
            r.x |= (uint32_t)sin[a * P + e] << (8 * a);
            r.y |= (uint32_t)sin[(kPY + a) * P + e] << (8 * a);
            r.h |= (uint32_t)sin[(kPH + a) * P + e] << (8 * a);
        }
        for (int j = 0; j < K; ++j) {
            r.loc[j >> 3] |= (uint64_t)sin[(kPL + j) * P + e] << (8 * (j & 7));
            r.mask[j >> 3] |= (uint64_t)sin[(kPM + j) * P + e] << (8 * (j & 7));
        }
        ocro::RowOps<A, K> ops(L, blob);
        for (int i = 0; i < nsub; ++i) {
            const oc_subtask& o = subs[i];
            ocro::Sub s{o.kind, o.num_agents, {o.agent[0], (uint8_t)(o.num_agents == 2 ? o.agent[1] : o.agent[0])},
                        {o.start_mask[0], o.start_mask[1]}, o.goal_mask, o.goal_count, o.level, 0};
            float v;
            doable[i * P + e] = ops.full_bound(r, s, v) ? 1 : 0;
            lb[i * P + e] = v;
        }
    }
}

extern "C" int bounds_host(const oc_level_desc* lv, int A, int K, const uint8_t* sin, const oc_subtask* subs, int nsub,
                           float* lb, uint8_t* doable, int64_t B, int64_t P) {
#define B_(a, k) \
    if (A == a && K == k) { bounds<a, k>(lv, sin, subs, nsub, lb, doable, B, P); return 0; }
    B_(1, 4) B_(2, 4) B_(3, 4) B_(4, 4) B_(1, 8) B_(2, 8) B_(3, 8) B_(4, 8) B_(1, 16) B_(2, 16) B_(3, 16) B_(4, 16)
#undef B_
    return -1;
}
