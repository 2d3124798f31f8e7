// TEST INFRASTRUCTURE: host build of the device SWAR step (gym-cooking_amd/csrc/oc_swar.h)
// so its logic can be checked against the CPU oracle without a GPU.  The two AMDGCN
// intrinsics it uses have bit-exact host restatements in the header (the host pass of
// oc_swar.h, which is also oc_cpu_step's); the product library never contains this file.
#include <stdint.h>
#include <string.h>

#define __device__
#define __host__
#define __forceinline__ inline

#include "../../gym-cooking_amd/csrc/oc_swar.h"
#include "../../include/oc_engine.h"

// n steps per call with the state kept between steps (what oc_step_n_kernel does per lane):
// the loaded state is `pending` once, later steps take the rare-event split on their own
// (any_of tests this lane's 4 envs).  n = 1 is one oc_step.  Outputs of step r go to
// sout + r * NP * P, exo + r * A * P, coll + r * P.
template <int A, int K>
static void run(const oc_level_desc* lv, int max_T, const uint8_t* sin, uint8_t* sout, const uint8_t* act,
                uint8_t* exo, uint8_t* coll, int64_t B, int64_t P, int n = 1) {
    const int W = lv->width, H = lv->height;
    int done_cell = -1;
    uint8_t tbl[256] = {0};
    for (int c = 0; c < W * H; ++c) {
        tbl[c] = ocsw::tile_class(lv->tiles[c]);
        if (lv->tiles[c] == OC_TILE_DELIVERY && done_cell < 0) done_cell = c;
    }
    uint8_t cell[16], mask[16];
    for (int j = 0; j < 16; ++j) { cell[j] = j < lv->num_items ? lv->item_cell[j] : 0xFF; mask[j] = j < lv->num_items ? lv->item_mask[j] : 0; }
    ocsw::SwarLevel S;
    ocsw::build_swar_level(S, W, H, done_cell, lv->goal_mask, lv->num_goals, max_T, lv->spawn_x, lv->spawn_y, A, cell, mask,
                           lv->encoding, lv->tiles);
    auto cls_of = [&](uint32_t cells) -> uint32_t {
        return (uint32_t)tbl[cells & 0xFF] | ((uint32_t)tbl[(cells >> 8) & 0xFF] << 8) |
               ((uint32_t)tbl[(cells >> 16) & 0xFF] << 16) | ((uint32_t)tbl[cells >> 24] << 24);
    };
    auto rd = [&](const uint8_t* base, int plane, int64_t g) { uint32_t v; memcpy(&v, base + plane * P + 4 * g, 4); return v; };
    auto wr = [&](uint8_t* base, int plane, int64_t g, uint32_t v) { memcpy(base + plane * P + 4 * g, &v, 4); };
    for (int64_t g = 0; g < (B + 3) / 4; ++g) {
        uint32_t X[A], Y[A], Hh[A], Lc[K], M[K], AC[A], EX[A], T0, T1, F, CM;
        for (int a = 0; a < A; ++a) { X[a] = rd(sin, a, g); Y[a] = rd(sin, A + a, g); Hh[a] = rd(sin, 2 * A + a, g); AC[a] = rd(act, a, g); }
        for (int j = 0; j < K; ++j) { Lc[j] = rd(sin, 3 * A + j, g); M[j] = rd(sin, 3 * A + K + j, g); }
        const int pt = 3 * A + 2 * K;
        memcpy(&T0, sin + pt * P + 8 * g, 4);
        memcpy(&T1, sin + pt * P + 8 * g + 4, 4);
        F = rd(sin, pt + 2, g);
        uint32_t pending = ocsw::at_done80<K, 1>(S, Lc);
        const int64_t NP = pt + 3;
        for (int r = 0; r < n; ++r) {
            for (int a = 0; a < A; ++a) AC[a] = rd(act + (int64_t)r * A * P, a, g);
            // the device's dispatch: 4-slot levels of the common class take the MODE 0 build
            if (K == 4 && !S.tall && !S.big && !S.counts && !S.edge)
                ocsw::step4<A, K, 0>(S, X, Y, Hh, Lc, M, T0, T1, F, AC, EX, CM, cls_of,
                                     [](uint32_t v) { return v != 0u; }, pending);
            else
                ocsw::step4<A, K, 1>(S, X, Y, Hh, Lc, M, T0, T1, F, AC, EX, CM, cls_of,
                                     [](uint32_t v) { return v != 0u; }, pending);
            uint8_t* so = sout + (int64_t)r * NP * P;
            for (int a = 0; a < A; ++a) { wr(so, a, g, X[a]); wr(so, A + a, g, Y[a]); wr(so, 2 * A + a, g, Hh[a]); if (exo) wr(exo + (int64_t)r * A * P, a, g, EX[a]); }
            for (int j = 0; j < K; ++j) { wr(so, 3 * A + j, g, Lc[j]); wr(so, 3 * A + K + j, g, M[j]); }
            memcpy(so + pt * P + 8 * g, &T0, 4);
            memcpy(so + pt * P + 8 * g + 4, &T1, 4);
            wr(so, pt + 2, g, F);
            if (coll) memcpy(coll + (int64_t)r * P + 4 * g, &CM, 4);
        }
    }
}

extern "C" int swar_host_step_n(const oc_level_desc* lv, int A, int K, int max_T, const uint8_t* sin, uint8_t* traj,
                                const uint8_t* act, uint8_t* exo, uint8_t* coll, int64_t B, int64_t P, int n) {
#define RN(a, k) if (A == a && K == k) { run<a, k>(lv, max_T, sin, traj, act, exo, coll, B, P, n); return 0; }
    RN(1, 4) RN(2, 4) RN(3, 4) RN(4, 4) RN(1, 8) RN(2, 8) RN(3, 8) RN(4, 8) RN(1, 16) RN(2, 16) RN(3, 16) RN(4, 16)
    return -1;
}

extern "C" int swar_host_step(const oc_level_desc* lv, int A, int K, int max_T, const uint8_t* sin, uint8_t* sout,
                              const uint8_t* act, uint8_t* exo, uint8_t* coll, int64_t B, int64_t P) {
#define R(a, k) if (A == a && K == k) { run<a, k>(lv, max_T, sin, sout, act, exo, coll, B, P); return 0; }
    R(1, 4) R(2, 4) R(3, 4) R(4, 4) R(1, 8) R(2, 8) R(3, 8) R(4, 8) R(1, 16) R(2, 16) R(3, 16) R(4, 16)
    return -1;
}
