// oc_engine.hip -- MI355X (gfx950) batched Overcooked step engine + its C-ABI (include/oc_engine.h).
//
// One fused kernel steps a batch of independent kitchens.  The state is structure-of-arrays
// byte planes; each lane owns EPL consecutive envs, so every plane is read
// and written with one coalesced EPL-byte access per lane (EPL = 4: one dword, 256 B per
// wave-instruction).  The static level (7x7 tile classes) lives in three 64-bit cell masks
// in SGPRs, so a tile lookup is a 64-bit shift: no LDS, no table loads.  Per env the kernel
// runs, branch-free (selects, no divergent control flow):
//   pairwise collision resolution  <- check_collisions / is_collision
//                                     (gym_cooking/envs/overcooked_environment.py:671-762)
//   sequential per-agent interact  <- execute_navigation + interact
//                                     (overcooked_environment.py:767-770, gym_cooking/utils/interact.py:4-89)
//   the copy-crash (ERR) condition <- new_obs = copy.copy(self) (overcooked_environment.py:289, :108-113)
//   done() / reward()              <- overcooked_environment.py:316-376
// and accumulates per-block episode statistics for the all-gather of summaries.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/oc_engine.h"

namespace {

constexpr int kBlock = 256;  // 4 waves
constexpr int kEPL = 4;      // envs per lane: one dword per byte plane
constexpr int kEnvsPerBlock = kBlock * kEPL;

// Kernel argument block: everything static about the level, passed by value (SGPRs).
struct LevelArgs {
    uint64_t floor_mask;  // bit c: cell c is Floor (the only non-collidable tile)
    uint64_t cut_mask;    // Cutboard cells
    uint64_t deliv_mask;  // Delivery cells
    uint64_t dcell_lut;   // per action code: signed cell delta + 128 (byte lanes 0..4)
    int32_t W, H;
    int32_t done_cell;    // first Delivery in scan order (done() reads only it, :349)
    int32_t max_T;        // 0 = no limit
    uint32_t goals;       // up to 4 goal masks, one per byte
    int32_t ngoals;
    uint32_t tmpl_x, tmpl_y;          // spawn x / y of agents 0..3, one per byte
    uint32_t tmpl_cell[2], tmpl_mask[2];  // item slots 0..7, one per byte
    int64_t pitch;
    int64_t B;
};

// action code -> (dx + 1) / (dy + 1), 4 bits per code: World.NAV_ACTIONS (world.py:16) + noop
constexpr uint32_t kDXLUT = 0x12011u;  // codes 0..4 -> dx 0,0,-1,+1,0
constexpr uint32_t kDYLUT = 0x11102u;  // codes 0..4 -> dy +1,-1,0,0,0

__device__ __forceinline__ uint32_t bit64(uint64_t m, uint32_t c) {
    return (uint32_t)(m >> (c & 63u)) & 1u;
}
__device__ __forceinline__ uint32_t byte_of(uint32_t w, int j) { return (w >> (8 * j)) & 0xFFu; }
__device__ __forceinline__ uint32_t byte_of2(const uint32_t (&w)[2], int j) {
    return byte_of(w[j >> 2], j & 3);
}

// Object.is_deliverable (core.py:214-219): >= 2 contents, every food in its last state.
__device__ __forceinline__ bool deliverable(uint32_t m) {
    return __popc(m & 0xFu) >= 2 && ((m & 7u) & ~(m >> OC_M_CHOPPED_SHIFT)) == 0u;
}
// mergeable (core.py:222-241): at most one plate, every food chopped.
__device__ __forceinline__ bool mergeable(uint32_t a, uint32_t b) {
    const uint32_t c = a | b;
    return ((a & b) & OC_M_PLATE) == 0u && ((c & 7u) & ~(c >> OC_M_CHOPPED_SHIFT)) == 0u;
}
// Object.needs_chopped (core.py:176-178, 285-291): a single fresh food.
__device__ __forceinline__ bool needs_chop(uint32_t m) {
    return m != 0u && m <= 4u && (m & (m - 1u)) == 0u;
}

// One env transition (step(), overcooked_environment.py:255-306) on register-resident fields.
template <int A, int K>
__device__ __forceinline__ void step_env(const LevelArgs& L, uint32_t (&ax)[A], uint32_t (&ay)[A],
                                         uint32_t (&ah)[A], uint32_t (&il)[K], uint32_t (&im)[K],
                                         uint32_t& t, uint32_t& fl, const uint32_t (&act_in)[A],
                                         uint32_t (&ex)[A], uint32_t& coll) {
    const bool rst = (fl & OC_FLAG_DONE) != 0u;  // next-step auto-reset

    uint32_t act[A], loc[A], nraw[A], nxt[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        act[a] = min(act_in[a], (uint32_t)OC_ACT_NOOP);
        loc[a] = ay[a] * (uint32_t)L.W + ax[a];
        nraw[a] = loc[a] + ((uint32_t)(L.dcell_lut >> (8u * act[a])) & 0xFFu) - 128u;
        // is_collision: a collidable next square reverts to the current one (:692-700)
        nxt[a] = bit64(L.floor_mask, nraw[a]) ? nraw[a] : loc[a];
    }

    // check_collisions: pairs in itertools.combinations order on the ORIGINAL actions,
    // blocked agents zeroed after all pairs (:724-762).
    uint32_t blk = 0u, cm = 0u;
    int p = 0;
#pragma unroll
    for (int i = 0; i < A; ++i) {
#pragma unroll
        for (int j = i + 1; j < A; ++j, ++p) {
            const bool eq = nxt[i] == nxt[j];
            const bool c1 = nxt[i] == loc[i] && act[i] != OC_ACT_NOOP;
            const bool c2 = nxt[j] == loc[j] && act[j] != OC_ACT_NOOP;
            const bool sw = loc[i] == nxt[j] && loc[j] == nxt[i];
            const bool bi = eq ? !c1 : sw;
            const bool bj = eq ? (c1 || !c2) : sw;
            blk |= ((uint32_t)bi << i) | ((uint32_t)bj << j);
            cm |= (uint32_t)(bi || bj) << p;
        }
    }

    // execute_navigation: interact() per agent in order, each seeing earlier agents' effects.
#pragma unroll
    for (int k = 0; k < A; ++k) {
        const bool blocked = (blk >> k) & 1u;
        const uint32_t e = blocked ? (uint32_t)OC_ACT_NOOP : act[k];
        ex[k] = e;
        const bool go = e != OC_ACT_NOOP;
        // target = inbounds(loc + action) (interact.py:22); agents stand on Floor and the
        // border is never Floor, so the clamp is the identity and target = nraw.
        const uint32_t tc = nraw[k];
        const bool isF = bit64(L.floor_mask, tc);
        const bool isD = bit64(L.deliv_mask, tc);
        const bool isC = bit64(L.cut_mask, tc);
        const uint32_t h = ah[k];
        const bool hold = h != OC_HOLD_NONE;
        // the un-held object at target (world.is_occupied / get_object_at): any item on a
        // non-Floor cell is un-held, since held items sit on their holder's Floor cell.
        uint32_t o = OC_HOLD_NONE, om = 0u, hm = 0u;
#pragma unroll
        for (int j = K - 1; j >= 0; --j) {
            const bool at = il[j] == tc;
            o = at ? (uint32_t)j : o;
            om = at ? im[j] : om;
            hm = (h == (uint32_t)j) ? im[j] : hm;
        }
        const bool hasO = o != OC_HOLD_NONE;
        const bool nf = go && !isF;
        const bool move = go && isF;                                           // :28-30
        const bool deliver = nf && hold && isD && deliverable(hm);             // :35-40
        const bool merge = nf && hold && !isD && hasO && mergeable(hm, om);    // :43-56
        const bool empty = nf && hold && !isD && !hasO;                        // :60-70
        const bool chop = empty && isC && needs_chop(hm);
        const bool put = empty && !chop;
        const bool pick = nf && !hold && hasO && !isD;                         // :73-84
        const bool relocate_h = move || deliver || put;  // held item goes to tc
        const uint32_t dxp = (kDXLUT >> (4u * e)) & 0xFu;
        const uint32_t dyp = (kDYLUT >> (4u * e)) & 0xFu;
        ax[k] = move ? ax[k] + dxp - 1u : ax[k];
        ay[k] = move ? ay[k] + dyp - 1u : ay[k];
        const uint32_t merged = hm | om;
        const uint32_t chopped = hm | (hm << OC_M_CHOPPED_SHIFT);
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool isH = h == (uint32_t)j;
            const bool isO = o == (uint32_t)j;
            uint32_t l = il[j], m = im[j];
            l = (isH && relocate_h) ? tc : l;
            m = (isH && merge) ? merged : m;
            m = (isH && chop) ? chopped : m;
            l = (isO && merge) ? (uint32_t)OC_LOC_DEAD : l;
            m = (isO && merge) ? 0u : m;
            l = (isO && pick) ? loc[k] : l;
            il[j] = l;
            im[j] = m;
        }
        ah[k] = (deliver || put) ? (uint32_t)OC_HOLD_NONE : (pick ? o : h);
    }

    // new_obs = copy.copy(self) raises when two co-located agents both hold (ERR).
    bool err = false;
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = i + 1; j < A; ++j)
            err |= ax[i] == ax[j] && ay[i] == ay[j] && ah[i] != OC_HOLD_NONE && ah[j] != OC_HOLD_NONE;

    const uint32_t tn = t + 1u;  // :257
    // done(): timeout first (:328-332), then every Deliver goal on the delivery cell (:344-363)
    const bool tout = L.max_T != 0 && tn >= (uint32_t)L.max_T;
    bool all_ok = true;
    for (int g = 0; g < L.ngoals; ++g) {  // wave-uniform trip count
        const uint32_t gm = (L.goals >> (8 * g)) & 0xFFu;
        bool ok = false;
#pragma unroll
        for (int j = 0; j < K; ++j) ok |= il[j] == (uint32_t)L.done_cell && im[j] == gm;
        all_ok &= ok;
    }
    const uint32_t fn = err ? (OC_FLAG_DONE | OC_FLAG_ERR)
                            : (tout ? OC_FLAG_DONE : (all_ok ? (OC_FLAG_DONE | OC_FLAG_SUCCESS) : 0u));

    // auto-reset: an env that was done at the input restarts from the level template
#pragma unroll
    for (int a = 0; a < A; ++a) {
        ax[a] = rst ? byte_of(L.tmpl_x, a) : ax[a];
        ay[a] = rst ? byte_of(L.tmpl_y, a) : ay[a];
        ah[a] = rst ? (uint32_t)OC_HOLD_NONE : ah[a];
        ex[a] = rst ? (uint32_t)OC_ACT_NOOP : ex[a];
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        il[j] = rst ? byte_of2(L.tmpl_cell, j) : il[j];
        im[j] = rst ? byte_of2(L.tmpl_mask, j) : im[j];
    }
    t = rst ? 0u : tn;
    fl = rst ? 0u : fn;
    coll = rst ? 0u : cm;
}

// Statistics partial sums, one row of OC_NSTATS uint64 per block.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <int A, int K>
__global__ __launch_bounds__(kBlock) void oc_step_kernel(LevelArgs L, const uint8_t* __restrict__ sin,
                                                         uint8_t* __restrict__ sout,
                                                         const uint8_t* __restrict__ actions,
                                                         uint8_t* __restrict__ exec_out,
                                                         uint8_t* __restrict__ coll_out,
                                                         uint64_t* __restrict__ stats) {
    const int64_t P = L.pitch;
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t e0 = g * kEPL;  // first env of this lane
    constexpr int kPA = 0, kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K, kPT = 3 * A + 2 * K,
                  kPF = 3 * A + 2 * K + 2;
    auto ld32 = [&](int plane) -> uint32_t {
        return *reinterpret_cast<const uint32_t*>(sin + plane * P + e0);
    };
    // ---- coalesced loads: one dword per byte plane, 8 bytes of the u16 t plane
    uint32_t wx[A], wy[A], wh[A], wl[K], wm[K], wa[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        wx[a] = ld32(kPA + a);
        wy[a] = ld32(kPY + a);
        wh[a] = ld32(kPH + a);
        wa[a] = *reinterpret_cast<const uint32_t*>(actions + a * P + e0);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        wl[j] = ld32(kPL + j);
        wm[j] = ld32(kPM + j);
    }
    const uint2 wt = *reinterpret_cast<const uint2*>(sin + kPT * P + 2 * e0);
    const uint32_t wf = ld32(kPF);

    uint32_t ox[A] = {}, oy[A] = {}, oh[A] = {}, ol[K] = {}, om[K] = {}, oe[A] = {};
    uint32_t ot[2] = {0u, 0u}, of = 0u, oc = 0u;
    uint32_t s_eps = 0u, s_succ = 0u, s_steps = 0u, s_coll = 0u, s_err = 0u;

#pragma unroll
    for (int q = 0; q < kEPL; ++q) {
        uint32_t ax[A], ay[A], ah[A], il[K], im[K], ac[A], ex[A];
#pragma unroll
        for (int a = 0; a < A; ++a) {
            ax[a] = byte_of(wx[a], q);
            ay[a] = byte_of(wy[a], q);
            ah[a] = byte_of(wh[a], q);
            ac[a] = byte_of(wa[a], q);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            il[j] = byte_of(wl[j], q);
            im[j] = byte_of(wm[j], q);
        }
        uint32_t t = ((q < 2 ? wt.x : wt.y) >> (16 * (q & 1))) & 0xFFFFu;
        uint32_t fl = byte_of(wf, q);
        const bool was_done = (fl & OC_FLAG_DONE) != 0u;
        uint32_t coll;
        step_env<A, K>(L, ax, ay, ah, il, im, t, fl, ac, ex, coll);
        const int sh = 8 * q;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            ox[a] |= (ax[a] & 0xFFu) << sh;
            oy[a] |= (ay[a] & 0xFFu) << sh;
            oh[a] |= (ah[a] & 0xFFu) << sh;
            oe[a] |= ex[a] << sh;
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            ol[j] |= (il[j] & 0xFFu) << sh;
            om[j] |= (im[j] & 0xFFu) << sh;
        }
        ot[q >> 1] |= (t & 0xFFFFu) << (16 * (q & 1));
        of |= fl << sh;
        oc |= coll << sh;
        const bool valid = e0 + q < L.B;
        const bool ended = valid && !was_done && (fl & OC_FLAG_DONE);
        s_eps += ended;
        s_succ += ended && (fl & OC_FLAG_SUCCESS);
        s_steps += ended ? t : 0u;
        s_err += ended && (fl & OC_FLAG_ERR);
        s_coll += valid ? __popc(coll) : 0u;
    }

    auto st32 = [&](int plane, uint32_t v) {
        *reinterpret_cast<uint32_t*>(sout + plane * P + e0) = v;
    };
#pragma unroll
    for (int a = 0; a < A; ++a) {
        st32(kPA + a, ox[a]);
        st32(kPY + a, oy[a]);
        st32(kPH + a, oh[a]);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        st32(kPL + j, ol[j]);
        st32(kPM + j, om[j]);
    }
    *reinterpret_cast<uint2*>(sout + kPT * P + 2 * e0) = make_uint2(ot[0], ot[1]);
    st32(kPF, of);
    if (exec_out != nullptr) {
#pragma unroll
        for (int a = 0; a < A; ++a) *reinterpret_cast<uint32_t*>(exec_out + a * P + e0) = oe[a];
    }
    if (coll_out != nullptr) *reinterpret_cast<uint32_t*>(coll_out + e0) = oc;

    if (stats != nullptr) {
        __shared__ uint32_t red[kBlock / 64][OC_NSTATS];
        const uint32_t v[OC_NSTATS] = {s_eps, s_succ, s_steps, s_coll, s_err};
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
        for (int c = 0; c < OC_NSTATS; ++c) {
            const uint32_t r = wave_sum(v[c]);
            if (lane == 0) red[wid][c] = r;
        }
        __syncthreads();
        if (threadIdx.x < OC_NSTATS) {
            uint64_t s = 0;
#pragma unroll
            for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
            stats[(int64_t)blockIdx.x * OC_NSTATS + threadIdx.x] += s;  // block-private row
        }
    }
}

// reset(): broadcast the level template (overcooked_environment.py:201-250).
template <int A, int K>
__global__ __launch_bounds__(kBlock) void oc_reset_kernel(LevelArgs L, uint8_t* __restrict__ s) {
    const int64_t P = L.pitch;
    const int64_t e0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kEPL;
    auto rep = [](uint32_t b) { return (b & 0xFFu) * 0x01010101u; };
    auto st32 = [&](int plane, uint32_t v) { *reinterpret_cast<uint32_t*>(s + plane * P + e0) = v; };
#pragma unroll
    for (int a = 0; a < A; ++a) {
        st32(a, rep(byte_of(L.tmpl_x, a)));
        st32(A + a, rep(byte_of(L.tmpl_y, a)));
        st32(2 * A + a, rep(OC_HOLD_NONE));
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        st32(3 * A + j, rep(byte_of2(L.tmpl_cell, j)));
        st32(3 * A + K + j, rep(byte_of2(L.tmpl_mask, j)));
    }
    *reinterpret_cast<uint2*>(s + (3 * A + 2 * K) * P + 2 * e0) = make_uint2(0u, 0u);
    st32(3 * A + 2 * K + 2, 0u);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void oc_gen_actions_kernel(uint8_t* __restrict__ act, int A, int64_t B,
                                                                int64_t pitch, int64_t env_offset,
                                                                uint64_t step, uint64_t seed) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= pitch) return;
    const uint64_t base = seed ^ ((uint64_t)(env_offset + e) * 0x9E3779B97F4A7C15ull) ^
                          (step * 0xC2B2AE3D27D4EB4Full);
    for (int a = 0; a < A; ++a)
        act[a * pitch + e] = e < B ? (uint8_t)(splitmix64(base ^ (uint64_t)a) % 5u) : (uint8_t)OC_ACT_NOOP;
}

__global__ __launch_bounds__(kBlock) void oc_stats_reduce_kernel(const uint64_t* __restrict__ part,
                                                                 int64_t nrows, uint64_t* __restrict__ out) {
    __shared__ uint64_t red[kBlock];
    for (int c = 0; c < OC_NSTATS; ++c) {
        uint64_t s = 0;
        for (int64_t r = threadIdx.x; r < nrows; r += kBlock) s += part[r * OC_NSTATS + c];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int w = kBlock / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[c] = red[0];
        __syncthreads();
    }
}

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int hip_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(OC_EHIP, "%s: %s", what, hipGetErrorString(e));
    return OC_OK;
}

int64_t pitch_for(int64_t B) {
    int64_t p = (B + OC_PITCH_ALIGN - 1) / OC_PITCH_ALIGN * OC_PITCH_ALIGN;
    return p < OC_PITCH_ALIGN ? OC_PITCH_ALIGN : p;
}

}  // namespace

struct oc_handle {
    oc_level_desc level;
    int32_t A, K, max_T, device;
    LevelArgs args;
};

extern "C" {

int oc_abi_version(void) { return OC_ABI_VERSION; }

const char* oc_last_error(void) { return g_last_error.c_str(); }

int oc_create(const oc_level_desc* lv, int32_t num_agents, int32_t max_T, int32_t device, oc_handle** out) {
    if (lv == nullptr || out == nullptr) return fail(OC_EINVAL, "null argument");
    const int W = lv->width, H = lv->height;
    if (W < 3 || H < 3 || W * H > OC_MAX_CELLS) return fail(OC_ELEVEL, "grid %dx%d outside 3..64 cells", W, H);
    if (num_agents < 1 || num_agents > OC_MAX_AGENTS) return fail(OC_EINVAL, "num_agents %d", num_agents);
    if (lv->num_spawns < num_agents || lv->num_spawns > OC_MAX_AGENTS) return fail(OC_ELEVEL, "num_spawns %d", lv->num_spawns);
    if (lv->num_items < 0 || lv->num_items > OC_MAX_ITEMS) return fail(OC_ELEVEL, "num_items %d", lv->num_items);
    if (lv->num_goals < 1 || lv->num_goals > OC_MAX_GOALS) return fail(OC_ELEVEL, "num_goals %d", lv->num_goals);
    if (max_T < 0 || max_T > 65535) return fail(OC_EINVAL, "max_T %d", max_T);
    LevelArgs L{};
    L.W = W;
    L.H = H;
    L.done_cell = -1;
    for (int c = 0; c < W * H; ++c) {
        const int t = lv->tiles[c];
        if (t < OC_TILE_FLOOR || t > OC_TILE_DELIVERY) return fail(OC_ELEVEL, "tile %d at cell %d", t, c);
        const int x = c % W, y = c / W;
        if (t == OC_TILE_FLOOR && (x == 0 || y == 0 || x == W - 1 || y == H - 1))
            return fail(OC_ELEVEL, "Floor on the border at (%d,%d)", x, y);
        if (t == OC_TILE_FLOOR) L.floor_mask |= 1ull << c;
        if (t == OC_TILE_CUTBOARD) L.cut_mask |= 1ull << c;
        if (t == OC_TILE_DELIVERY) {
            L.deliv_mask |= 1ull << c;
            if (L.done_cell < 0) L.done_cell = c;
        }
    }
    if (L.done_cell < 0) return fail(OC_ELEVEL, "no Delivery tile");
    uint32_t seen_food = 0;
    const int K = lv->num_items <= 4 ? 4 : 8;
    uint8_t cell[8], mask[8];
    for (int j = 0; j < 8; ++j) {
        cell[j] = OC_LOC_DEAD;
        mask[j] = 0;
    }
    for (int j = 0; j < lv->num_items; ++j) {
        const int c = lv->item_cell[j], m = lv->item_mask[j];
        if (c >= W * H || lv->tiles[c] == OC_TILE_FLOOR) return fail(OC_ELEVEL, "item %d not on a counter", j);
        if (m == 0 || (m & 0x80) || (((m >> OC_M_CHOPPED_SHIFT) & 7) & ~(m & 7))) return fail(OC_ELEVEL, "item mask 0x%x", m);
        if (seen_food & m & 7u) return fail(OC_ELEVEL, "food type present twice (mask ambiguity)");
        seen_food |= m & 7u;
        cell[j] = (uint8_t)c;
        mask[j] = (uint8_t)m;
    }
    for (int a = 0; a < num_agents; ++a) {
        const int x = lv->spawn_x[a], y = lv->spawn_y[a];
        if (x >= W || y >= H || lv->tiles[y * W + x] != OC_TILE_FLOOR) return fail(OC_ELEVEL, "spawn %d not on Floor", a);
        L.tmpl_x |= (uint32_t)x << (8 * a);
        L.tmpl_y |= (uint32_t)y << (8 * a);
    }
    for (int j = 0; j < 8; ++j) {
        L.tmpl_cell[j >> 2] |= (uint32_t)cell[j] << (8 * (j & 3));
        L.tmpl_mask[j >> 2] |= (uint32_t)mask[j] << (8 * (j & 3));
    }
    for (int g = 0; g < lv->num_goals; ++g) L.goals |= (uint32_t)lv->goal_mask[g] << (8 * g);
    L.ngoals = lv->num_goals;
    L.max_T = max_T;
    const int dcell[5] = {W, -W, -1, 1, 0};
    for (int c = 0; c < 5; ++c) L.dcell_lut |= (uint64_t)((dcell[c] + 128) & 0xFF) << (8 * c);
    oc_handle* h = new oc_handle;
    h->level = *lv;
    h->A = num_agents;
    h->K = K;
    h->max_T = max_T;
    h->device = device;
    h->args = L;
    *out = h;
    return OC_OK;
}

int oc_destroy(oc_handle* h) {
    delete h;
    return OC_OK;
}

int oc_get_layout(const oc_handle* h, int64_t B, oc_layout* out) {
    if (h == nullptr || out == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    const int A = h->A, K = h->K;
    out->pitch = pitch_for(B);
    out->num_agents = A;
    out->num_items = K;
    out->plane_agent_x = 0;
    out->plane_agent_y = A;
    out->plane_agent_hold = 2 * A;
    out->plane_item_loc = 3 * A;
    out->plane_item_mask = 3 * A + K;
    out->plane_t = 3 * A + 2 * K;
    out->plane_flags = 3 * A + 2 * K + 2;
    out->num_planes = 3 * A + 2 * K + 3;
    out->state_bytes = out->num_planes * out->pitch;
    return OC_OK;
}

#define OC_DISPATCH(A_, K_, LAUNCH)                                                         \
    switch ((A_) * 10 + (K_)) {                                                             \
        case 14: LAUNCH(1, 4); break;                                                       \
        case 24: LAUNCH(2, 4); break;                                                       \
        case 34: LAUNCH(3, 4); break;                                                       \
        case 44: LAUNCH(4, 4); break;                                                       \
        case 18: LAUNCH(1, 8); break;                                                       \
        case 28: LAUNCH(2, 8); break;                                                       \
        case 38: LAUNCH(3, 8); break;                                                       \
        case 48: LAUNCH(4, 8); break;                                                       \
        default: return fail(OC_EINVAL, "unsupported (A,K)=(%d,%d)", (A_), (K_));           \
    }

int oc_reset(const oc_handle* h, void* state, int64_t B, void* stream) {
    if (h == nullptr || state == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    if (B == 0) return OC_OK;
    LevelArgs L = h->args;
    L.pitch = pitch_for(B);
    L.B = B;
    const dim3 grid((unsigned)(L.pitch / kEnvsPerBlock));
    hipStream_t s = (hipStream_t)stream;
#define OC_LAUNCH_RESET(A, K) hipLaunchKernelGGL((oc_reset_kernel<A, K>), grid, dim3(kBlock), 0, s, L, (uint8_t*)state)
    OC_DISPATCH(h->A, h->K, OC_LAUNCH_RESET)
    return hip_check("oc_reset launch");
}

int oc_step(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
            uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* stats, int64_t B, void* stream) {
    if (h == nullptr || state_in == nullptr || state_out == nullptr || actions == nullptr || B < 0)
        return fail(OC_EINVAL, "bad argument");
    if (B == 0) return OC_OK;
    if (((uintptr_t)state_in | (uintptr_t)state_out | (uintptr_t)actions | (uintptr_t)exec_actions |
         (uintptr_t)coll_mask) & 15u)
        return fail(OC_EINVAL, "buffers must be 16-byte aligned");
    LevelArgs L = h->args;
    L.pitch = pitch_for(B);
    L.B = B;
    const dim3 grid((unsigned)(L.pitch / kEnvsPerBlock));
    hipStream_t s = (hipStream_t)stream;
#define OC_LAUNCH_STEP(A, K)                                                                          \
    hipLaunchKernelGGL((oc_step_kernel<A, K>), grid, dim3(kBlock), 0, s, L, (const uint8_t*)state_in, \
                       (uint8_t*)state_out, actions, exec_actions, coll_mask, stats)
    OC_DISPATCH(h->A, h->K, OC_LAUNCH_STEP)
    return hip_check("oc_step launch");
}

int oc_gen_actions(const oc_handle* h, uint8_t* actions, int64_t B, int64_t env_offset, int64_t step,
                   uint64_t seed, void* stream) {
    if (h == nullptr || actions == nullptr || B < 0 || env_offset < 0 || step < 0) return fail(OC_EINVAL, "bad argument");
    if (B == 0) return OC_OK;
    const int64_t P = pitch_for(B);
    hipLaunchKernelGGL(oc_gen_actions_kernel, dim3((unsigned)(P / kBlock)), dim3(kBlock), 0, (hipStream_t)stream,
                       actions, h->A, B, P, env_offset, (uint64_t)step, seed);
    return hip_check("oc_gen_actions launch");
}

int oc_stats_size(const oc_handle* h, int64_t B, int64_t* nbytes) {
    if (h == nullptr || nbytes == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    *nbytes = (pitch_for(B) / kEnvsPerBlock) * OC_NSTATS * (int64_t)sizeof(uint64_t);
    return OC_OK;
}

int oc_stats_reduce(const oc_handle* h, const uint64_t* stats, int64_t B, uint64_t* totals, void* stream) {
    if (h == nullptr || stats == nullptr || totals == nullptr || B < 0) return fail(OC_EINVAL, "bad argument");
    const int64_t rows = pitch_for(B) / kEnvsPerBlock;
    hipLaunchKernelGGL(oc_stats_reduce_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, stats, rows, totals);
    return hip_check("oc_stats_reduce launch");
}

}  // extern "C"
