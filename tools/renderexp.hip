// tools/renderexp.hip -- oc_render experiment (includes the engine TU).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -o /tmp/renderexp tools/renderexp.hip
// Workload: bench.py's render shape -- 1,024 random-play states (37 steps) of a 7x7 kitchen
// (full-divider_salad, 4 agents), 80-px cells, a synthetic atlas (random RGBA, a third of the
// sprite pixels fully transparent, a third opaque) and a random level image; any pixels do for
// an identity check against the product kernel.
// Variants:
//   lane blend  the round-2 kernel: lane = 16 consecutive pixels, each lane blends its own
//               pixels (per-channel SDL blend with the a = 0 branch); lanes over sprite-free
//               cells idle in the blend loop
//   product     oc_render_kernel: the wave's listed lanes put their pixels in LDS and the wave
//               blends them one pixel per lane, two 24-bit multiply-adds per channel pair
//   product, N blocks per strip   the strip of one (env, cell row) split over N blocks (oc_render: 2)
//   compact E   the product's scheme with E envs per block (the level-image pixels loaded once
//               for E envs); modes: no blend, no blend and no level-image loads (store floor),
//               sprite loads of 4 draws batched before blending
// Outputs compared byte for byte with the product's.
#include "../gym-cooking_amd/csrc/oc_engine.hip"

#include <random>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

namespace {

// The round-2 blend: per channel, with the a = 0 branch (SDL's ALPHA_BLEND as written)
__device__ __forceinline__ uint32_t sdl_blend_channels(uint32_t d, uint32_t s) {
    const int a = (int)(s >> 24);
    if (a == 0) return d;
    uint32_t out = 0u;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int sc = (int)((s >> (8 * c)) & 0xFFu), dc = (int)((d >> (8 * c)) & 0xFFu);
        out |= (uint32_t)((((sc - dc) * a + 255) >> 8) + dc) << (8 * c);
    }
    return out;
}

// The round-2 product kernel: each lane blends its own 16 pixels
template <int A, int K>
__global__ __launch_bounds__(kBlock) void render_lane_blend(RenderArgs R, const uint8_t* __restrict__ state,
                                                           const uint32_t* __restrict__ atlas,
                                                           const uint32_t* __restrict__ bg,
                                                           uint8_t* __restrict__ out) {
    __shared__ uint32_t dl_off[kRenderMaxW][kRenderMaxDraw];
    __shared__ uint32_t dl_geo[kRenderMaxW][kRenderMaxDraw];  // size | offset << 16
    __shared__ int32_t dl_n[kRenderMaxW];
    const int64_t e = blockIdx.x / (uint32_t)R.H;
    const int ty = (int)(blockIdx.x % (uint32_t)R.H);
    const int W = R.W, tile = R.tile;
    constexpr int kPX = 0, kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K;
    if ((int)threadIdx.x < W) {
        const int tx = threadIdx.x, cell = ty * W + tx;
        const uint8_t* s = state + e;
        const int64_t P = R.pitch;
        uint32_t held = 0u;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const uint32_t h = s[(kPH + a) * P];
            if (h < (uint32_t)K) held |= 1u << h;
        }
        int n = 0;
        auto push = [&](int32_t off, int cls) {
            dl_off[tx][n] = (uint32_t)off;
            dl_geo[tx][n] = (uint32_t)R.size[cls] | ((uint32_t)R.offset[cls] << 16);
            ++n;
        };
        // an item: a plate first, its contents at the container class; else the food itself
        auto push_item = [&](uint32_t m, int cls_plain, int cls_in_plate, int plate) {
            const uint32_t f = m & ~OC_M_PLATE;
            if (m & OC_M_PLATE) push(R.plate_off[plate], cls_plain);
            const int cls = (m & OC_M_PLATE) ? cls_in_plate : cls_plain;
            if (f != 0u && R.food_sprite[f] != 0xFFu)
                push(R.food_base[cls] + (int32_t)R.food_sprite[f] * R.size[cls] * R.size[cls], cls);
        };
        // Game.on_render: objects not held (draw_object, game.py:138-160) ...
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (s[(kPL + j) * P] == (uint8_t)cell && !((held >> j) & 1u)) push_item(s[(kPM + j) * P], 0, 1, 0);
        // ... then the agents in order, each with its held object (draw_agent / draw_agent_object, :98-136)
#pragma unroll
        for (int a = 0; a < A; ++a) {
            if ((int)s[(kPY + a) * P] * W + (int)s[(kPX + a) * P] != cell) continue;
            push(R.agent_off[a], 0);
            const uint32_t h = s[(kPH + a) * P];
            if (h < (uint32_t)K) push_item(s[(kPM + h) * P], 2, 3, 1);
        }
        dl_n[tx] = n;
    }
    __syncthreads();
    const int row_px = W * tile, G = row_px / kRenderPx;  // 16-pixel groups per image row
    const int items = tile * G;
    const int64_t img_bytes = (int64_t)R.H * tile * row_px * 3;
    uint8_t* img = out + e * img_bytes;
    // chan_map -> v_perm selector: output byte c <- pixel byte (chan_map >> 8c), 0x0C = zero
    uint32_t psel = 0x0C000000u;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t ch = (R.chan_map >> (8 * c)) & 0xFFu;
        psel |= (ch >= 3u ? 0x0Cu : ch) << (8 * c);
    }
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    // The block's output rows are contiguous and group i lands at byte 48 i, so a wave's 64
    // groups are 3 KB contiguous.  Each lane packs its 48 bytes into the wave's LDS slice, and
    // the wave then stores the slice as three fully contiguous 1 KB instructions (16 B per
    // lane) instead of three 16 B-per-lane instructions at a 48 B stride.
    __shared__ u32x4 stage[kBlock / 64][64 * 3];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* const blk_out = img + (int64_t)ty * tile * row_px * 3;
    for (int base = 0; base < items; base += kBlock) {
        const int i = base + threadIdx.x;
        if (i < items) {
            const int r = i / G, g = i - r * G;
            const int py = ty * tile + r, px0 = kRenderPx * g;
            const u32x4* bsrc = (const u32x4*)(bg + (int64_t)py * row_px + px0);
            uint32_t p[kRenderPx];
#pragma unroll
            for (int q = 0; q < kRenderPx / 4; ++q) {
                const u32x4 v = bsrc[q];
                p[4 * q] = v.x;
                p[4 * q + 1] = v.y;
                p[4 * q + 2] = v.z;
                p[4 * q + 3] = v.w;
            }
            const int tx = px0 / tile, lx0 = px0 - tx * tile;  // a group never straddles two cells
            const int n = dl_n[tx];
            for (int d = 0; d < n; ++d) {
                const uint32_t geo = dl_geo[tx][d];
                const int sz = (int)(geo & 0xFFFFu), o = (int)(geo >> 16);
                const int dy = r - o;
                if ((unsigned)dy >= (unsigned)sz || lx0 + kRenderPx <= o || lx0 >= o + sz) continue;
                const uint32_t* spr = atlas + dl_off[tx][d] + dy * sz;
#pragma unroll
                for (int k = 0; k < kRenderPx; ++k) {
                    const int dx = lx0 + k - o;
                    if ((unsigned)dx < (unsigned)sz) p[k] = sdl_blend_channels(p[k], spr[dx]);
                }
            }
            // 16 pixels -> 48 bytes: per 4 pixels three dwords of packed 3-byte pixels
            uint32_t w[12];
#pragma unroll
            for (int q = 0; q < kRenderPx / 4; ++q) {
                const uint32_t a0 = __builtin_amdgcn_perm(0u, p[4 * q], psel),
                               a1 = __builtin_amdgcn_perm(0u, p[4 * q + 1], psel),
                               a2 = __builtin_amdgcn_perm(0u, p[4 * q + 2], psel),
                               a3 = __builtin_amdgcn_perm(0u, p[4 * q + 3], psel);
                w[3 * q] = a0 | (a1 << 24);
                w[3 * q + 1] = (a1 >> 8) | (a2 << 16);
                w[3 * q + 2] = (a2 >> 16) | (a3 << 8);
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) stage[wave][3 * lane + q] = u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        }
        __builtin_amdgcn_wave_barrier();  // LDS is in order within a wave; keep the compiler from moving reads up
        const int w0 = base + wave * 64;  // the wave's first group
        const int nbytes = 48 * (items - w0 < 64 ? (items - w0 > 0 ? items - w0 : 0) : 64);
        u32x4* dst = (u32x4*)(blk_out + (int64_t)w0 * 48);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int off = q * 64 + lane;  // 16-byte units
            if (off * 16 < nbytes) __builtin_nontemporal_store(stage[wave][off], dst + off);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <int A, int K, int EPB, int kMode>  // kMode 0 full, 1 no blend, 2 no blend and no level-image loads, 3 full without load batching, 4 stores only (constant data, no LDS staging)
__global__ __launch_bounds__(kBlock) void render_compact(RenderArgs R, const uint8_t* __restrict__ state,
                                                         const uint32_t* __restrict__ atlas,
                                                         const uint32_t* __restrict__ bg, uint8_t* __restrict__ out,
                                                         int64_t B) {
    // draw lists [EPB][W][kRenderMaxDraw] (offset, size | offset << 16), counts [EPB][W]: dynamic LDS
    extern __shared__ uint32_t dyn[];
    const int W = R.W, tile = R.tile;
    uint32_t* const dl_off = dyn;
    uint32_t* const dl_geo = dyn + EPB * W * kRenderMaxDraw;
    int32_t* const dl_n = (int32_t*)(dyn + 2 * EPB * W * kRenderMaxDraw);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    __shared__ u32x4 pix4[kBlock / 64][64 * 4];  // a wave's 1,024 pixels, then its 3 KB packed stage
    __shared__ uint32_t list[kBlock / 64][64];  // lane | r << 6 | tx << 16 | lx0 << 21
    const int64_t e0 = (int64_t)(blockIdx.x / (uint32_t)R.H) * EPB;
    const int ty = (int)(blockIdx.x % (uint32_t)R.H);
    constexpr int kPX = 0, kPY = A, kPH = 2 * A, kPL = 3 * A, kPM = 3 * A + K;
    if ((int)threadIdx.x < EPB * W) {
        const int qe = threadIdx.x / W, tx = threadIdx.x - qe * W, cell = ty * W + tx;
        const int lst = qe * W + tx;
        int n = 0;
        if (e0 + qe < B) {
            const uint8_t* s = state + e0 + qe;
            const int64_t P = R.pitch;
            uint32_t held = 0u;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                const uint32_t h = s[(kPH + a) * P];
                if (h < (uint32_t)K) held |= 1u << h;
            }
            auto push = [&](int32_t off, int cls) {
                dl_off[lst * kRenderMaxDraw + n] = (uint32_t)off;
                dl_geo[lst * kRenderMaxDraw + n] = (uint32_t)R.size[cls] | ((uint32_t)R.offset[cls] << 16);
                ++n;
            };
            auto push_item = [&](uint32_t m, int cls_plain, int cls_in_plate, int plate) {
                const uint32_t f = m & ~OC_M_PLATE;
                if (m & OC_M_PLATE) push(R.plate_off[plate], cls_plain);
                const int cls = (m & OC_M_PLATE) ? cls_in_plate : cls_plain;
                if (f != 0u && R.food_sprite[f] != 0xFFu)
                    push(R.food_base[cls] + (int32_t)R.food_sprite[f] * R.size[cls] * R.size[cls], cls);
            };
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (s[(kPL + j) * P] == (uint8_t)cell && !((held >> j) & 1u)) push_item(s[(kPM + j) * P], 0, 1, 0);
#pragma unroll
            for (int a = 0; a < A; ++a) {
                if ((int)s[(kPY + a) * P] * W + (int)s[(kPX + a) * P] != cell) continue;
                push(R.agent_off[a], 0);
                const uint32_t h = s[(kPH + a) * P];
                if (h < (uint32_t)K) push_item(s[(kPM + h) * P], 2, 3, 1);
            }
        }
        dl_n[lst] = n;
    }
    __syncthreads();
    const int row_px = W * tile, G = row_px / kRenderPx;
    const int items = tile * G;
    const int64_t img_bytes = (int64_t)R.H * tile * row_px * 3;
    uint32_t psel = 0x0C000000u;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t ch = (R.chan_map >> (8 * c)) & 0xFFu;
        psel |= (ch >= 3u ? 0x0Cu : ch) << (8 * c);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* const pix = (uint32_t*)pix4[wave];
    const int nenv = B - e0 < EPB ? (int)(B - e0) : EPB;
    const float rcpG = 1.0f / (float)G, rcpT = 1.0f / (float)tile;
    for (int base = 0; base < items; base += kBlock) {
        const int w0 = base + wave * 64;  // the wave's first group
        const int i = w0 + lane;
        uint32_t p0[kRenderPx];
        int r = 0, tx = 0, lx0 = 0;
        if (i < items) {
            r = div_small(i, G, rcpG);
            const int g = i - r * G;
            const int py = ty * tile + r, px0 = kRenderPx * g;
            tx = div_small(px0, tile, rcpT);
            lx0 = px0 - tx * tile;
            if (kMode == 2 || kMode == 4) {
#pragma unroll
                for (int k = 0; k < kRenderPx; ++k) p0[k] = (uint32_t)(py * 977 + px0 + k);
            } else {
                const u32x4* bsrc = (const u32x4*)(bg + (int64_t)py * row_px + px0);
#pragma unroll
                for (int q = 0; q < kRenderPx / 4; ++q) {
                    const u32x4 v = bsrc[q];
                    p0[4 * q] = v.x;
                    p0[4 * q + 1] = v.y;
                    p0[4 * q + 2] = v.z;
                    p0[4 * q + 3] = v.w;
                }
            }
        }
        for (int qe = 0; qe < nenv; ++qe) {
            uint32_t p[kRenderPx];
#pragma unroll
            for (int k = 0; k < kRenderPx; ++k) p[k] = p0[k];
            const int lst = qe * W;
            bool need = false;
            if ((kMode == 0 || kMode == 3) && i < items) {
                const int n = dl_n[lst + tx];
                for (int d = 0; d < n; ++d) {
                    const uint32_t geo = dl_geo[(lst + tx) * kRenderMaxDraw + d];
                    const int sz = (int)(geo & 0xFFFFu), o = (int)(geo >> 16);
                    need |= (unsigned)(r - o) < (unsigned)sz && lx0 + kRenderPx > o && lx0 < o + sz;
                }
            }
            const uint64_t mask = __ballot(need);
            if (mask != 0ull) {
                if (need) {
#pragma unroll
                    for (int q = 0; q < kRenderPx / 4; ++q)
                        pix4[wave][4 * lane + q] = u32x4{p[4 * q], p[4 * q + 1], p[4 * q + 2], p[4 * q + 3]};
                    list[wave][__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))] =
                        (uint32_t)lane | ((uint32_t)r << 6) | ((uint32_t)tx << 16) | ((uint32_t)lx0 << 21);
                }
                __builtin_amdgcn_wave_barrier();
                const int work = kRenderPx * __popcll(mask);
                for (int t = lane; t < work; t += 64) {
                    const uint32_t ent = list[wave][t >> 4];
                    const int k = t & (kRenderPx - 1), gl = (int)(ent & 63u);
                    const int rr = (int)((ent >> 6) & 0x3FFu), ctx = (int)((ent >> 16) & 31u);
                    const int lx = (int)(ent >> 21) + k;
                    uint32_t dpx = pix[kRenderPx * gl + k];
                    const int n = dl_n[lst + ctx];
                    const uint32_t* dgeo = dl_geo + (lst + ctx) * kRenderMaxDraw;
                    const uint32_t* doff = dl_off + (lst + ctx) * kRenderMaxDraw;
                    if (kMode == 3) {
                        for (int d = 0; d < n; ++d) {
                            const uint32_t geo = dgeo[d];
                            const int sz = (int)(geo & 0xFFFFu), o = (int)(geo >> 16);
                            const int dy = rr - o, dx = lx - o;
                            if ((unsigned)dy < (unsigned)sz && (unsigned)dx < (unsigned)sz)
                                dpx = sdl_blend(dpx, atlas[doff[d] + dy * sz + dx]);
                        }
                    } else {
                        // sprite pixels of up to 4 draws loaded before any is blended (an
                        // uncovered draw loads a transparent stand-in: a = 0 leaves d as is)
                        for (int d0 = 0; d0 < n; d0 += 4) {
                            uint32_t sp[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                sp[u] = 0u;
                                if (d0 + u < n) {
                                    const uint32_t geo = dgeo[d0 + u];
                                    const int sz = (int)(geo & 0xFFFFu), o = (int)(geo >> 16);
                                    const int dy = rr - o, dx = lx - o;
                                    if ((unsigned)dy < (unsigned)sz && (unsigned)dx < (unsigned)sz)
                                        sp[u] = atlas[doff[d0 + u] + dy * sz + dx];
                                }
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) dpx = sdl_blend(dpx, sp[u]);
                        }
                    }
                    pix[kRenderPx * gl + k] = dpx;
                }
                __builtin_amdgcn_wave_barrier();
                if (need) {
#pragma unroll
                    for (int q = 0; q < kRenderPx / 4; ++q) {
                        const u32x4 v = pix4[wave][4 * lane + q];
                        p[4 * q] = v.x;
                        p[4 * q + 1] = v.y;
                        p[4 * q + 2] = v.z;
                        p[4 * q + 3] = v.w;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (kMode != 4 && i < items) {
                uint32_t w[12];
#pragma unroll
                for (int q = 0; q < kRenderPx / 4; ++q) {
                    const uint32_t a0 = __builtin_amdgcn_perm(0u, p[4 * q], psel),
                                   a1 = __builtin_amdgcn_perm(0u, p[4 * q + 1], psel),
                                   a2 = __builtin_amdgcn_perm(0u, p[4 * q + 2], psel),
                                   a3 = __builtin_amdgcn_perm(0u, p[4 * q + 3], psel);
                    w[3 * q] = a0 | (a1 << 24);
                    w[3 * q + 1] = (a1 >> 8) | (a2 << 16);
                    w[3 * q + 2] = (a2 >> 16) | (a3 << 8);
                }
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    pix4[wave][3 * lane + q] = u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
            }
            __builtin_amdgcn_wave_barrier();
            const int nbytes = 48 * (items - w0 < 64 ? (items - w0 > 0 ? items - w0 : 0) : 64);
            u32x4* dst = (u32x4*)(out + (e0 + qe) * img_bytes + (int64_t)ty * tile * row_px * 3 + (int64_t)w0 * 48);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int off = q * 64 + lane;
                const u32x4 val = kMode == 4 ? u32x4{(uint32_t)off, p0[0], (uint32_t)w0, 0u} : pix4[wave][off];
                if (off * 16 < nbytes) __builtin_nontemporal_store(val, dst + off);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

}  // namespace

int main() {
    const int64_t B = 1024;
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
    uint8_t *s0, *s1, *acts;
    CK(hipMalloc(&s0, S)); CK(hipMalloc(&s1, S)); CK(hipMalloc(&acts, 4 * P));
    oc_reset(h, s0, B, nullptr);
    for (int r = 0; r < 37; ++r) {
        oc_gen_actions(h, acts, B, 0, r, 13, nullptr);
        oc_step(h, r & 1 ? s1 : s0, r & 1 ? s0 : s1, acts, nullptr, nullptr, nullptr, B, nullptr);
    }
    uint8_t* st = s1;  // after 37 steps (odd count) the state is in s1
    // the bench's desc shape: sizes 80/56/40/28 at 0/12/40/46, 10 food sprites per class, 2 plates, 4 agents
    oc_render_desc desc{};
    desc.tile = 80;
    const int sizes[4] = {80, 56, 40, 28}, offs[4] = {0, 12, 40, 46};
    int off = 0;
    for (int c = 0; c < 4; ++c) {
        desc.size[c] = sizes[c];
        desc.offset[c] = offs[c];
        desc.food_base[c] = off;
        off += 10 * sizes[c] * sizes[c];
    }
    desc.plate_off[0] = off; off += 80 * 80;
    desc.plate_off[1] = off; off += 40 * 40;
    for (int a = 0; a < 4; ++a) { desc.agent_off[a] = off; off += 80 * 80; }
    for (int m = 0; m < 128; ++m) desc.food_sprite[m] = (m & ~OC_M_PLATE) == 0 ? 0xFF : (uint8_t)(m % 10);
    desc.chan_map = OC_CHAN_REFERENCE;
    std::mt19937 rng(5);
    std::vector<uint32_t> atlas(off), bgh(7 * 80 * 7 * 80);
    for (auto& v : atlas) {
        const uint32_t rgb = rng() & 0xFFFFFFu, k = rng() % 3;
        v = rgb | (k == 0 ? 0u : k == 1 ? 0xFF000000u : (rng() & 0xFFu) << 24);
    }
    for (auto& v : bgh) v = rng();
    uint32_t *atlas_d, *bg_d;
    CK(hipMalloc(&atlas_d, atlas.size() * 4)); CK(hipMalloc(&bg_d, bgh.size() * 4));
    CK(hipMemcpy(atlas_d, atlas.data(), atlas.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bg_d, bgh.data(), bgh.size() * 4, hipMemcpyHostToDevice));
    const int64_t img = 560 * 560 * 3;
    uint8_t *o0, *o1;
    CK(hipMalloc(&o0, B * img)); CK(hipMalloc(&o1, B * img));
    // RenderArgs exactly as oc_render builds them
    RenderArgs R;
    R.W = 7; R.H = 7; R.tile = 80;
    for (int c = 0; c < 4; ++c) { R.size[c] = desc.size[c]; R.offset[c] = desc.offset[c]; R.food_base[c] = desc.food_base[c]; }
    R.plate_off[0] = desc.plate_off[0]; R.plate_off[1] = desc.plate_off[1];
    for (int a = 0; a < OC_MAX_AGENTS; ++a) R.agent_off[a] = desc.agent_off[a];
    R.chan_map = desc.chan_map;
    R.parts = 1;
    R.pitch = P;
    for (int m = 0; m < 128; ++m) R.food_sprite[m] = desc.food_sprite[m];
    const dim3 grid((unsigned)(B * 7));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto time = [&](const char* name, auto&& fn) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; ++i) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 20;
        printf("%-40s %8.2f us/launch  %.2f TB/s\n", name, us, B * (double)img / (us * 1e-6) / 1e12);
    };
    auto product = [&]() {
        if (oc_render(h, st, atlas_d, bg_d, &desc, o0, B, nullptr) != 0) { printf("render: %s\n", oc_last_error()); exit(1); }
    };
    auto launch = [&](auto kern, int epb) {
        const dim3 g((unsigned)((B + epb - 1) / epb * 7));
        const size_t lds = (size_t)epb * 7 * (2 * kRenderMaxDraw + 1) * 4;
        hipLaunchKernelGGL(kern, g, dim3(kBlock), lds, nullptr, R, st, atlas_d, bg_d, o1, B);
    };
    auto lane_blend = [&]() {
        hipLaunchKernelGGL((render_lane_blend<4, 4>), grid, dim3(kBlock), 0, nullptr, R, st, atlas_d, bg_d, o1);
    };
    auto c1 = [&]() { launch(render_compact<4, 4, 1, 3>, 1); };
    auto c1b = [&]() { launch(render_compact<4, 4, 1, 0>, 1); };
    auto c2 = [&]() { launch(render_compact<4, 4, 2, 3>, 2); };
    auto c4 = [&]() { launch(render_compact<4, 4, 4, 3>, 4); };
    auto nb1 = [&]() { launch(render_compact<4, 4, 1, 1>, 1); };
    auto so1 = [&]() { launch(render_compact<4, 4, 1, 4>, 1); };
    auto nl1 = [&]() { launch(render_compact<4, 4, 1, 2>, 1); };
    std::vector<uint8_t> h0(B * img), h1(B * img);
    auto check = [&](const char* name) {
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h0.data(), o0, B * img, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h1.data(), o1, B * img, hipMemcpyDeviceToHost));
        int64_t diff = 0;
        for (int64_t k = 0; k < B * img; ++k) diff += h0[k] != h1[k];
        printf("%s: %lld differing bytes\n", name, (long long)diff);
    };
    auto parts = [&](int n) {
        RenderArgs Rp = R;
        Rp.parts = n;
        hipLaunchKernelGGL((oc_render_kernel<4, 4>), dim3((unsigned)(B * 7 * n)), dim3(kBlock), 0, nullptr, Rp, st, atlas_d,
                           bg_d, o1);
    };
    auto p1 = [&]() { parts(1); };
    auto p2 = [&]() { parts(2); };
    auto p3 = [&]() { parts(3); };
    auto p4 = [&]() { parts(4); };
    product();
    CK(hipMemset(o1, 0, B * img)); lane_blend(); check("lane blend");
    CK(hipMemset(o1, 0, B * img)); c1(); check("compact 1");
    CK(hipMemset(o1, 0, B * img)); p1(); check("product, 1 block per strip");
    CK(hipMemset(o1, 0, B * img)); p3(); check("product, 3 blocks per strip");
    CK(hipMemset(o1, 0, B * img)); p4(); check("product, 4 blocks per strip");
    for (int rep = 0; rep < 3; ++rep) {
        time("lane blend (round-2 kernel)", lane_blend);
        time("product (oc_render: 2 blocks per strip)", product);
        time("product, 1 block per strip", p1);
        time("product, 2 blocks per strip", p2);
        time("product, 3 blocks per strip", p3);
        time("product, 4 blocks per strip", p4);
        time("compact 1, no blend", nb1);
        time("compact 1, no blend, no level image", nl1);
        time("compact 1, stores only (no LDS staging)", so1);
    }
    return 0;
}
