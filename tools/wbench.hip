// tools/wbench.hip -- write-only HBM bandwidth in oc_step_n's output shape: per "step", 20 byte
// planes of P bytes (17 state + 2 exec + 1 coll), written one dword per lane (4 envs), vs wider
// per-lane stores and non-temporal hints.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/wbench tools/wbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                          \
    do {                                                                                               \
        hipError_t e = (x);                                                                            \
        if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

constexpr int NPL = 20;

// one dword per lane per plane per step (the kernel's pattern); value depends on r so nothing folds
template <bool NT>
__global__ __launch_bounds__(256) void w_dword(uint32_t* out, long P4, int steps) {
    const long g = blockIdx.x * 256l + threadIdx.x;
    if (g >= P4) return;
    uint32_t v = (uint32_t)g * 2654435761u;
    for (int r = 0; r < steps; ++r) {
        uint32_t* base = out + (long)r * NPL * P4;
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
            v = v * 1664525u + 1013904223u;
            if (NT) __builtin_nontemporal_store(v, base + p * P4 + g);
            else base[p * P4 + g] = v;
        }
    }
}

// same bytes, 16 B per lane: a quarter of the lanes, each writes 4 consecutive dwords of a plane
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void w_dwordx4(u32x4* out, long P16, int steps) {
    const long g = blockIdx.x * 256l + threadIdx.x;
    if (g >= P16) return;
    uint32_t v = (uint32_t)g * 2654435761u;
    for (int r = 0; r < steps; ++r) {
        u32x4* base = out + (long)r * NPL * P16;
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
            v = v * 1664525u + 1013904223u;
            const u32x4 w = {v, v ^ 1u, v ^ 2u, v ^ 3u};
            if (NT) __builtin_nontemporal_store(w, base + p * P16 + g);
            else base[p * P16 + g] = w;
        }
    }
}

// plane-major layout ([step][plane][P]), waves staggered: wave w starts at step (w * 37) % steps
// and wraps, so concurrently running waves write different steps (as oc_step_n's waves drift)
template <bool TILED>
__global__ __launch_bounds__(256) void w_stagger(uint32_t* out, long P4, int steps, int stagger) {
    const long g = blockIdx.x * 256l + threadIdx.x;
    if (g >= P4) return;
    const long wave = g >> 6, lane = g & 63;
    uint32_t v = (uint32_t)g * 2654435761u;
    const int r0 = stagger ? (int)((wave * 37) % steps) : 0;
    for (int i = 0; i < steps; ++i) {
        int r = r0 + i;
        r = r >= steps ? r - steps : r;
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
            v = v * 1664525u + 1013904223u;
            long off;
            if (TILED)  // [step][wave tile][plane][64 dwords]: a wave's 20 stores fill one 5 KB block
                off = ((long)r * (P4 / 64) + wave) * (NPL * 64) + p * 64 + lane;
            else
                off = (long)r * NPL * P4 + p * P4 + g;
            out[off] = v;
        }
    }
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : (1l << 20);
    const int steps = 100;
    const long bytes = (long)steps * NPL * B;
    uint8_t* buf;
    CK(hipMalloc(&buf, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int i = 0; i < 5; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1000.0 / 5;
        printf("%-34s %8.1f us/launch  %6.2f us/step  %5.2f TB/s\n", name, us, us / steps, bytes / us / 1e6);
    };
    const long P4 = B / 4, P16 = B / 16;
    for (int grid_scale : {1}) {
        (void)grid_scale;
        run("dword per lane", [&] { hipLaunchKernelGGL(w_dword<false>, dim3((P4 + 255) / 256), dim3(256), 0, 0, (uint32_t*)buf, P4, steps); });
        run("dword per lane, nontemporal", [&] { hipLaunchKernelGGL(w_dword<true>, dim3((P4 + 255) / 256), dim3(256), 0, 0, (uint32_t*)buf, P4, steps); });
        run("dwordx4 per lane", [&] { hipLaunchKernelGGL(w_dwordx4<false>, dim3((P16 + 255) / 256), dim3(256), 0, 0, (u32x4*)buf, P16, steps); });
        run("plane-major, staggered waves", [&] { hipLaunchKernelGGL(w_stagger<false>, dim3((P4 + 255) / 256), dim3(256), 0, 0, (uint32_t*)buf, P4, steps, 1); });
        run("tiled 5 KB per wave, lockstep", [&] { hipLaunchKernelGGL(w_stagger<true>, dim3((P4 + 255) / 256), dim3(256), 0, 0, (uint32_t*)buf, P4, steps, 0); });
        run("tiled 5 KB per wave, staggered", [&] { hipLaunchKernelGGL(w_stagger<true>, dim3((P4 + 255) / 256), dim3(256), 0, 0, (uint32_t*)buf, P4, steps, 1); });
        run("dwordx4 per lane, nontemporal", [&] { hipLaunchKernelGGL(w_dwordx4<true>, dim3((P16 + 255) / 256), dim3(256), 0, 0, (u32x4*)buf, P16, steps); });
    }
    return 0;
}
