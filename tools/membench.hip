// tools/membench.hip -- memory-pattern microbenchmark for the step kernel's plane layout.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/membench tools/membench.hip
// Each variant moves the same bytes as one oc_step<2,4> at B envs (19 read planes, 20 write
// planes of B bytes) with no compute, so the difference to the step kernel is compute/latency.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

constexpr int NR = 19, NW = 20;

// read NR planes, write NW planes, `EPL` bytes per lane per plane, plane stride `pitch`
template <int W>  // bytes per lane: 4 (dword), 8, 16
__global__ __launch_bounds__(256) void planes_copy(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                   long pitch, unsigned nlanes) {
    using V = typename std::conditional<W == 4, unsigned, typename std::conditional<W == 8, uint2, uint4>::type>::type;
    const unsigned stride = gridDim.x * 256;
    for (unsigned g = blockIdx.x * 256 + threadIdx.x; g < nlanes; g += stride) {
        V v[NR];
#pragma unroll
        for (int p = 0; p < NR; ++p) v[p] = reinterpret_cast<const V*>(in + p * pitch)[g];
#pragma unroll
        for (int p = 0; p < NW; ++p) reinterpret_cast<V*>(out + p * pitch)[g] = v[p % NR];
    }
}

__global__ __launch_bounds__(256) void flat_copy(const uint4* __restrict__ in, uint4* __restrict__ out, long n16) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

template <class F>
float time_it(F f, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) f();
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;  // us
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : (1l << 20);
    const int iters = 200;
    const long maxpitch = B + 64 * 4096;
    uint8_t *in, *out;
    CK(hipMalloc(&in, NR * maxpitch + (1 << 20)));
    CK(hipMalloc(&out, NW * maxpitch + (1 << 20)));
    CK(hipMemset(in, 1, NR * maxpitch));
    CK(hipMemset(out, 0, NW * maxpitch));
    const double bytes = (double)(NR + NW) * B;
    printf("B=%ld bytes/launch=%.1f MB\n", B, bytes / 1e6);
    {
        const long n16 = (long)(bytes / 2) / 16;
        for (int grid : {1024, 2048, 4096, 8192}) {
            float us = time_it([&] { hipLaunchKernelGGL(flat_copy, dim3(grid), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, n16); }, iters);
            printf("flat_copy16 grid %5d: %7.2f us  %6.2f TB/s\n", grid, us, 2.0 * n16 * 16 / us / 1e6);
        }
    }
    for (long pad : {0l, 4096l, 12288l, 65536l + 4096l}) {
        const long pitch = B + pad;
        for (int grid : {512, 1024, 2048, 4096}) {
            const unsigned n4 = (unsigned)(B / 4), n8 = (unsigned)(B / 8), n16 = (unsigned)(B / 16);
            float u4 = time_it([&] { hipLaunchKernelGGL(planes_copy<4>, dim3(std::min<long>(grid, n4 / 256)), dim3(256), 0, 0, in, out, pitch, n4); }, iters);
            float u8 = time_it([&] { hipLaunchKernelGGL(planes_copy<8>, dim3(std::min<long>(grid, n8 / 256)), dim3(256), 0, 0, in, out, pitch, n8); }, iters);
            float u16 = time_it([&] { hipLaunchKernelGGL(planes_copy<16>, dim3(std::min<long>(grid, n16 / 256)), dim3(256), 0, 0, in, out, pitch, n16); }, iters);
            printf("planes pad %6ld grid %5d: dword %7.2f us (%5.2f TB/s)  dwordx2 %7.2f us (%5.2f)  dwordx4 %7.2f us (%5.2f)\n",
                   pad, grid, u4, bytes / u4 / 1e6, u8, bytes / u8 / 1e6, u16, bytes / u16 / 1e6);
        }
    }
    return 0;
}
