// tools/valubench.hip -- per-SIMD VALU throughput of the integer ops the step kernel uses.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/valubench tools/valubench.hip
// Each lane runs 8 independent asm chains of one instruction; waves per SIMD = W.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

constexpr int ITERS = 2048;

#define CHAIN8(INS)                                                                          \
    asm volatile(INS : "+v"(a0) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a1) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a2) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a3) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a4) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a5) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a6) : "v"(b), "v"(c));                                                  \
    asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(unsigned* out, unsigned seed) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, b = seed, c = seed * 3u;
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (OP == 0) { CHAIN8("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 1) { CHAIN8("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96") }
        if constexpr (OP == 2) { CHAIN8("v_bfi_b32 %0, %1, %0, %1") }
        if constexpr (OP == 3) { CHAIN8("v_perm_b32 %0, %0, %1, %1") }
        if constexpr (OP == 4) { CHAIN8("v_bfe_u32 %0, %0, %1, 8") }
        if constexpr (OP == 5) { CHAIN8("v_cndmask_b32_e64 %0, %0, %1, vcc") }
        if constexpr (OP == 6) { CHAIN8("v_cmp_eq_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e64 %0, 0, -1, vcc") }
        if constexpr (OP == 7) { CHAIN8("v_lshl_or_b32 %0, %0, 3, %1") }
        if constexpr (OP == 8) { CHAIN8("v_mad_u32_u24 %0, %0, %1, %1") }
        if constexpr (OP == 9) { CHAIN8("v_xor_b32 %0, %0, %1") }
        if constexpr (OP == 10) { CHAIN8("v_cndmask_b32_e32 %0, %0, %1, vcc") }
        if constexpr (OP == 11) { CHAIN8("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xCA") }
        if constexpr (OP == 12) { CHAIN8("v_and_or_b32 %0, %0, %1, %2") }
        if constexpr (OP == 13) { CHAIN8("v_add3_u32 %0, %0, %1, %2") }
        if constexpr (OP == 14) { CHAIN8("v_lshrrev_b32 %0, %1, %0") }
        if constexpr (OP == 15) { CHAIN8("v_min_u32 %0, %0, %1") }
        if constexpr (OP == 16) { CHAIN8("v_mul_u32_u24 %0, %0, %1") }
        if constexpr (OP == 17) { CHAIN8("v_bcnt_u32_b32 %0, %0, %1") }
        if constexpr (OP == 18) { CHAIN8("v_ashrrev_i32 %0, 31, %0") }
        if constexpr (OP == 19) { CHAIN8("v_cmp_eq_u32_e64 s[40:41], %0, %1") }
        if constexpr (OP == 20) { CHAIN8("v_pk_add_u16 %0, %0, %1") }
        if constexpr (OP == 21) { CHAIN8("v_or3_b32 %0, %0, %1, %2") }
        if constexpr (OP == 22) { CHAIN8("v_lshl_add_u32 %0, %0, 2, %1") }
        if constexpr (OP == 23) { CHAIN8("v_add_u32_e64 %0, %0, %1") }
        if constexpr (OP == 24) { CHAIN8("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x96") }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
void run(const char* name, unsigned* out, int insts_per_chain) {
    for (int W : {4}) {
        const int grid = 256 * W;  // 256-thread blocks = one wave per SIMD each
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        hipLaunchKernelGGL(valu_kernel<OP>, dim3(grid), dim3(256), 0, 0, out, 7u);
        CK(hipEventRecord(a));
        const int reps = 5;
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(valu_kernel<OP>, dim3(grid), dim3(256), 0, 0, out, 7u);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double wave_insts_per_simd = (double)W * ITERS * 8 * insts_per_chain;  // per launch
        const double ns = ms * 1e6 / reps;
        printf("%-28s W=%d  %8.1f us  %.3f wave-instr/ns/SIMD  (%.2f cycles/instr at 2.4 GHz)\n", name, W, ns / 1e3,
               wave_insts_per_simd / ns, ns * 2.4 / wave_insts_per_simd);
    }
}

int main() {
    unsigned* out;
    CK(hipMalloc(&out, 256 * 8 * 256 * sizeof(unsigned)));
    run<0>("v_add_u32", out, 1);
    run<9>("v_xor_b32", out, 1);
    run<1>("v_bitop3_b32", out, 1);
    run<2>("v_bfi_b32", out, 1);
    run<3>("v_perm_b32", out, 1);
    run<4>("v_bfe_u32", out, 1);
    run<5>("v_cndmask_b32 (vcc)", out, 1);
    run<6>("v_cmp+v_cndmask pair", out, 2);
    run<7>("v_lshl_or_b32", out, 1);
    run<8>("v_mad_u32_u24", out, 1);
    run<10>("v_cndmask_b32_e32 (vcc)", out, 1);
    run<11>("v_bitop3 select 3 regs", out, 1);
    run<24>("v_bitop3 xor3 3 regs", out, 1);
    run<12>("v_and_or_b32", out, 1);
    run<13>("v_add3_u32", out, 1);
    run<21>("v_or3_b32", out, 1);
    run<14>("v_lshrrev_b32", out, 1);
    run<15>("v_min_u32", out, 1);
    run<16>("v_mul_u32_u24", out, 1);
    run<17>("v_bcnt_u32_b32", out, 1);
    run<18>("v_ashrrev_i32", out, 1);
    run<19>("v_cmp_eq_u32_e64 -> sgpr", out, 1);
    run<20>("v_pk_add_u16", out, 1);
    run<22>("v_lshl_add_u32", out, 1);
    run<23>("v_add_u32_e64", out, 1);
    return 0;
}
