// Issue rate of single VALU opcodes on the GPU it runs on (profiling aid for the
// lane-phase instruction mix): every wave runs N iterations of 16 independent
// instances of one opcode (inline asm, no memory traffic); the whole grid is
// timed with HIP events, and the rate is reported as wave-instructions per CU
// per cycle at the measured shader clock (MI355X: 256 CUs).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
//   tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(X) X X X X X X X X X X X X X X X X

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(int n, unsigned* out) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 1u, a5 = a0 + 2u, a6 = a0 + 3u,
             a7 = a0 + 4u;
    unsigned long long b0 = a0, b1 = a1, b2 = a2, b3 = a3;
    const unsigned sh = threadIdx.x & 31u;
    for (int i = 0; i < n; ++i) {
        if constexpr (OP == 0) {   // v_lshlrev_b64
            asm volatile(REP16("v_lshlrev_b64 %0, %4, %0\n v_lshlrev_b64 %1, %4, %1\n v_lshlrev_b64 %2, %4, %2\n v_lshlrev_b64 %3, %4, %3\n")
                         : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(sh));
        } else if constexpr (OP == 1) {   // v_lshlrev_b32
            asm volatile(REP16("v_lshlrev_b32 %0, %8, %0\n v_lshlrev_b32 %1, %8, %1\n v_lshlrev_b32 %2, %8, %2\n v_lshlrev_b32 %3, %8, %3\n"
                               "v_lshlrev_b32 %4, %8, %4\n v_lshlrev_b32 %5, %8, %5\n v_lshlrev_b32 %6, %8, %6\n v_lshlrev_b32 %7, %8, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(sh));
        } else if constexpr (OP == 2) {   // v_or3_b32
            asm volatile(REP16("v_or3_b32 %0, %0, %8, %8\n v_or3_b32 %1, %1, %8, %8\n v_or3_b32 %2, %2, %8, %8\n v_or3_b32 %3, %3, %8, %8\n"
                               "v_or3_b32 %4, %4, %8, %8\n v_or3_b32 %5, %5, %8, %8\n v_or3_b32 %6, %6, %8, %8\n v_or3_b32 %7, %7, %8, %8\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(sh));
        } else if constexpr (OP == 3) {   // v_mul_lo_u32
            asm volatile(REP16("v_mul_lo_u32 %0, %8, %0\n v_mul_lo_u32 %1, %8, %1\n v_mul_lo_u32 %2, %8, %2\n v_mul_lo_u32 %3, %8, %3\n"
                               "v_mul_lo_u32 %4, %8, %4\n v_mul_lo_u32 %5, %8, %5\n v_mul_lo_u32 %6, %8, %6\n v_mul_lo_u32 %7, %8, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(sh));
        } else if constexpr (OP == 4) {   // v_bcnt_u32_b32
            asm volatile(REP16("v_bcnt_u32_b32 %0, %8, %0\n v_bcnt_u32_b32 %1, %8, %1\n v_bcnt_u32_b32 %2, %8, %2\n v_bcnt_u32_b32 %3, %8, %3\n"
                               "v_bcnt_u32_b32 %4, %8, %4\n v_bcnt_u32_b32 %5, %8, %5\n v_bcnt_u32_b32 %6, %8, %6\n v_bcnt_u32_b32 %7, %8, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(sh));
        } else if constexpr (OP == 5) {   // v_lshl_or_b32
            asm volatile(REP16("v_lshl_or_b32 %0, %8, %8, %0\n v_lshl_or_b32 %1, %8, %8, %1\n v_lshl_or_b32 %2, %8, %8, %2\n v_lshl_or_b32 %3, %8, %8, %3\n"
                               "v_lshl_or_b32 %4, %8, %8, %4\n v_lshl_or_b32 %5, %8, %8, %5\n v_lshl_or_b32 %6, %8, %8, %6\n v_lshl_or_b32 %7, %8, %8, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(sh));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)(b0 ^ b1 ^ b2 ^ b3);
}

template <int OP>
static double run(int grid, int n, unsigned* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(grid), dim3(256), 0, 0, n, out);   // warm-up
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(grid), dim3(256), 0, 0, n, out);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms;
}

int main() {
    int dev = 0, cus = 0, clk_khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    const int grid = cus * 8, n = 2000;     // 8 workgroups of 4 waves per CU
    unsigned* out = nullptr;
    if (hipMalloc(&out, sizeof(unsigned) * grid * 256) != hipSuccess) return 1;
    const char* names[] = {"v_lshlrev_b64", "v_lshlrev_b32", "v_or3_b32", "v_mul_lo_u32", "v_bcnt_u32_b32", "v_lshl_or_b32"};
    const int per_iter[] = {64, 128, 128, 128, 128, 128};
    double ms[6] = {run<0>(grid, n, out), run<1>(grid, n, out), run<2>(grid, n, out), run<3>(grid, n, out),
                    run<4>(grid, n, out), run<5>(grid, n, out)};
    const double waves = (double)grid * 4.0, cyc = (double)clk_khz * 1e3;
    printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"rates\": {", cus, cyc / 1e6);
    for (int i = 0; i < 6; ++i) {
        const double winstr = waves * n * per_iter[i];
        const double per_cu_cycle = winstr / (ms[i] * 1e-3 * cyc * cus);
        printf("%s\"%s\": {\"ms\": %.3f, \"wave_instr_per_cu_cycle\": %.3f}", i ? ", " : "", names[i], ms[i], per_cu_cycle);
    }
    printf("}}\n");
    (void)hipFree(out);
    return 0;
}
