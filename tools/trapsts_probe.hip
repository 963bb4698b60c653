// trapsts_probe.hip -- do the per-wave sticky fp exception bits (TRAPSTS.EXCP) accumulate on
// gfx950 with traps disabled, and can a kernel clear and read them?  If so, the block sweep can
// replace its per-element exponent-window tracking (1.5 integer VALU ops per element and pivot,
// csrc/smx_block.hpp win_term) by one read of the wave's exception bits per unit.
//
// Every case: clear EXCP (s_setreg), one fp64 op on operands loaded from memory (no constant
// folding), wait for its result (v_readfirstlane into an SGPR that the read then depends on),
// read TRAPSTS[8:0] (s_getreg), store the bits with a vector store.  Case "race" reads with no
// wait right after a dependent chain of 16 ops whose LAST op overflows.
// EXCP bits (GCN/CDNA): 0 invalid, 1 input denormal, 2 div by zero, 3 overflow, 4 underflow,
// 5 inexact, 6 int div by zero, 7 address watch, 8 memory violation.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/trapsts_probe.hip -o tools/trapsts_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

// the operands pass through the asm, so the op that uses them cannot be hoisted above the clear
__device__ __forceinline__ void excp_clear(double& a, double& b) {
    asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_TRAPSTS, 0, 9), 0\n s_nop 3"
                 : "+v"(a), "+v"(b)::"memory");
}

// the bits after the op that produced v (v's producer has completed: the SGPR copy of v's low
// dword is an input of the s_or that precedes the read)
__device__ __forceinline__ unsigned excp_read_after(double v) {
    unsigned f, t;
    asm volatile(
        "v_readfirstlane_b32 %1, %2\n"
        "s_or_b32 %1, %1, 0\n"
        "s_nop 3\n"
        "s_getreg_b32 %0, hwreg(HW_REG_TRAPSTS, 0, 9)\n"
        : "=s"(f), "=&s"(t)
        : "v"(__double2loint(v))
        : "memory");
    return f;
}

// no wait: v is only an operand of the asm for the compiler (the read is placed after v's
// producer is ISSUED; the hardware does not wait for it to complete)
__device__ __forceinline__ unsigned excp_read_now(double v = 0.0) {
    unsigned f;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_TRAPSTS, 0, 9)" : "=s"(f) : "v"(v) : "memory");
    return f;
}

constexpr int kCases = 16;

__global__ void k_probe(const double* __restrict__ in, unsigned* __restrict__ out,
                        double* __restrict__ vals) {
    const int lane = threadIdx.x;
    // operands (host-filled): see main
    const double one = in[0], tiny = in[1], huge = in[2], inf = in[3], den = in[4],
                 third = in[5], qnan = in[6], p530 = in[7], three = in[8], negz = in[9];
    unsigned f[kCases];
    double v;
    int k = 0;
    // one case: the operands pass through the clear, so the op cannot be hoisted above it
#define CASE(A, B, EXPR)                                                   \
    do {                                                                   \
        double a = (A), b = (B);                                           \
        excp_clear(a, b);                                                  \
        v = (EXPR);                                                        \
        f[k] = excp_read_after(v);                                         \
        vals[k++ * 64 + lane] = v;                                         \
    } while (0)
    CASE(one, 1.5, a * b);                          // 0 exact
    CASE(tiny, tiny, a * b);                        // 1 underflow
    CASE(huge, huge, a * b);                        // 2 overflow
    CASE(inf, inf, a - b);                          // 3 invalid
    CASE(den, one, a * b);                          // 4 denormal input
    CASE(one, third, a * b);                        // 5 exact (1 * x)
    CASE(third, three, a * b);                      // 6 inexact
    CASE(qnan, three, a * b);                       // 7 quiet NaN input
    CASE(p530, p530, a * b);                        // 8 exact denormal result
    CASE(one, three, a / b);                        // 9 IEEE division sequence
    CASE(third, three, fma(-b, a, one));            // 10 fma residual
    CASE(lane == 5 ? tiny : one, tiny, a * b);      // 11 only lane 5 underflows
    {   // 12 race: a dependent chain of 16 multiplies, the last overflows; read with no wait
        double a = one, b = huge;
        excp_clear(a, b);
        double x = a;
#pragma unroll
        for (int q = 0; q < 15; ++q) x = x * a;
        x = x * b * b;
        f[k] = excp_read_now(x);
        vals[k++ * 64 + lane] = x;
    }
    CASE(huge, huge, (a * b) * 0.0 + 1.5);          // 13 sticky: overflow, then exact ops
    CASE(negz, three, a * b);                       // 14 -0 * 3
    {   // 15 cleared
        double a = one, b = one;
        excp_clear(a, b);
        f[k] = excp_read_now();
        vals[k++ * 64 + lane] = a + b;
    }
    if (lane == 0)
        for (int i = 0; i < kCases; ++i) out[i] = f[i];
}

int main() {
    double h[10];
    h[0] = 1.0;
    h[1] = 1e-300;
    h[2] = 1e300;
    h[3] = INFINITY;
    h[4] = 4.9406564584124654e-324 * 7;
    h[5] = 1.0 / 3.0;
    h[6] = NAN;
    h[7] = ldexp(1.0, -530);
    h[8] = 3.0;
    h[9] = -0.0;
    double *din, *dv;
    unsigned* dout;
    if (hipMalloc(&din, sizeof h) || hipMalloc(&dout, kCases * 4) ||
        hipMalloc(&dv, kCases * 64 * 8)) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipMemset(dout, 0xff, kCases * 4);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, din, dout, dv);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        fprintf(stderr, "kernel: %s\n", hipGetErrorString(e));
        return 1;
    }
    unsigned o[kCases];
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    const char* names[kCases] = {"exact", "underflow", "overflow", "invalid", "denorm_in",
                                 "one_times", "inexact", "qnan_in", "exact_denorm", "ieee_div",
                                 "fma_resid", "lane5_underflow", "race_no_wait", "sticky",
                                 "negzero", "cleared"};
    printf("{");
    for (int i = 0; i < kCases; ++i)
        printf("%s\"%s\": \"0x%03x\"", i ? ", " : "", names[i], o[i]);
    printf("}\n");
    return 0;
}
