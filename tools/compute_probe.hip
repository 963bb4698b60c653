// fp64 arithmetic rate of the block sweep's per-element chain, without memory traffic.
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang fp contract(off)
typedef double dbl2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool fd_in(double x) {
    const unsigned bexp = ((unsigned)(__double_as_longlong(x) >> 52)) & 0x7ffu;
    return bexp - 896u <= 1152u - 896u;
}
struct Piv { int r[8], c[8]; double e[8], y[8]; };
// V: 0 full (num + fd check/branch), 1 fast div no check, 2 numerator + IEEE div, 3 numerator only,
//    4 fma chain (6 fma per step), 5 num + fast div + accumulated check (no branch)
template <int V, int NE>
__global__ __launch_bounds__(256) void k_comp(double* out, int iters, Piv pv, double pr0, double pc0) {
    double v[NE];
    for (int h = 0; h < NE; ++h) v[h] = 0.5 + 1e-3 * (threadIdx.x + h);
    int bad = 0;
    double mn = 1e300, mx = 0.0;
    unsigned emn = 0xffffffffu, emx = 0u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const double e = pv.e[l], y = pv.y[l];
            const double pr = pr0 + l, pc = pc0 - l;
#pragma unroll
            for (int h = 0; h < NE; ++h) {
                if (V == 4) {
                    double t = fma(v[h], e, pr);
                    t = fma(t, y, pc); t = fma(t, e, pr); t = fma(t, y, pc); t = fma(t, e, pr);
                    v[h] = fma(t, y, pc);
                    continue;
                }
                const double num = v[h] * e - pr * pc;
                if (V == 3) { v[h] = num; continue; }
                if (V == 2) { v[h] = num / e; continue; }
                const double q = num * y;
                const double r = fma(-e, q, num);
                const double f = fma(r, y, q);
                if (V == 1) { v[h] = f; continue; }
                if (V == 5) { bad |= !fd_in(num); v[h] = f; continue; }
                if (V == 6) { mn = fmin(mn, fabs(num)); mx = fmax(mx, fabs(num)); v[h] = f; continue; }
                if (V == 7) {
                    const unsigned ex = ((unsigned)(__double_as_longlong(num) >> 52)) & 0x7ffu;
                    emn = min(emn, ex); emx = max(emx, ex); v[h] = f; continue;
                }
                v[h] = fd_in(num) ? f : num / e;
            }
        }
    }
    double s = 0;
    for (int h = 0; h < NE; ++h) s += v[h];
    out[blockIdx.x * 256 + threadIdx.x] = s + bad + mn + mx + emn + emx;
}
template <int V, int NE>
void run(double* out, Piv pv, const char* name) {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 8, iters = 2000;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k_comp<V, NE>), dim3(grid), dim3(256), 0, 0, out, 10, pv, 0.3, 0.7);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_comp<V, NE>), dim3(grid), dim3(256), 0, 0, out, iters, pv, 0.3, 0.7);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double ep = (double)grid * 256 * iters * 8 * NE;
    printf("{\"variant\": \"%s\", \"NE\": %d, \"ms\": %.3f, \"Gelem_pivots_s\": %.1f, \"ns_per_elem_pivot_per_CU\": %.4f, \"cyc_per_64ep_per_SIMD\": %.1f}\n",
           name, NE, ms, ep / ms / 1e6, ms * 1e6 * cus / ep, ms * 1e-3 * 2.4e9 * cus * 4 / ep * 64);
}
int main() {
    double* out; hipMalloc(&out, 1 << 26);
    Piv pv; for (int l = 0; l < 8; ++l) { pv.e[l] = 0.75 + 0.01 * l; pv.y[l] = 1.0 / pv.e[l]; pv.r[l] = l; pv.c[l] = l; }
    run<4, 4>(out, pv, "fma_chain_6");
    run<3, 4>(out, pv, "numerator_only");
    run<1, 4>(out, pv, "num_fastdiv_nocheck");
    run<5, 4>(out, pv, "num_fastdiv_acccheck");
    run<0, 4>(out, pv, "num_fastdiv_branch");
    run<2, 4>(out, pv, "num_ieee_div");
    run<6, 4>(out, pv, "num_fastdiv_minmax_f64");
    run<7, 4>(out, pv, "num_fastdiv_minmax_exp");
    run<6, 8>(out, pv, "num_fastdiv_minmax_f64");
    run<7, 8>(out, pv, "num_fastdiv_minmax_exp");
    run<1, 8>(out, pv, "num_fastdiv_nocheck");
    run<0, 8>(out, pv, "num_fastdiv_branch");
    return 0;
}
