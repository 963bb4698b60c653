// hbm_probe2.hip -- wider sweep of read+write streaming shapes on MI355X: bytes per lane (16/32),
// loads in flight per lane (U), non-temporal loads/stores, threads per block, blocks per CU.
// hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/hbm_probe2.hip -o tools/hbm_probe2
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ dbl2 L(const dbl2* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void S(dbl2* p, dbl2 v) {
    if (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// V = dbl2 per lane per unit (1: 16 B, 2: 32 B contiguous); U units in flight; grid-stride
template <int V, int U, bool NTL, bool NTS>
__global__ void k_copy(const dbl2* __restrict__ a, dbl2* __restrict__ b, long n) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long s = (long)gridDim.x * blockDim.x;
    const long units = n / V;
    for (long u = t; u < units; u += (long)U * s) {
        dbl2 v[U][V];
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int q = 0; q < V; ++q)
                v[k][q] = (u + k * s < units) ? L<NTL>(a + (u + k * s) * V + q) : dbl2{0, 0};
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int q = 0; q < V; ++q)
                if (u + k * s < units) S<NTS>(b + (u + k * s) * V + q, v[k][q]);
    }
}

template <typename F>
float timeit(F f, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

int main(int argc, char** argv) {
    double gib = argc > 1 ? atof(argv[1]) : 2.0;
    long bytes = (long)(gib * (1L << 30));
    long n = bytes / 16;
    dbl2 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int iters = 8;
#define RUN(V, U, NTL, NTS)                                                                   \
    {                                                                                         \
        float ms = timeit([&] { hipLaunchKernelGGL((k_copy<V, U, NTL, NTS>), dim3(blocks),     \
                                                   dim3(threads), 0, 0, a, b, n); }, iters);  \
        printf("{\"v\":%d,\"u\":%d,\"ntl\":%d,\"nts\":%d,\"threads\":%d,\"bpc\":%d,"            \
               "\"ms\":%.4f,\"gbs\":%.1f}\n", V, U, (int)NTL, (int)NTS, threads, bpc, ms,      \
               2.0 * bytes / ms / 1e6);                                                       \
        fflush(stdout);                                                                       \
    }
    for (int threads : {256, 512, 1024}) {
        for (int bpc : {1, 2, 3, 4, 6, 8}) {
            const int blocks = cus * bpc;
            if ((long)threads * bpc > 2048) continue;
            RUN(1, 1, false, false)
            RUN(1, 2, false, true)
            RUN(1, 4, false, true)
            RUN(1, 4, true, true)
            RUN(1, 8, true, true)
            RUN(2, 1, false, true)
            RUN(2, 2, false, true)
            RUN(2, 2, true, true)
            RUN(2, 4, true, true)
        }
    }
    return 0;
}
