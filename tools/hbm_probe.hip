// hbm_probe.hip -- calibrate achievable HBM streaming rates on the box (read+write copy, read-only,
// write-only) for the access shapes the update kernel can use.  Standalone: hipcc -O3
// --offload-arch=gfx950 tools/hbm_probe.hip -o tools/hbm_probe && tools/hbm_probe [GiB]
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));

// grid-stride copy, U 16-B loads in flight per lane
template <int U, bool NT>
__global__ void k_copy_gs(const dbl2* __restrict__ a, dbl2* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long s = (long)gridDim.x * blockDim.x;
    for (; i + (U - 1) * s < n; i += U * s) {
        dbl2 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = a[i + k * s];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (NT)
                __builtin_nontemporal_store(v[k], &b[i + k * s]);
            else
                b[i + k * s] = v[k];
        }
    }
    for (; i < n; i += s) b[i] = a[i];
}

// each wave owns a contiguous range; per iteration 64 lanes x U x 16 B
template <int U>
__global__ void k_copy_wave(const dbl2* __restrict__ a, dbl2* __restrict__ b, long n) {
    const long nw = (long)gridDim.x * (blockDim.x / 64);
    const long w = (long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long per = (n + nw - 1) / nw;
    long lo = w * per, hi = lo + per;
    if (hi > n) hi = n;
    for (long i = lo + lane; i < hi; i += 64 * U) {
        dbl2 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = (i + 64 * k < hi) ? a[i + 64 * k] : dbl2{0, 0};
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (i + 64 * k < hi) b[i + 64 * k] = v[k];
    }
}

template <int U>
__global__ void k_read(const dbl2* __restrict__ a, double* out, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long s = (long)gridDim.x * blockDim.x;
    double acc = 0;
    for (; i + (U - 1) * s < n; i += U * s) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            dbl2 v = a[i + k * s];
            acc += v.x + v.y;
        }
    }
    if (acc == 12345.678) out[0] = acc;
}

__global__ void k_fill(dbl2* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long s = (long)gridDim.x * blockDim.x;
    for (; i < n; i += s) b[i] = dbl2{1.0, 2.0};
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
    double* out;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int iters = 10;
    printf("{\"probe\":\"config\",\"bytes_per_buffer\":%ld,\"cus\":%d}\n", bytes, cus);
    for (int threads : {256, 512, 1024}) {
        for (int bpc : {1, 2, 4, 8, 16}) {
            int blocks = cus * bpc * 256 / threads;
            if (blocks < cus) continue;
            float ms;
#define RUN(NAME, KERNEL, TRAFFIC)                                                         \
    ms = timeit([&] { hipLaunchKernelGGL(KERNEL, dim3(blocks), dim3(threads), 0, 0, a, b, n); }, iters); \
    printf("{\"probe\":\"%s\",\"threads\":%d,\"blocks\":%d,\"ms\":%.4f,\"gbs\":%.1f}\n", NAME, threads, \
           blocks, ms, (TRAFFIC) / ms / 1e6);
            RUN("copy_gs_u1", (k_copy_gs<1, false>), 2.0 * bytes)
            RUN("copy_gs_u4", (k_copy_gs<4, false>), 2.0 * bytes)
            RUN("copy_gs_u8", (k_copy_gs<8, false>), 2.0 * bytes)
            RUN("copy_gs_u4_nt", (k_copy_gs<4, true>), 2.0 * bytes)
            RUN("copy_wave_u4", (k_copy_wave<4>), 2.0 * bytes)
            RUN("copy_wave_u8", (k_copy_wave<8>), 2.0 * bytes)
            ms = timeit([&] { hipLaunchKernelGGL((k_read<4>), dim3(blocks), dim3(threads), 0, 0, a, out, n); }, iters);
            printf("{\"probe\":\"read_u4\",\"threads\":%d,\"blocks\":%d,\"ms\":%.4f,\"gbs\":%.1f}\n", threads,
                   blocks, ms, 1.0 * bytes / ms / 1e6);
            ms = timeit([&] { hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(threads), 0, 0, b, n); }, iters);
            printf("{\"probe\":\"fill\",\"threads\":%d,\"blocks\":%d,\"ms\":%.4f,\"gbs\":%.1f}\n", threads,
                   blocks, ms, 1.0 * bytes / ms / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
