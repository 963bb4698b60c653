// glds_probe.hip -- can a block sweep overlap its fp64 arithmetic with the HBM stream if every
// wave keeps S units of the tableau in flight through LDS-DMA (global_load_lds_dwordx4 into a
// per-wave LDS ring), instead of holding loads in VGPRs only while it is not computing?
// Same per-element work as smx_block.hpp's sweep fast path (P chained steps, numerators in the
// hoisted-reciprocal division, |num| min/max tracked, one vote per unit); pivot data synthetic.
// Standalone: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/glds_probe.hip \
//             -o tools/glds_probe && tools/glds_probe [size]
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#pragma clang fp contract(off)

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
constexpr int kWave = 64, kBlock = 256, kWaves = kBlock / kWave, kChunk = 2 * kWave;
constexpr int kMaxP = 8;
constexpr double kMinAbs = 0x1p-127, kMaxAbs = 0x1p130;

struct Piv {
    int r[kMaxP], c[kMaxP];
    double e[kMaxP], y[kMaxP];
};

// wait until at most n vector-memory operations of this wave are outstanding (gfx9 encoding:
// vmcnt[3:0], expcnt[6:4] = 7 and lgkmcnt[11:8] = 15 mean "do not wait on those")
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: __builtin_amdgcn_s_waitcnt(0xF70); break;
        case 1: __builtin_amdgcn_s_waitcnt(0xF71); break;
        case 2: __builtin_amdgcn_s_waitcnt(0xF72); break;
        case 3: __builtin_amdgcn_s_waitcnt(0xF73); break;
        case 4: __builtin_amdgcn_s_waitcnt(0xF74); break;
        case 5: __builtin_amdgcn_s_waitcnt(0xF75); break;
        case 6: __builtin_amdgcn_s_waitcnt(0xF76); break;
        case 7: __builtin_amdgcn_s_waitcnt(0xF77); break;
        case 8: __builtin_amdgcn_s_waitcnt(0xF78); break;
        case 9: __builtin_amdgcn_s_waitcnt(0xF79); break;
        case 10: __builtin_amdgcn_s_waitcnt(0xF7A); break;
        case 11: __builtin_amdgcn_s_waitcnt(0xF7B); break;
        case 12: __builtin_amdgcn_s_waitcnt(0xF7C); break;
        case 13: __builtin_amdgcn_s_waitcnt(0xF7D); break;
        case 14: __builtin_amdgcn_s_waitcnt(0xF7E); break;
        default: __builtin_amdgcn_s_waitcnt(0xF7F); break;
    }
}

template <int P>
__device__ __forceinline__ dbl2 steps_exact(dbl2 v, int row, int j, const Piv& pv, const dbl2* pr,
                                            const double* pc) {
#pragma unroll
    for (int l = 0; l < P; ++l) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int jj = j + h;
            double num;
            if (row == pv.r[l])
                num = (jj == pv.c[l]) ? 1.0 : -v[h];
            else
                num = (jj == pv.c[l]) ? v[h] : (v[h] * pv.e[l] - pr[l][h] * pc[l]);
            v[h] = num / pv.e[l];
        }
    }
    return v;
}

template <int P>
__device__ __forceinline__ dbl2 steps_fast(dbl2 x, int row, int j, bool cspecial, const Piv& pv,
                                           const dbl2* pr, const double* pc) {
    bool special = cspecial;
#pragma unroll
    for (int l = 0; l < P; ++l) special = special || row == pv.r[l];
    if (special) return steps_exact<P>(x, row, j, pv, pr, pc);
    dbl2 v = x;
    double mn = kMaxAbs, mx = 0.0;
#pragma unroll
    for (int l = 0; l < P; ++l) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const double num = v[h] * pv.e[l] - pr[l][h] * pc[l];
            mn = fmin(mn, fabs(num));
            mx = fmax(mx, fabs(num));
            const double t = num * pv.y[l];
            const double rr = fma(-pv.e[l], t, num);
            v[h] = fma(rr, pv.y[l], t);
        }
    }
    const bool in = mn >= kMinAbs && mx < kMaxAbs && v[0] == v[0] && v[1] == v[1];
    if (!__all(in)) v = steps_exact<P>(x, row, j, pv, pr, pc);
    return v;
}

// S-slot per-wave LDS ring fed by global_load_lds_dwordx4; one unit (row x 128 doubles) per
// iteration.  AUX: cache policy bits of the LDS-DMA load (0 default, 2 non-temporal).
template <int P, int S, int AUX>
__global__ __launch_bounds__(kBlock) void k_glds(const double* __restrict__ Tin, double* Tout,
                                                  int64_t ld, int R, int C,
                                                  const double* __restrict__ PR,
                                                  const double* __restrict__ M, Piv pv) {
    __shared__ dbl2 ring[kWaves][S][kWave];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NW = gridDim.x * kWaves;
    const int w = blockIdx.x * kWaves + wv;
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int64_t units = (int64_t)nchunks * R;
    const int64_t cnt = units > w ? (units - w + NW - 1) / NW : 0;   // this wave's units
    const int qs = NW / nchunks, rs = NW % nchunks;
    // unit t of this wave: (row, chunk) advanced incrementally, for issue (ahead) and compute
    int ri = w / nchunks, ci = w % nchunks;   // issue cursor
    int rc = ri;                              // compute cursor (row; the chunk is fixed)
    auto issue = [&](int64_t t) {
        const int j = ci * kChunk + 2 * lane;
        const int jj = j < C ? j : 0;         // padded lanes load a valid address (unused)
        const double* g = Tin + (int64_t)ri * ld + jj;
        __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)&ring[wv][t % S][0], 16, 0,
                                         AUX);
        ci += rs;
        ri += qs;
        if (ci >= nchunks) {
            ci -= nchunks;
            ++ri;
        }
    };
    // every wave keeps one chunk for the whole sweep (the launcher makes NW a multiple of
    // nchunks), so its pivot-row slices are loaded once, before any LDS-DMA is in flight: an
    // ordinary VGPR load inside the loop would make hipcc drain the ring with vmcnt(0)
    const int ch = w % nchunks;
    const int j = ch * kChunk + 2 * lane;
    dbl2 pr[P];
    bool cspecial = false;
#pragma unroll
    for (int l = 0; l < P; ++l) {
        pr[l] = (j < C) ? *reinterpret_cast<const dbl2*>(PR + (int64_t)l * ld + j)
                        : dbl2{0.0, 0.0};
        cspecial = cspecial || (pv.c[l] >= ch * kChunk && pv.c[l] < ch * kChunk + kChunk);
    }
    wait_vm(0);
    const int64_t pre = cnt < S - 1 ? cnt : S - 1;
    for (int64_t t = 0; t < pre; ++t) issue(t);
    for (int64_t t = 0; t < cnt; ++t) {
        if (t + S - 1 < cnt) issue(t + S - 1);
        // vector-memory ops issued after unit t's load (in-order vmcnt): the stores of the
        // iterations from the one that issued it up to t-1, and the loads of units after it
        const int64_t lt = t < S - 1 ? 0 : t - (S - 1);   // iteration that issued unit t's load
        int after = (int)(t - lt);
        after += (int)((t + S - 1 < cnt ? t + S - 1 : cnt - 1) - t);
        wait_vm(after);
        const int row = rc;
        rc += qs;   // rs == 0: the chunk never changes
        // the slot is read with an inline-asm ds_read: hipcc would otherwise put vmcnt(0) before
        // an LDS read that may alias a pending LDS-DMA, draining the whole ring every unit
        dbl2 x;
        {
            typedef __attribute__((address_space(3))) dbl2 lds_dbl2_t;
            const unsigned addr = (unsigned)(size_t)(lds_dbl2_t*)&ring[wv][t % S][lane];
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(addr)
                         : "memory");
        }
        double pc[P];
#pragma unroll
        for (int l = 0; l < P; ++l) pc[l] = M[(int64_t)row * kMaxP + l];
        const dbl2 v = steps_fast<P>(x, row, j, cspecial, pv, pr, pc);
        if (j < C)
            __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(Tout + (int64_t)row * ld + j));
    }
    wait_vm(0);
}

// reference: register loads, U units per batch (the form smx_block.hpp uses)
template <int P>
__global__ __launch_bounds__(kBlock) void k_reg(const double* __restrict__ Tin, double* Tout,
                                                 int64_t ld, int R, int C,
                                                 const double* __restrict__ PR,
                                                 const double* __restrict__ M, Piv pv) {
    const int lane = threadIdx.x & 63;
    const int NW = gridDim.x * kWaves;
    const int w = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int64_t units = (int64_t)nchunks * R;
    const int qs = NW / nchunks, rs = NW % nchunks;
    int i = w / nchunks, ch = w % nchunks;
    int ch_pr = -1;
    bool cspecial = false;
    dbl2 pr[P];
    constexpr int U = 2;
    for (int64_t u = w; u < units; u += (int64_t)U * NW) {
        int ii[U], cc[U];
        dbl2 x[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            ii[k] = i;
            cc[k] = ch;
            ch += rs;
            i += qs;
            if (ch >= nchunks) {
                ch -= nchunks;
                ++i;
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int j = cc[k] * kChunk + 2 * lane;
            x[k] = dbl2{0.0, 0.0};
            if (ii[k] < R && j < C)
                x[k] = __builtin_nontemporal_load(
                    reinterpret_cast<const dbl2*>(Tin + (int64_t)ii[k] * ld + j));
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int row = ii[k];
            if (row >= R) continue;
            const int j = cc[k] * kChunk + 2 * lane;
            if (cc[k] != ch_pr) {
                ch_pr = cc[k];
                cspecial = false;
                const int c0 = cc[k] * kChunk;
#pragma unroll
                for (int l = 0; l < P; ++l) {
                    pr[l] = (j < C) ? *reinterpret_cast<const dbl2*>(PR + (int64_t)l * ld + j)
                                    : dbl2{0.0, 0.0};
                    cspecial = cspecial || (pv.c[l] >= c0 && pv.c[l] < c0 + kChunk);
                }
            }
            double pc[P];
#pragma unroll
            for (int l = 0; l < P; ++l) pc[l] = M[(int64_t)row * kMaxP + l];
            const dbl2 v = steps_fast<P>(x[k], row, j, cspecial, pv, pr, pc);
            if (j < C)
                __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(Tout + (int64_t)row * ld + j));
        }
    }
}

// U = 2 units computed together: one branch for "neither is special", their four element chains
// interleaved in one unrolled loop (ILP 4 per wave instead of 2), one vote for both
template <int P>
__global__ __launch_bounds__(kBlock) void k_reg2(const double* __restrict__ Tin, double* Tout,
                                                  int64_t ld, int R, int C,
                                                  const double* __restrict__ PR,
                                                  const double* __restrict__ M, Piv pv) {
    const int lane = threadIdx.x & 63;
    const int NW = gridDim.x * kWaves;
    const int w = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int64_t units = (int64_t)nchunks * R;
    const int qs = NW / nchunks;
    // fixed chunk per wave (NW a multiple of nchunks)
    const int ch = w % nchunks;
    const int j = ch * kChunk + 2 * lane;
    dbl2 pr[P];
    bool cspecial = false;
#pragma unroll
    for (int l = 0; l < P; ++l) {
        pr[l] = (j < C) ? *reinterpret_cast<const dbl2*>(PR + (int64_t)l * ld + j) : dbl2{0.0, 0.0};
        cspecial = cspecial || (pv.c[l] >= ch * kChunk && pv.c[l] < ch * kChunk + kChunk);
    }
    int i = w / nchunks;
    for (int64_t u = w; u < units; u += 2 * (int64_t)NW) {
        const int i0 = i, i1 = i + qs;
        i += 2 * qs;
        const bool h1 = i1 < R;
        dbl2 x0 = dbl2{0.0, 0.0}, x1 = dbl2{0.0, 0.0};
        if (j < C) {
            x0 = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(Tin + (int64_t)i0 * ld + j));
            if (h1)
                x1 = __builtin_nontemporal_load(
                    reinterpret_cast<const dbl2*>(Tin + (int64_t)i1 * ld + j));
        }
        double pc0[P], pc1[P];
        bool special = cspecial || !h1;
#pragma unroll
        for (int l = 0; l < P; ++l) {
            pc0[l] = M[(int64_t)i0 * kMaxP + l];
            pc1[l] = h1 ? M[(int64_t)i1 * kMaxP + l] : 0.0;
            special = special || i0 == pv.r[l] || i1 == pv.r[l];
        }
        dbl2 v0 = x0, v1 = x1;
        bool ok = false;
        if (!special) {
            double mn = kMaxAbs, mx = 0.0;
#pragma unroll
            for (int l = 0; l < P; ++l) {
                const double e = pv.e[l], y = pv.y[l];
                double n[4];
                n[0] = v0[0] * e - pr[l][0] * pc0[l];
                n[1] = v0[1] * e - pr[l][1] * pc0[l];
                n[2] = v1[0] * e - pr[l][0] * pc1[l];
                n[3] = v1[1] * e - pr[l][1] * pc1[l];
                double r[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    mn = fmin(mn, fabs(n[q]));
                    mx = fmax(mx, fabs(n[q]));
                    const double t = n[q] * y;
                    const double rr = fma(-e, t, n[q]);
                    r[q] = fma(rr, y, t);
                }
                v0 = dbl2{r[0], r[1]};
                v1 = dbl2{r[2], r[3]};
            }
            ok = __all(mn >= kMinAbs && mx < kMaxAbs && v0[0] == v0[0] && v0[1] == v0[1] &&
                       v1[0] == v1[0] && v1[1] == v1[1]);
        }
        if (!ok) {
            v0 = steps_exact<P>(x0, i0, j, pv, pr, pc0);
            if (h1) v1 = steps_exact<P>(x1, i1, j, pv, pr, pc1);
        }
        if (j < C) {
            __builtin_nontemporal_store(v0, reinterpret_cast<dbl2*>(Tout + (int64_t)i0 * ld + j));
            if (h1)
                __builtin_nontemporal_store(v1, reinterpret_cast<dbl2*>(Tout + (int64_t)i1 * ld + j));
        }
    }
}

__global__ void k_fill(double* a, int64_t n, unsigned long long seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        a[i] = ((double)(z >> 11) / 9007199254740992.0) * 2.0 - 1.0;
    }
}

template <typename K>
float timeit(K kern, int grid, const double* a, double* b, int64_t ld, int R, int C,
             const double* PR, const double* M, const Piv& pv, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int t = 0; t < reps; ++t)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <typename K>
void row(const char* name, int P, K kern, int cus, const double* a, double* b, int64_t ld, int R,
         int C, const double* PR, const double* M, const Piv& pv, int reps) {
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void*)kern));
    for (int bpc : {4, 5, 6, 8}) {
        const float t = timeit(kern, cus * bpc, a, b, ld, R, C, PR, M, pv, reps);
        printf("{\"size\": %d, \"kernel\": \"%s\", \"P\": %d, \"bpc\": %d, \"us\": %.1f, "
               "\"gbs\": %.0f, \"vgpr\": %d, \"lds\": %d}\n",
               R, name, P, bpc, t * 1e3, 16.0 * R * C / t / 1e6, fa.numRegs,
               (int)fa.sharedSizeBytes);
        fflush(stdout);
    }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int R = N, C = N;
    const int64_t ld = C;
    double *a, *b, *PR, *M, *chk;
    CK(hipMalloc(&a, (size_t)R * ld * 8));
    CK(hipMalloc(&b, (size_t)R * ld * 8));
    CK(hipMalloc(&chk, (size_t)R * ld * 8));
    CK(hipMalloc(&PR, (size_t)kMaxP * ld * 8));
    CK(hipMalloc(&M, (size_t)R * kMaxP * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, (int64_t)R * ld, 1ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, PR, (int64_t)kMaxP * ld, 2ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, M, (int64_t)R * kMaxP, 3ull);
    CK(hipDeviceSynchronize());
    Piv pv;
    for (int l = 0; l < kMaxP; ++l) {
        pv.r[l] = (l * 977 + 5) % R;
        pv.c[l] = (l * 1231 + 7) % C;
        pv.e[l] = 0.75 + 0.125 * l;
        pv.y[l] = 1.0 / pv.e[l];   // not fd_prep's value: both kernels use the same y here
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = N >= 16384 ? 8 : 30;
    // correctness: the glds kernel must write exactly what the register kernel writes
    hipLaunchKernelGGL((k_reg<8>), dim3(cus * 5), dim3(kBlock), 0, 0, a, chk, ld, R, C, PR, M, pv);
    hipLaunchKernelGGL((k_glds<8, 3, 0>), dim3(cus * 5), dim3(kBlock), 0, 0, a, b, ld, R, C, PR,
                       M, pv);
    CK(hipDeviceSynchronize());
    {
        const size_t nb = (size_t)R * ld * 8;
        double* h1 = (double*)malloc(nb);
        double* h2 = (double*)malloc(nb);
        CK(hipMemcpy(h1, chk, nb, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2, b, nb, hipMemcpyDeviceToHost));
        long bad = 0;
        for (long q = 0; q < (long)R * ld; ++q)
            if (__builtin_memcmp(&h1[q], &h2[q], 8) != 0) ++bad;
        printf("{\"check\": \"glds vs reg\", \"mismatches\": %ld}\n", bad);
        fflush(stdout);
        free(h1);
        free(h2);
    }
    hipLaunchKernelGGL((k_reg2<8>), dim3(cus * 5), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
    CK(hipDeviceSynchronize());
    {
        const size_t nb = (size_t)R * ld * 8;
        double* h1 = (double*)malloc(nb);
        double* h2 = (double*)malloc(nb);
        CK(hipMemcpy(h1, chk, nb, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2, b, nb, hipMemcpyDeviceToHost));
        long bad = 0;
        for (long q = 0; q < (long)R * ld; ++q)
            if (__builtin_memcmp(&h1[q], &h2[q], 8) != 0) ++bad;
        printf("{\"check\": \"reg2 vs reg\", \"mismatches\": %ld}\n", bad);
        fflush(stdout);
        free(h1);
        free(h2);
    }
    row("reg", 8, k_reg<8>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("reg2", 8, k_reg2<8>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("reg2", 6, k_reg2<6>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("reg2", 4, k_reg2<4>, cus, a, b, ld, R, C, PR, M, pv, reps);
    return 0;
    row("glds_s3", 8, k_glds<8, 3, 0>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("glds_s4", 8, k_glds<8, 4, 0>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("glds_s3_nt", 8, k_glds<8, 3, 2>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("glds_s6", 8, k_glds<8, 6, 0>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("reg", 4, k_reg<4>, cus, a, b, ld, R, C, PR, M, pv, reps);
    row("glds_s4", 4, k_glds<4, 4, 0>, cus, a, b, ld, R, C, PR, M, pv, reps);
    return 0;
}
