// sweep_lab2.hip -- lab for the block sweep at LARGE pivot counts (P = 10..24): where the pivot
// elements, reciprocals and pivot-row slices live once they no longer fit in registers beside the
// row's multipliers.  Fast path only (a bounded table: every unit takes the unchecked
// hoisted-reciprocal sequence, which is bit-identical to the IEEE division there, smx_block.hpp
// kBndSpan), so each variant's output is checked bit for bit against V0 (the IEEE division).
//
//   V0 ieee     reference: x = (x e - p mq) / e with the hardware division sequence
//   V1 prod     the production flag form's shape: pivot-row slices in VGPRs, e / y hoisted into
//               scalar registers, the 2P products first, multipliers per row as scalar loads
//   V2 eylds    V1's slices in VGPRs; (e, y) pairs read from LDS per pivot; products inline
//   V3 alllds   slices in LDS shared by the workgroup's four waves (one chunk per workgroup),
//               (e, y) from LDS; products inline
//   V4 alllds2  V3 with two rows in flight while one is computed
//   V5 prlds    slices in LDS, e / y left to the compiler (hoisted scalars)
//   V6 ey4      V3 with (e, y) of four pivots read as one 64-B LDS broadcast
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/sweep_lab2.hip \
//          -o tools/sweep_lab2
// Run:   tools/sweep_lab2 [N=16384] [P=16] [reps=5] [bpc=5] [variants=0123456]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang fp contract(off)

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

namespace {

constexpr int kWave = 64;
constexpr int kBlk = 256;
constexpr int kWaves = kBlk / kWave;
constexpr int kMaxP = 32;
typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double fd_recip(double e) {
    const double y0 = __builtin_amdgcn_rcp(e);
    const double t0 = fma(-e, y0, 1.0);
    const double y1 = fma(y0, t0, y0);
    const double t1 = fma(-e, y1, 1.0);
    return fma(y1, t1, y1);
}

__global__ void k_fill(double* p, int64_t n, unsigned long long seed, double lo, double hi) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        unsigned long long z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed * 0xD1B54A32D192ED03ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = lo + (hi - lo) * (double)(z >> 11) * 0x1p-53;
    }
}

// (e, y) pairs: e alternating in sign, |e| in [0.6, 3.8]
__global__ void k_hdr(dbl2* ey) {
    const int q = threadIdx.x;
    if (q >= kMaxP) return;
    const double e = (q & 1 ? -1.0 : 1.0) * (0.6 + 0.1 * q);
    ey[q] = dbl2{e, fd_recip(e)};
}

__global__ void k_cmp(const double* a, const double* b, int64_t n, unsigned long long* bad) {
    unsigned long long k = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * blockDim.x)
        k += __double_as_longlong(a[t]) != __double_as_longlong(b[t]);
    if (k) atomicAdd(bad, k);
}

__device__ __forceinline__ dbl2 ldnt(const double* p) {
    dbl2 v;
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    return v;
}

__device__ __forceinline__ double fdq(double n, double e, double y) {
    const double t = n * y;
    const double r = fma(-e, t, n);
    return fma(r, y, t);
}

template <int P, int V>
__global__ __launch_bounds__(kBlk) void k_sweep(double* T, int64_t ld, int R, int C,
                                                const dbl2* __restrict__ eyg,
                                                const double* __restrict__ pr,
                                                const double* __restrict__ mul) {
    constexpr bool PRLDS = V == 3 || V == 4 || V == 5 || V == 6;
    constexpr bool EYLDS = V == 2 || V == 3 || V == 4 || V == 6;
    constexpr int DEPTH = V == 4 ? 2 : 1;
    __shared__ dbl2 s_pr[PRLDS ? P : 1][kWave];
    __shared__ dbl2 s_ey[P];
    const int lane = threadIdx.x & (kWave - 1);
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int kChunk = 2 * kWave;
    const int nchunks = (C + kChunk - 1) / kChunk;
    int ch, base, qs;
    if (PRLDS) {   // one chunk per workgroup, its four waves on interleaved rows
        ch = blockIdx.x % nchunks;
        base = (blockIdx.x / nchunks) * kWaves + wib;
        qs = (gridDim.x / nchunks) * kWaves;
    } else {
        const int NW = gridDim.x * kWaves;
        const int w = blockIdx.x * kWaves + wib;
        ch = w % nchunks;
        base = w / nchunks;
        qs = NW / nchunks;
    }
    const int j = ch * kChunk + 2 * lane;
    dbl2 prs[PRLDS ? 1 : P];
    double eq[EYLDS ? 1 : P], yq[EYLDS ? 1 : P];
    if (threadIdx.x < P) s_ey[threadIdx.x] = eyg[threadIdx.x];
    if (PRLDS) {
        for (int t = threadIdx.x; t < P * kWave; t += kBlk) {
            const int q = t / kWave, l = t % kWave;
            s_pr[q][l] = *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + ch * kChunk + 2 * l);
        }
    } else {
#pragma unroll
        for (int q = 0; q < P; ++q) prs[q] = *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j);
    }
    if (!EYLDS) {
#pragma unroll
        for (int q = 0; q < P; ++q) {
            eq[q] = eyg[q][0];
            yq[q] = eyg[q][1];
        }
    }
    __syncthreads();
    auto row = [&](dbl2 x0, int i0) {
        const double* m0 = mul + (int64_t)i0 * kMaxP;
        double pc[P];
#pragma unroll
        for (int q = 0; q < P; ++q) pc[q] = m0[q];
        dbl2 v = x0;
        if (V == 0) {
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const dbl2 p = PRLDS ? s_pr[q][lane] : prs[q];
                const double e = s_ey[q][0];
#pragma unroll
                for (int k = 0; k < 2; ++k) v[k] = (v[k] * e - p[k] * pc[q]) / e;
            }
        } else if (V == 1) {
            dbl2 bq[P];
#pragma unroll
            for (int q = 0; q < P; ++q) bq[q] = dbl2{prs[q][0] * pc[q], prs[q][1] * pc[q]};
#pragma unroll
            for (int q = 0; q < P; ++q) asm volatile("" : "+v"(bq[q]));
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                v = dbl2{fdq(v[0] * e - bq[q][0], e, y), fdq(v[1] * e - bq[q][1], e, y)};
            }
        } else if (V == 6) {
#pragma unroll
            for (int q0 = 0; q0 < P; q0 += 2) {
                dbl2 eyv[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) eyv[u] = q0 + u < P ? s_ey[q0 + u] : dbl2{1.0, 1.0};
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int q = q0 + u;
                    if (q < P) {
                        const dbl2 p = s_pr[q][lane];
                        const double e = eyv[u][0], y = eyv[u][1];
                        v = dbl2{fdq(v[0] * e - p[0] * pc[q], e, y),
                                 fdq(v[1] * e - p[1] * pc[q], e, y)};
                    }
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const dbl2 p = PRLDS ? s_pr[q][lane] : prs[q];
                double e, y;
                if (EYLDS) {
                    const dbl2 ey = s_ey[q];
                    e = ey[0];
                    y = ey[1];
                } else {
                    e = eq[q];
                    y = yq[q];
                }
                v = dbl2{fdq(v[0] * e - p[0] * pc[q], e, y), fdq(v[1] * e - p[1] * pc[q], e, y)};
            }
        }
        if (j < C) __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(T + (int64_t)i0 * ld + j));
    };
    const int jc = min(j, (C - 1) & ~1);
    auto ldc = [&](int r) { return ldnt(T + (int64_t)min(r, R - 1) * ld + jc); };
    if (base >= R) return;
    if (DEPTH == 1) {
        dbl2 a = ldc(base), b = ldc(base + qs);
        asm volatile("s_waitcnt vmcnt(1)" : "+v"(a)::"memory");
        for (int i0 = base; i0 < R; i0 += 2 * qs) {
            row(a, i0);
            if (i0 + qs >= R) break;
            a = ldc(i0 + 2 * qs);
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(b)::"memory");
            row(b, i0 + qs);
            if (i0 + 2 * qs >= R) break;
            b = ldc(i0 + 3 * qs);
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(a)::"memory");
        }
    } else {
        dbl2 a = ldc(base), b = ldc(base + qs), c = ldc(base + 2 * qs);
        asm volatile("s_waitcnt vmcnt(2)" : "+v"(a)::"memory");
        int i0 = base;
        bool first = true;
        for (;; i0 += 3 * qs) {
            row(a, i0);
            if (i0 + qs >= R) break;
            a = ldc(i0 + 3 * qs);
            if (first)
                asm volatile("s_waitcnt vmcnt(3)" : "+v"(b)::"memory");
            else
                asm volatile("s_waitcnt vmcnt(4)" : "+v"(b)::"memory");
            first = false;
            row(b, i0 + qs);
            if (i0 + 2 * qs >= R) break;
            b = ldc(i0 + 4 * qs);
            asm volatile("s_waitcnt vmcnt(4)" : "+v"(c)::"memory");
            row(c, i0 + 2 * qs);
            if (i0 + 3 * qs >= R) break;
            c = ldc(i0 + 5 * qs);
            asm volatile("s_waitcnt vmcnt(4)" : "+v"(a)::"memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

using Fn = void (*)(double*, int64_t, int, int, const dbl2*, const double*, const double*);

template <int P>
Fn pick(int v) {
    switch (v) {
        case 0: return k_sweep<P, 0>;
        case 1: return k_sweep<P, 1>;
        case 2: return k_sweep<P, 2>;
        case 3: return k_sweep<P, 3>;
        case 4: return k_sweep<P, 4>;
        case 5: return k_sweep<P, 5>;
        default: return k_sweep<P, 6>;
    }
}
Fn pickP(int P, int v) {
    switch (P) {
        case 10: return pick<10>(v);
        case 12: return pick<12>(v);
        case 14: return pick<14>(v);
        case 16: return pick<16>(v);
        case 20: return pick<20>(v);
        case 24: return pick<24>(v);
        default: return nullptr;
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int P = argc > 2 ? atoi(argv[2]) : 16;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int bpc = argc > 4 ? atoi(argv[4]) : 5;
    const char* only = argc > 5 ? argv[5] : "0123456";
    if (!pickP(P, 0)) {
        fprintf(stderr, "P must be one of 10 12 14 16 20 24\n");
        return 2;
    }
    const int R = N, C = N;
    const int64_t ld = C;
    const int64_t nel = (int64_t)R * ld;
    double *T0, *T, *ref, *pr, *mul;
    dbl2* ey;
    unsigned long long* bad;
    CK(hipMalloc(&T0, nel * 8));
    CK(hipMalloc(&T, nel * 8));
    CK(hipMalloc(&ref, nel * 8));
    CK(hipMalloc(&pr, (int64_t)kMaxP * ld * 8));
    CK(hipMalloc(&mul, (int64_t)R * kMaxP * 8));
    CK(hipMalloc(&ey, kMaxP * sizeof(dbl2)));
    CK(hipMalloc(&bad, 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, T0, nel, 1ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, pr, (int64_t)kMaxP * ld, 2ull, 0.25, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, mul, (int64_t)R * kMaxP, 3ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_hdr, dim3(1), dim3(64), 0, 0, ey);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nchunks = (C + 127) / 128;
    int grid = cus * bpc;
    grid -= grid % nchunks;   // every variant: a multiple of the chunks (waves and workgroups)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 16.0 * R * C;
    bool have_ref = false;
    for (const char* o = only; *o; ++o) {
        const int v = *o - '0';
        Fn fn = pickP(P, v);
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, (const void*)fn));
        std::vector<float> ms;
        unsigned long long nbad = 0;
        for (int r = 0; r < reps + 1; ++r) {
            CK(hipMemcpy(T, T0, nel * 8, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlk), 0, 0, T, ld, R, C, ey, pr, mul);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r > 0) ms.push_back(t);
        }
        if (v == 0) {
            CK(hipMemcpy(ref, T, nel * 8, hipMemcpyDeviceToDevice));
            have_ref = true;
        } else if (have_ref) {
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, ref, T, nel, bad);
            CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
        }
        std::sort(ms.begin(), ms.end());
        printf("{\"N\": %d, \"P\": %d, \"variant\": %d, \"grid\": %d, \"bpc\": %d, \"vgprs\": %d, "
               "\"best_us\": %.1f, \"median_us\": %.1f, \"us_per_pivot\": %.2f, \"tbs\": %.3f, "
               "\"checked\": %s, \"mismatch\": %llu}\n",
               N, P, v, grid, bpc, fa.numRegs, ms[0] * 1e3, ms[ms.size() / 2] * 1e3,
               ms[0] * 1e3 / P, bytes / (ms[0] * 1e-3) / 1e12, have_ref && v ? "true" : "false",
               nbad);
        fflush(stdout);
    }
    return 0;
}
