// multipivot_probe.hip -- how many Jordan steps can one HBM sweep of the tableau apply before the
// fp64 arithmetic, not the stream, sets the time?  Applies P consecutive pivots per element
// (pivot rows and per-row multipliers given, as a block sweep would have them from its planner)
// with the reference's per-element expression (simplex.py:166-175: (x*e - pr*pc)/e per step),
// either the compiler's IEEE division or the hoisted-reciprocal form of smx_resident.hpp, in
// place or out of place, and prints us per sweep and the effective pivots/s.
// Standalone: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/multipivot_probe.hip \
//             -o tools/multipivot_probe && tools/multipivot_probe [size]
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
constexpr int kWave = 64, kBlock = 256, kWaves = kBlock / kWave, kChunk = 2 * kWave;
constexpr int kMaxP = 8;

struct Piv {
    int r[kMaxP], c[kMaxP];
    double e[kMaxP], y[kMaxP];
};

__device__ __forceinline__ bool fd_in(double x) {
    const unsigned bexp = ((unsigned)(__double_as_longlong(x) >> 52)) & 0x7ffu;
    return bexp - 896u <= 1152u - 896u;
}

template <bool FD>
__device__ __forceinline__ double dv(double x, double e, double y) {
    if (FD && fd_in(x) && fd_in(e)) {
        const double q = x * y;
        const double r = fma(-e, q, x);
        return fma(r, y, q);
    }
    return x / e;
}

template <int P, bool FD>
__global__ __launch_bounds__(kBlock) void k_multi(const double* __restrict__ Tin,
                                                   double* Tout, int64_t ld, int R, int C,
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
#pragma unroll
                for (int l = 0; l < P; ++l)
                    pr[l] = (j < C) ? *reinterpret_cast<const dbl2*>(PR + (int64_t)l * ld + j)
                                    : dbl2{0.0, 0.0};
            }
            double pc[P];
#pragma unroll
            for (int l = 0; l < P; ++l) pc[l] = M[(int64_t)row * kMaxP + l];
            dbl2 v = x[k];
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
                    v[h] = dv<FD>(num, pv.e[l], pv.y[l]);
                }
            }
            if (j < C)
                __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(Tout + (int64_t)row * ld + j));
        }
    }
}

// Variant 2 (the form smx_block.hpp uses): the pivot-row test hoisted to one scalar branch
// per unit, the pivot-column select only in the chunk that holds the column, and the division
// window checked by accumulating a lane mask over all P steps with ONE wave vote per unit; a
// unit whose vote fails is recomputed with the per-element exact path.
template <int P>
__device__ __forceinline__ dbl2 chain_exact(dbl2 v, int row, int j, const Piv& pv,
                                            const dbl2* pr, const double* pc) {
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
            v[h] = dv<true>(num, pv.e[l], pv.y[l]);
        }
    }
    return v;
}

template <int P, bool FD>
__global__ __launch_bounds__(kBlock) void k_multi2(const double* __restrict__ Tin,
                                                    double* Tout, int64_t ld, int R, int C,
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
    dbl2 pr[P];
    unsigned cmask = 0;   // bit l: this chunk holds column c_l (wave-uniform)
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
                cmask = 0;
#pragma unroll
                for (int l = 0; l < P; ++l) {
                    pr[l] = (j < C) ? *reinterpret_cast<const dbl2*>(PR + (int64_t)l * ld + j)
                                    : dbl2{0.0, 0.0};
                    const int c0 = cc[k] * kChunk;
                    if (pv.c[l] >= c0 && pv.c[l] < c0 + kChunk) cmask |= 1u << l;
                }
            }
            double pc[P];
#pragma unroll
            for (int l = 0; l < P; ++l) pc[l] = M[(int64_t)row * kMaxP + l];
            bool special = cmask != 0;
#pragma unroll
            for (int l = 0; l < P; ++l) special |= row == pv.r[l];
            dbl2 v = x[k];
            if (!special) {
                int bad = 0;
#pragma unroll
                for (int l = 0; l < P; ++l) {
                    const double e = pv.e[l], y = pv.y[l];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const double num = v[h] * e - pr[l][h] * pc[l];
                        bad |= !fd_in(num);
                        if (FD) {
                            const double t = num * y;
                            const double rr = fma(-e, t, num);
                            v[h] = fma(rr, y, t);
                        } else {
                            v[h] = num / e;
                        }
                    }
                }
                if (FD && !__all(!bad)) v = chain_exact<P>(x[k], row, j, pv, pr, pc);
            } else {
                v = chain_exact<P>(v, row, j, pv, pr, pc);
            }
            if (j < C)
                __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(Tout + (int64_t)row * ld + j));
        }
    }
}

// Variant 3 (smx_block.hpp's sweep): fast path with the smallest / largest |numerator| tracked
// per lane and one wave vote per unit; PF: the next batch's loads issued before the arithmetic.
constexpr double kMinAbs = 0x1p-127, kMaxAbs = 0x1p130;
template <int P, bool PF>
__global__ __launch_bounds__(kBlock) void k_multi3(const double* __restrict__ Tin,
                                                    double* Tout, int64_t ld, int R, int C,
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
    bool cspecial = true;
    dbl2 pr[P];
    constexpr int U = 2;
    struct Bt {
        int ii[U], cc[U];
        dbl2 x[U];
    };
    auto fetch = [&](Bt& bt) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            bt.ii[k] = i;
            bt.cc[k] = ch;
            ch += rs;
            i += qs;
            if (ch >= nchunks) {
                ch -= nchunks;
                ++i;
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int j = bt.cc[k] * kChunk + 2 * lane;
            bt.x[k] = dbl2{0.0, 0.0};
            if (bt.ii[k] < R && j < C)
                bt.x[k] = __builtin_nontemporal_load(
                    reinterpret_cast<const dbl2*>(Tin + (int64_t)bt.ii[k] * ld + j));
        }
    };
    Bt cur;
    if (PF && w < units) fetch(cur);
    for (int64_t u = w; u < units; u += (int64_t)U * NW) {
        Bt nxt;
        if (PF) {
            if (u + (int64_t)U * NW < units) fetch(nxt);
        } else {
            fetch(cur);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int row = cur.ii[k];
            if (row >= R) continue;
            const int j = cur.cc[k] * kChunk + 2 * lane;
            if (cur.cc[k] != ch_pr) {
                ch_pr = cur.cc[k];
                cspecial = false;
                const int c0 = cur.cc[k] * kChunk;
#pragma unroll
                for (int l = 0; l < P; ++l) {
                    pr[l] = (j < C) ? *reinterpret_cast<const dbl2*>(PR + (int64_t)l * ld + j)
                                    : dbl2{0.0, 0.0};
                    cspecial = cspecial || (pv.c[l] >= c0 && pv.c[l] < c0 + kChunk);
                }
            }
            double pc[P];
            bool special = cspecial;
#pragma unroll
            for (int l = 0; l < P; ++l) {
                pc[l] = M[(int64_t)row * kMaxP + l];
                special = special || row == pv.r[l];
            }
            dbl2 v = cur.x[k];
            if (!special) {
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
                if (!__all(in)) v = chain_exact<P>(cur.x[k], row, j, pv, pr, pc);
            } else {
                v = chain_exact<P>(v, row, j, pv, pr, pc);
            }
            if (j < C)
                __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(Tout + (int64_t)row * ld + j));
        }
        if (PF) cur = nxt;
    }
}

template <int P, bool PF>
float run3(const double* a, double* b, int64_t ld, int R, int C, const double* PR, const double* M,
           const Piv& pv, int grid, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_multi3<P, PF>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
    CK(hipEventRecord(e0));
    for (int t = 0; t < reps; ++t)
        hipLaunchKernelGGL((k_multi3<P, PF>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR,
                           M, pv);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <int P>
void row3(int R, const double* a, double* b, int64_t ld, int C, const double* PR, const double* M,
          const Piv& pv, int cus, int reps) {
    hipFuncAttributes fa0, fa1;
    CK(hipFuncGetAttributes(&fa0, (const void*)k_multi3<P, false>));
    CK(hipFuncGetAttributes(&fa1, (const void*)k_multi3<P, true>));
    for (int bpc : {4, 5, 6, 8}) {
        const float t0 = run3<P, false>(a, b, ld, R, C, PR, M, pv, cus * bpc, reps);
        const float t1 = run3<P, true>(a, b, ld, R, C, PR, M, pv, cus * bpc, reps);
        printf("{\"size\": %d, \"P\": %d, \"bpc\": %d, \"v3_us\": %.1f, \"v3_pf_us\": %.1f, "
               "\"vgpr\": %d, \"vgpr_pf\": %d}\n", R, P, bpc, t0 * 1e3, t1 * 1e3, fa0.numRegs,
               fa1.numRegs);
        fflush(stdout);
    }
}

// Variant 4: one double per lane (64-double = 512-B chunks), U units in flight; halves the
// pivot-row registers (P doubles per lane instead of 2P) so more waves fit per SIMD.
template <int P>
__device__ __forceinline__ double chain_exact1(double v, int row, int j, const Piv& pv,
                                               const double* pr, const double* pc) {
#pragma unroll
    for (int l = 0; l < P; ++l) {
        double num;
        if (row == pv.r[l])
            num = (j == pv.c[l]) ? 1.0 : -v;
        else
            num = (j == pv.c[l]) ? v : (v * pv.e[l] - pr[l] * pc[l]);
        v = num / pv.e[l];
    }
    return v;
}

template <int P, int U>
__global__ __launch_bounds__(kBlock) void k_multi4(const double* __restrict__ Tin,
                                                    double* Tout, int64_t ld, int R, int C,
                                                    const double* __restrict__ PR,
                                                    const double* __restrict__ M, Piv pv) {
    constexpr int kCh = kWave;
    const int lane = threadIdx.x & 63;
    const int NW = gridDim.x * kWaves;
    const int w = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nchunks = (C + kCh - 1) / kCh;
    const int64_t units = (int64_t)nchunks * R;
    const int qs = NW / nchunks, rs = NW % nchunks;
    int i = w / nchunks, ch = w % nchunks;
    int ch_pr = -1;
    bool cspecial = true;
    double pr[P];
    for (int64_t u = w; u < units; u += (int64_t)U * NW) {
        int ii[U], cc[U];
        double x[U];
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
            const int j = cc[k] * kCh + lane;
            x[k] = 0.0;
            if (ii[k] < R && j < C) x[k] = __builtin_nontemporal_load(Tin + (int64_t)ii[k] * ld + j);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int row = ii[k];
            if (row >= R) continue;
            const int j = cc[k] * kCh + lane;
            if (cc[k] != ch_pr) {
                ch_pr = cc[k];
                cspecial = false;
                const int c0 = cc[k] * kCh;
#pragma unroll
                for (int l = 0; l < P; ++l) {
                    pr[l] = (j < C) ? PR[(int64_t)l * ld + j] : 0.0;
                    cspecial = cspecial || (pv.c[l] >= c0 && pv.c[l] < c0 + kCh);
                }
            }
            double pc[P];
            bool special = cspecial;
#pragma unroll
            for (int l = 0; l < P; ++l) {
                pc[l] = M[(int64_t)row * kMaxP + l];
                special = special || row == pv.r[l];
            }
            double v = x[k];
            if (!special) {
                double mn = kMaxAbs, mx = 0.0;
#pragma unroll
                for (int l = 0; l < P; ++l) {
                    const double num = v * pv.e[l] - pr[l] * pc[l];
                    mn = fmin(mn, fabs(num));
                    mx = fmax(mx, fabs(num));
                    const double t = num * pv.y[l];
                    const double rr = fma(-pv.e[l], t, num);
                    v = fma(rr, pv.y[l], t);
                }
                const bool in = mn >= kMinAbs && mx < kMaxAbs && v == v;
                if (!__all(in)) v = chain_exact1<P>(x[k], row, j, pv, pr, pc);
            } else {
                v = chain_exact1<P>(v, row, j, pv, pr, pc);
            }
            if (j < C) __builtin_nontemporal_store(v, Tout + (int64_t)row * ld + j);
        }
    }
}

template <int P, int U>
void row4(int R, const double* a, double* b, int64_t ld, int C, const double* PR, const double* M,
          const Piv& pv, int cus, int reps) {
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void*)k_multi4<P, U>));
    for (int bpc : {5, 6, 8}) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int grid = cus * bpc;
        hipLaunchKernelGGL((k_multi4<P, U>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
        CK(hipEventRecord(e0));
        for (int t = 0; t < reps; ++t)
            hipLaunchKernelGGL((k_multi4<P, U>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR,
                               M, pv);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"size\": %d, \"P\": %d, \"U\": %d, \"bpc\": %d, \"v4_us\": %.1f, \"vgpr\": %d}\n",
               R, P, U, bpc, ms / reps * 1e3, fa.numRegs);
        fflush(stdout);
    }
}

template <int P>
float run2(const double* a, double* b, int64_t ld, int R, int C, const double* PR, const double* M,
           const Piv& pv, int grid, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_multi2<P, true>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
    CK(hipEventRecord(e0));
    for (int t = 0; t < reps; ++t)
        hipLaunchKernelGGL((k_multi2<P, true>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR,
                           M, pv);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <int P, bool FD>
float run(const double* a, double* b, int64_t ld, int R, int C, const double* PR, const double* M,
          const Piv& pv, int grid, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_multi<P, FD>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M, pv);
    CK(hipEventRecord(e0));
    for (int t = 0; t < reps; ++t)
        hipLaunchKernelGGL((k_multi<P, FD>), dim3(grid), dim3(kBlock), 0, 0, a, b, ld, R, C, PR, M,
                           pv);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

__global__ void k_fill(double* a, int64_t n, unsigned long long seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        a[i] = ((double)(z >> 11) / 9007199254740992.0) * 2.0 - 1.0;
    }
}

template <int P>
void row(const char* label, const double* a, double* b, int64_t ld, int R, int C, const double* PR,
         const double* M, const Piv& pv, int grid, int reps) {
    const double bytes = 16.0 * R * C;
    const float t0 = run<P, false>(a, b, ld, R, C, PR, M, pv, grid, reps);
    const float t1 = run<P, true>(a, b, ld, R, C, PR, M, pv, grid, reps);
    const float t2 = run2<P>(a, b, ld, R, C, PR, M, pv, grid, reps);
    printf("{\"size\": %d, \"P\": %d, \"mode\": \"%s\", \"ieee_us\": %.1f, \"fastdiv_us\": %.1f, "
           "\"v2_us\": %.1f, \"ieee_gbs\": %.0f, \"fastdiv_gbs\": %.0f, \"v2_gbs\": %.0f, "
           "\"ieee_pivots_s\": %.0f, \"fastdiv_pivots_s\": %.0f, \"v2_pivots_s\": %.0f}\n",
           R, P, label, t0 * 1e3, t1 * 1e3, t2 * 1e3, bytes / t0 / 1e6, bytes / t1 / 1e6,
           bytes / t2 / 1e6, P * 1e3 / t0, P * 1e3 / t1, P * 1e3 / t2);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int R = N, C = N;
    const int64_t ld = C;
    double *a, *b, *PR, *M;
    CK(hipMalloc(&a, (size_t)R * ld * 8));
    CK(hipMalloc(&b, (size_t)R * ld * 8));
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
        pv.y[l] = 1.0 / pv.e[l];
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = N >= 16384 ? 10 : 40;
    if (argc > 2 && argv[2][0] == '4') {
        row4<4, 4>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row4<6, 4>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row4<8, 4>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row4<8, 2>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row4<8, 8>(R, a, b, ld, C, PR, M, pv, cus, reps);
        return 0;
    }
    if (argc > 2 && argv[2][0] == '3') {
        row3<2>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row3<4>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row3<6>(R, a, b, ld, C, PR, M, pv, cus, reps);
        row3<8>(R, a, b, ld, C, PR, M, pv, cus, reps);
        return 0;
    }
    for (int bpc : {5, 8}) {
        const int grid = cus * bpc;
        char lab[64];
        snprintf(lab, sizeof lab, "out-of-place bpc%d", bpc);
        row<1>(lab, a, b, ld, R, C, PR, M, pv, grid, reps);
        row<2>(lab, a, b, ld, R, C, PR, M, pv, grid, reps);
        row<3>(lab, a, b, ld, R, C, PR, M, pv, grid, reps);
        row<4>(lab, a, b, ld, R, C, PR, M, pv, grid, reps);
        row<6>(lab, a, b, ld, R, C, PR, M, pv, grid, reps);
        row<8>(lab, a, b, ld, R, C, PR, M, pv, grid, reps);
    }
    row<4>("in-place bpc5", a, a, ld, R, C, PR, M, pv, cus * 5, reps);
    row<8>("in-place bpc5", a, a, ld, R, C, PR, M, pv, cus * 5, reps);
    return 0;
}
