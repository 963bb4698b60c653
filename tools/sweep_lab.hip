// sweep_lab.hip -- standalone lab for the block sweep's inner loop (k_blk_sweep, one row per
// batch, csrc/smx_block.hpp blk_sweep_body_row1): the bounded fast path only (every unit free:
// no pivot rows, no pivot columns in the table), so variants of the loop structure can be timed
// in seconds of compile time.  Every variant's output is compared bit for bit with variant 0.
//
//   V0 prod      production structure: wave keeps chunk w % nchunks, next row's load issued before
//                this row's arithmetic; per row the multipliers' bound check (scalar + v_max3)
//                and the inputs' bound check (one vote)
//   V1 rowflag   V0 with the multipliers' bound check replaced by a per-row flag precomputed by
//                the planner (one scalar load + compare)
//   V2 ldspr     V1 with the pivot-row slices in LDS, shared by the 4 waves of a workgroup
//                (all four work on one chunk): ~40 fewer VGPRs at P = 10
//   V3 ldspr2    V2 with two rows prefetched instead of one
//   V4 depth2    V1 with two rows prefetched (registers)
//   V5 nocheck   V1 without the inputs' vote (timing only: not safe in general)
//   V6 nofall    V1 without the exact fallback (timing only: register floor of the fast path)
//   V7 selbr     V6 plus the flag form's per-pivot uniform branch selecting a pivot column's
//                numerator (never taken here: no pivot columns in the lab's table)
//   V8 window    V7 plus the window-tracked path in the else branch and the exact fallback
//   V9 window2   V1 plus the window-tracked path in the else branch (no selects anywhere): the
//                compiler hoists the two paths' common arithmetic and computes the window terms
//                on the fast path too (60 extra VALU per row)
//   V10 (arg 'a') V9 with an empty volatile asm heading the window path, which stops that
//   V11 (arg 'b') V10 plus a second fast path with v_div_fixup (the production flag form's
//                zero-safe path) between the fast and the window paths
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/sweep_lab.hip \
//          -o tools/sweep_lab
// Run:   tools/sweep_lab [N=16384] [P=10] [reps=5] [bpc=7]
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
constexpr int kMaxP = 16;
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kBndBias = 0u - (923u << 21);
constexpr uint32_t kBndSpan = 201u << 21;
constexpr uint32_t kBndXMax = 1124u << 21;
__device__ __forceinline__ uint32_t bnd_term(double v) {
    return ((uint32_t)__double2hiint(v) << 1) + kBndBias;
}

struct Hdr {
    double e[kMaxP], y[kMaxP];
};

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

__global__ void k_hdr(Hdr* h) {
    const int q = threadIdx.x;
    if (q >= kMaxP) return;
    const double e = (q & 1 ? -1.0 : 1.0) * (0.6 + 0.1 * q);
    h->e[q] = e;
    h->y[q] = fd_recip(e);
}

// per-row flag: every multiplier of the row bounded (what the planner would write)
template <int P>
__global__ void k_rowflag(const double* mul, int R, int32_t* flag) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R; i += gridDim.x * blockDim.x) {
        uint32_t mt = 0;
        for (int q = 0; q < P; ++q) mt = max(mt, bnd_term(mul[(int64_t)i * kMaxP + q]));
        flag[i] = mt < kBndSpan ? 1 : 0;
    }
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

template <int P, int V>
__global__ __launch_bounds__(kBlk) void k_sweep(double* T, int64_t ld, int R, int C,
                                                const Hdr* __restrict__ h,
                                                const double* __restrict__ pr,
                                                const double* __restrict__ mul,
                                                const int32_t* __restrict__ rowok,
                                                uint32_t cmask_arg) {
    constexpr bool LDSPR = V == 2 || V == 3;
    constexpr int DEPTH = (V == 3 || V == 4) ? 2 : 1;
    __shared__ dbl2 s_pr[LDSPR ? P : 1][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double eq[P], yq[P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
        eq[q] = h->e[q];
        yq[q] = h->y[q];
    }
    constexpr int kChunk = 2 * kWave;
    const int nchunks = (C + kChunk - 1) / kChunk;
    int ch, base, qs;
    if (LDSPR) {
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
    dbl2 prs[LDSPR ? 1 : P];
    uint32_t pt = 0;
    if (LDSPR) {
        for (int t = threadIdx.x; t < P * kWave; t += kBlk) {
            const int q = t / kWave, l = t % kWave;
            s_pr[q][l] = *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + ch * kChunk + 2 * l);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const dbl2 p = s_pr[q][lane];
            pt = max(pt, max(bnd_term(p[0]), bnd_term(p[1])));
        }
    } else {
#pragma unroll
        for (int q = 0; q < P; ++q) {
            prs[q] = *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j);
            pt = max(pt, max(bnd_term(prs[q][0]), bnd_term(prs[q][1])));
        }
    }
#pragma unroll
    for (int q = 0; q < P; ++q) pt = max(pt, bnd_term(eq[q]));
    const bool chunk_free = __all(pt < kBndSpan);
    const uint32_t cmask = (V >= 7) ? cmask_arg : 0u;
    const uint32_t cbits = (V >= 7) ? (cmask_arg >> (lane & 15)) : 0u;
    auto row = [&](dbl2 x0, int i0) {
        const double* m0 = mul + (int64_t)i0 * kMaxP;
        double pc[P];
        bool rfree;
        if (V == 0) {
            uint32_t mt = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                pc[q] = m0[q];
                mt = max(mt, bnd_term(pc[q]));
            }
            rfree = mt < kBndSpan;
        } else {
#pragma unroll
            for (int q = 0; q < P; ++q) pc[q] = m0[q];
            rfree = rowok[i0] != 0;
        }
        dbl2 v = x0;
        bool ok = false;
        bool xok = true;
        if (V != 5) {
            const uint32_t xt = max((uint32_t)__double2hiint(x0[0]) << 1,
                                    (uint32_t)__double2hiint(x0[1]) << 1);
            xok = __all(xt < kBndXMax);
        }
        if (chunk_free && rfree && xok) {
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                dbl2 p;
                if (LDSPR)
                    p = s_pr[q][lane];
                else
                    p = prs[q];
                double n[2];
                n[0] = v[0] * e - p[0] * pc[q];
                n[1] = v[1] * e - p[1] * pc[q];
                if ((V == 7 || V == 8) && (cmask & (1u << q))) {
                    n[0] = ((cbits >> (2 * q)) & 1u) ? v[0] : n[0];
                    n[1] = ((cbits >> (2 * q + 1)) & 1u) ? v[1] : n[1];
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const double tq = n[k] * y;
                    const double r = fma(-e, tq, n[k]);
                    v[k] = fma(r, y, tq);
                }
            }
            ok = true;
        } else if (V == 11 && __all((((uint32_t)__double2hiint(x0[0]) << 1) + kBndBias < kBndSpan) &&
                                    (((uint32_t)__double2hiint(x0[1]) << 1) + kBndBias < kBndSpan))) {
            // V11: a production-like second fast path (v_div_fixup per step) ...
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                const dbl2 p = prs[q];
                double n[2];
                n[0] = v[0] * e - p[0] * pc[q];
                n[1] = v[1] * e - p[1] * pc[q];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const double tq = n[k] * y;
                    const double r = fma(-e, tq, n[k]);
                    v[k] = __builtin_amdgcn_div_fixup(fma(r, y, tq), e, n[k]);
                }
            }
            ok = true;
        } else if (V == 8 || V == 9 || V == 10 || V == 11) {
            // V10: an empty volatile asm first, so the compiler cannot hoist this path's
            // arithmetic (and its window terms) into the common code of both branches
            if (V == 10 || V == 11) asm volatile("" ::: "memory");
            uint32_t wt = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                const dbl2 p = prs[q];
                double n[2];
                n[0] = v[0] * e - p[0] * pc[q];
                n[1] = v[1] * e - p[1] * pc[q];
                if (V == 8 && (cmask & (1u << q))) {  // (not V9 / V10)
                    n[0] = ((cbits >> (2 * q)) & 1u) ? v[0] : n[0];
                    n[1] = ((cbits >> (2 * q + 1)) & 1u) ? v[1] : n[1];
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    wt = max(wt, (uint32_t)(__double2hiint(n[k]) << 1) + 0x90000000u);
                    const double tq = n[k] * y;
                    const double r = fma(-e, tq, n[k]);
                    v[k] = fma(r, y, tq);
                }
            }
            ok = __all(wt < 0x20200000u);
        }
        if (V != 6 && V != 7 && !ok) {  // V8 included
            // reloaded (this row is not written yet), so x0 need not stay live beside the chain
            v = *reinterpret_cast<const dbl2*>(T + (int64_t)i0 * ld + min(j, (C - 1) & ~1));
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const dbl2 p = LDSPR ? s_pr[q][lane] : prs[q];
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) v[hh] = (v[hh] * eq[q] - p[hh] * pc[q]) / eq[q];
            }
        }
        if (j < C) __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(T + (int64_t)i0 * ld + j));
    };
    const int jc = min(j, (C - 1) & ~1);
    auto ldc = [&](int r) { return ldnt(T + (int64_t)min(r, R - 1) * ld + jc); };
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
        // three register sets, two rows in flight while one is computed: before a set is used
        // the ops issued after its load are the other two sets' loads and (steady state) two
        // stores -> vmcnt(4); the prologue waits vmcnt(2) then vmcnt(3)
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

using Fn = void (*)(double*, int64_t, int, int, const Hdr*, const double*, const double*,
                    const int32_t*, uint32_t);

template <int P>
Fn pick(int v) {
    switch (v) {
        case 0: return k_sweep<P, 0>;
        case 1: return k_sweep<P, 1>;
        case 2: return k_sweep<P, 2>;
        case 3: return k_sweep<P, 3>;
        case 4: return k_sweep<P, 4>;
        case 5: return k_sweep<P, 5>;
        case 6: return k_sweep<P, 6>;
        case 7: return k_sweep<P, 7>;
        case 8: return k_sweep<P, 8>;
        case 9: return k_sweep<P, 9>;
        case 10: return k_sweep<P, 10>;
        default: return k_sweep<P, 11>;
    }
}
Fn pickP(int P, int v) {
    switch (P) {
        case 8: return pick<8>(v);
        case 10: return pick<10>(v);
        case 12: return pick<12>(v);
        default: return pick<10>(v);
    }
}
void rowflag(int P, const double* mul, int R, int32_t* f) {
    if (P == 8) hipLaunchKernelGGL(k_rowflag<8>, dim3(256), dim3(256), 0, 0, mul, R, f);
    else if (P == 12) hipLaunchKernelGGL(k_rowflag<12>, dim3(256), dim3(256), 0, 0, mul, R, f);
    else hipLaunchKernelGGL(k_rowflag<10>, dim3(256), dim3(256), 0, 0, mul, R, f);
}

}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int P = argc > 2 ? atoi(argv[2]) : 10;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int bpc = argc > 4 ? atoi(argv[4]) : 7;
    const char* only = argc > 5 ? argv[5] : "012345";   // variant digits; 'a' = V10
    const int R = N, C = N;
    const int64_t ld = C;
    const int64_t nel = (int64_t)R * ld;
    double *T0, *T, *ref, *pr, *mul;
    Hdr* h;
    int32_t* flag;
    unsigned long long* bad;
    CK(hipMalloc(&T0, nel * 8));
    CK(hipMalloc(&T, nel * 8));
    CK(hipMalloc(&ref, nel * 8));
    CK(hipMalloc(&pr, (int64_t)kMaxP * ld * 8));
    CK(hipMalloc(&mul, (int64_t)R * kMaxP * 8));
    CK(hipMalloc(&h, sizeof(Hdr)));
    CK(hipMalloc(&flag, (int64_t)R * 4));
    CK(hipMalloc(&bad, 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, T0, nel, 1ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, pr, (int64_t)kMaxP * ld, 2ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, mul, (int64_t)R * kMaxP, 3ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_hdr, dim3(1), dim3(64), 0, 0, h);
    rowflag(P, mul, R, flag);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nchunks = (C + 127) / 128;
    int grid = cus * bpc;
    grid -= grid % nchunks;   // every variant: waves a multiple of the chunks, blocks too
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 16.0 * R * C;
    for (const char* o = only; *o; ++o) {
        const int v = *o == 'a' ? 10 : (*o == 'b' ? 11 : *o - '0');
        Fn fn = pickP(P, v);
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, (const void*)fn));
        std::vector<float> ms;
        unsigned long long nbad = 0;
        for (int r = 0; r < reps + 1; ++r) {
            CK(hipMemcpy(T, T0, nel * 8, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlk), 0, 0, T, ld, R, C, h, pr, mul, flag, 0u);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r > 0) ms.push_back(t);
        }
        if (v == 0) {
            CK(hipMemcpy(ref, T, nel * 8, hipMemcpyDeviceToDevice));
        } else {
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, ref, T, nel, bad);
            CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
        }
        std::sort(ms.begin(), ms.end());
        printf("{\"N\": %d, \"P\": %d, \"variant\": %d, \"grid\": %d, \"vgprs\": %d, "
               "\"best_us\": %.1f, \"median_us\": %.1f, \"tbs\": %.3f, \"mismatch\": %llu}\n",
               N, P, v, grid, fa.numRegs, ms[0] * 1e3, ms[ms.size() / 2] * 1e3,
               bytes / (ms[0] * 1e-3) / 1e12, nbad);
        fflush(stdout);
    }
    return 0;
}
