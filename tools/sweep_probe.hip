// sweep_probe.hip -- variants of the block sweep (k_blk_sweep<P>, csrc/smx_block.hpp) measured
// against the production kernel on the same synthetic block (16384^2 by default), bit for bit.
//
// Knobs (template parameters of k_var):
//   ROWS  rows per batch per wave (1 or 2): independent element chains per lane = 2 * ROWS
//   IWIN  1: the fast-division window tracked on the high dwords with 32-bit integer ops
//         (t = (hi << 1) + 0x90000000 is < 0x20200000 exactly when the biased exponent is in
//         [896, 1152], i.e. fd_in; one running unsigned max per lane), 0: fmin/fmax of |num|
//   LDSP  1: the four waves of a workgroup share one column chunk and read the P pivot-row
//         slices from LDS (frees 2*P VGPRs per lane), 0: slices held in VGPRs per wave
//   PF    1: the next batch's loads issued before this batch's arithmetic
// Runtime: blocks per CU.  Each variant's output is compared with the production sweep's.
//
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -I/opt/rocm/include \
//     -L/opt/rocm/lib -lrccl tools/sweep_probe.hip -o tools/sweep_probe
#include "../simplex-method-solver_amd/csrc/smx_kernels.hip"

#include <type_traits>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

namespace {

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

__global__ void k_hdr(BlkHdr* h, int P, int R, int C, int onechunk) {
    if (threadIdx.x != 0) return;
    h->peff = P;
    for (int q = 0; q < kBlkMax; ++q) {
        h->r[q] = (q * 977 + 5) % (R - 1);
        h->c[q] = onechunk ? 7 + 3 * q : (q * 1231 + 7) % C;
        const double e = (q & 1 ? -1.0 : 1.0) * (0.6 + 0.1 * q);
        const FastDiv fd = fd_prep(e);
        h->e[q] = e;
        h->y[q] = fd.y;
        h->ok[q] = fd.ok ? 1 : 0;
    }
}

__global__ void k_cmp(const double* a, const double* b, int64_t ld, int R, int C,
                      unsigned long long* bad) {
    unsigned long long n = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < (int64_t)R * C;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / C, j = t % C;
        n += __double_as_longlong(a[i * ld + j]) != __double_as_longlong(b[i * ld + j]);
    }
    if (n) atomicAdd(bad, n);
}

int64_t leading_dim_probe(int C) { return (C + 15) / 16 * 16; }

constexpr uint32_t kWinBias = 0x90000000u;   // -(896 << 21) mod 2^32
constexpr uint32_t kWinSpan = 0x20200000u;   // (1153 - 896) << 21

template <int IWIN>
struct Win {
    double mn = kFdMaxAbs, mx = 0.0;
    uint32_t t = 0;
    __device__ __forceinline__ void add(double n) {
        if (IWIN) {
            const uint32_t hi = (uint32_t)(__double_as_longlong(n) >> 32);
            t = max(t, (hi << 1) + kWinBias);
        } else {
            mn = fmin(mn, fabs(n));
            mx = fmax(mx, fabs(n));
        }
    }
    __device__ __forceinline__ bool ok() const {
        if (IWIN) return t < kWinSpan;
        return mn >= kFdMinAbs && mx < kFdMaxAbs;
    }
};

template <int P, int ROWS, int IWIN, int LDSP, int PF>
__global__ __launch_bounds__(kUpdBlock) void k_var(const double* __restrict__ Tin,
                                                   double* __restrict__ Tout, int64_t ld, int R,
                                                   int C, const BlkHdr* __restrict__ h,
                                                   const double* __restrict__ mul,
                                                   const double* __restrict__ pr) {
    constexpr int kChunk = 2 * kWave;
    __shared__ dbl2 s_pr[LDSP ? P : 1][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int rq[P], cq[P];
    double eq[P], yq[P];
    bool allok = true;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        rq[q] = h->r[q];
        cq[q] = h->c[q];
        eq[q] = h->e[q];
        yq[q] = h->y[q];
        allok = allok && h->ok[q] != 0;
    }
    const int nchunks = (C + kChunk - 1) / kChunk;
    int ch, base, qs;
    if (LDSP) {
        ch = (int)blockIdx.x % nchunks;
        const int NG = (int)gridDim.x / nchunks;
        base = ((int)blockIdx.x / nchunks) * kUpdWaves + wv;
        qs = NG * kUpdWaves;
    } else {
        const int NW = (int)gridDim.x * kUpdWaves;
        const int w = (int)blockIdx.x * kUpdWaves + wv;
        ch = w % nchunks;
        base = w / nchunks;
        qs = NW / nchunks;
    }
    const int j = ch * kChunk + 2 * lane;
    const int c0 = ch * kChunk;
    const int jc = min(j, (C - 1) & ~1);
    dbl2 prr[LDSP ? 1 : P];
    bool cspecial = !allok;
#pragma unroll
    for (int q = 0; q < P; ++q) cspecial = cspecial || (cq[q] >= c0 && cq[q] < c0 + kChunk);
    if (LDSP) {
        for (int t = threadIdx.x; t < P * kWave; t += kUpdBlock) {
            const int q = t / kWave, l = t % kWave;
            const int jj = ch * kChunk + 2 * l;
            s_pr[q][l] = jj < C ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + jj)
                                : dbl2{0.0, 0.0};
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int q = 0; q < P; ++q)
            prr[q] = (j < C) ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j)
                             : dbl2{0.0, 0.0};
    }
    auto prq = [&](int q) -> dbl2 {
        if (LDSP) return s_pr[q][lane];
        return prr[q];
    };
    auto row_special = [&](int i) {
        bool s = false;
#pragma unroll
        for (int q = 0; q < P; ++q) s = s || i == rq[q];
        return s;
    };
    auto ldrow = [&](int i) -> dbl2 {
        return __builtin_nontemporal_load(
            reinterpret_cast<const dbl2*>(Tin + (int64_t)min(i, R - 1) * ld + jc));
    };
    // one batch: rows i0 + r*qs (r < ROWS), loads in x[]
    auto batch = [&](dbl2* x, int i0) {
        double pc[ROWS][P];
        bool have[ROWS];
        bool special = cspecial;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int i = i0 + r * qs;
            have[r] = i < R;
            special = special || !have[r] || row_special(i);
            const double* m = mul + (int64_t)(have[r] ? i : i0) * kBlkMax;
#pragma unroll
            for (int q = 0; q < P; ++q) pc[r][q] = m[q];
        }
        dbl2 v[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) v[r] = x[r];
        bool ok = false;
        if (!special) {
            Win<IWIN> win;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                const dbl2 p = prq(q);
                double n[2 * ROWS];
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    n[2 * r] = v[r][0] * e - p[0] * pc[r][q];
                    n[2 * r + 1] = v[r][1] * e - p[1] * pc[r][q];
                }
#pragma unroll
                for (int k = 0; k < 2 * ROWS; ++k) {
                    win.add(n[k]);
                    const double tq = n[k] * y;
                    const double rr = fma(-e, tq, n[k]);
                    v[k >> 1][k & 1] = fma(rr, y, tq);
                }
            }
            bool fine = win.ok();
            if (!IWIN) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) fine = fine && v[r][0] == v[r][0] && v[r][1] == v[r][1];
            }
            ok = __all(fine);
        }
        if (!ok) {
            dbl2 ps[P];
#pragma unroll
            for (int q = 0; q < P; ++q) ps[q] = prq(q);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                if (!have[r]) continue;
                const int i = i0 + r * qs;
                const dbl2 xx = *reinterpret_cast<const dbl2*>(Tin + (int64_t)i * ld + jc);
                v[r] = blk_exact<P>(xx, i, j, rq, cq, eq, ps, pc[r]);
            }
        }
        if (j < C) {
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
                if (have[r])
                    __builtin_nontemporal_store(
                        v[r], reinterpret_cast<dbl2*>(Tout + (int64_t)(i0 + r * qs) * ld + j));
        }
    };
    const int step = ROWS * qs;
    if (!PF) {
        for (int i0 = base; i0 < R; i0 += step) {
            dbl2 x[ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) x[r] = ldrow(i0 + r * qs);
            batch(x, i0);
        }
        return;
    }
    dbl2 a[ROWS], b[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) a[r] = ldrow(base + r * qs);
    for (int i0 = base; i0 < R; i0 += 2 * step) {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) b[r] = ldrow(i0 + step + r * qs);
        batch(a, i0);
        if (i0 + step >= R) break;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) a[r] = ldrow(i0 + 2 * step + r * qs);
        batch(b, i0 + step);
    }
}

using VarFn = void (*)(const double*, double*, int64_t, int, int, const BlkHdr*, const double*,
                       const double*);

struct Var {
    const char* name;
    VarFn fn;
    int ldsp;
};

int grid_for(VarFn fn, int bpc, int nchunks, int ldsp, int cus, int R) {
    int blocks = cus * bpc;
    if (ldsp) {
        blocks -= blocks % nchunks;
    } else {
        const int waves = blocks * kUpdWaves;
        int g = nchunks, hh = kUpdWaves;
        while (hh) {
            const int t = g % hh;
            g = hh;
            hh = t;
        }
        const int lcm = nchunks / g * kUpdWaves;
        blocks = (waves - waves % lcm) / kUpdWaves;
    }
    (void)fn;
    (void)R;
    return blocks < 1 ? 1 : blocks;
}


// ---- v2: register-lean form -----------------------------------------------------------------
// The workgroup's four waves share one column chunk: the P pivot-row slices live in LDS, and so
// do the pivot records the rare exact path needs; only e, y (SGPRs) and the batch rows'
// multipliers (SGPRs, scalar loads) stay live in the fast loop.  Special batches (a pivot row
// among the batch's rows) come from a lane-held batch index per pivot (blk_special_batch's
// trick); the window is tracked with integer ops on the high dwords.  DEPTH = load sets in flight.
// an SGPR zero the compiler cannot see through: offsets built from it keep LDS reads (and what is
// computed from them) inside the rare path instead of hoisted into the hot loop's registers
__device__ __forceinline__ int opaque0() {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}
// running max of (hi << 1) + kWinBias (unsigned): one v_lshl_add_u32 per element
__device__ __forceinline__ uint32_t win_term(double n) {
    uint32_t t;
    asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(t) : "v"(__double2hiint(n)), "s"(kWinBias));
    return t;
}

template <int P, int ROWS>
__device__ __forceinline__ int v2_special_batch(const int* s_r, int base, int qs) {
    const int q = threadIdx.x & (kWave - 1);
    int tb = 0x7fffffff;
    if (q < P) {
        const int rq = s_r[q];
        const int d = rq - base;
        if (rq >= 0 && d >= 0 && d % qs == 0) tb = (d / qs) / ROWS;
    }
    return tb;
}

template <int P, int ROWS, int DEPTH, int EYL = 0>
__global__ __launch_bounds__(kUpdBlock) void k_v2(const double* __restrict__ Tin,
                                                  double* __restrict__ Tout, int64_t ld, int R,
                                                  int C, const BlkHdr* __restrict__ h,
                                                  const double* __restrict__ mul,
                                                  const double* __restrict__ pr) {
    constexpr int kChunk = 2 * kWave;
    __shared__ dbl2 s_pr[P][kWave];
    __shared__ double s_e[P];
    __shared__ dbl2 s_ey[P];
    __shared__ int s_r[P], s_c[P];
    __shared__ int s_ok;
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int ch = (int)blockIdx.x % nchunks;
    const int NG = (int)gridDim.x / nchunks;
    const int base = ((int)blockIdx.x / nchunks) * kUpdWaves + wv;
    const int qs = NG * kUpdWaves;
    const int c0 = ch * kChunk, j = c0 + 2 * lane, jc = min(j, (C - 1) & ~1);
    if (tid < P) {
        s_e[tid] = h->e[tid];
        s_ey[tid] = dbl2{h->e[tid], h->y[tid]};
        s_r[tid] = h->r[tid];
        s_c[tid] = h->c[tid];
    }
    if (tid == 0) {
        int ok = 1;
        for (int q = 0; q < P; ++q) ok &= h->ok[q] != 0;
        s_ok = ok;
    }
    for (int t = tid; t < P * kWave; t += kUpdBlock) {
        const int q = t / kWave, l = t % kWave, jj = c0 + 2 * l;
        s_pr[q][l] = jj < C ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + jj)
                            : dbl2{0.0, 0.0};
    }
    __syncthreads();
    double eq[EYL ? 1 : P], yq[EYL ? 1 : P];
    if (!EYL) {
#pragma unroll
        for (int q = 0; q < P; ++q) {
            eq[q] = h->e[q];
            yq[q] = h->y[q];
        }
    }
    bool cspecial = !s_ok;
#pragma unroll
    for (int q = 0; q < P; ++q) cspecial = cspecial || (s_c[q] >= c0 && s_c[q] < c0 + kChunk);
    const int tbq = v2_special_batch<P, ROWS>(s_r, base, qs);
    int tsp = blk_next_batch<P>(tbq, -1);
    auto ldrow = [&](int i) -> dbl2 {
        return __builtin_nontemporal_load(
            reinterpret_cast<const dbl2*>(Tin + (int64_t)min(i, R - 1) * ld + jc));
    };
    auto batch = [&](const dbl2* x, int i0, int t) {
        bool special = cspecial || t == tsp;
        if (t == tsp) tsp = blk_next_batch<P>(tbq, t);
        double pc[ROWS][P];
        bool have[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int i = i0 + r * qs;
            have[r] = i < R;
            special = special || !have[r];
            const double* m = mul + (int64_t)(have[r] ? i : i0) * kBlkMax;
#pragma unroll
            for (int q = 0; q < P; ++q) pc[r][q] = m[q];
        }
        dbl2 v[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) v[r] = x[r];
        bool ok = false;
        if (!special) {
            uint32_t wt = 0;
            const int zb = EYL ? opaque0() : 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                double e, y;
                if (EYL) {
                    const dbl2 ey = s_ey[q + zb];
                    e = ey[0];
                    y = ey[1];
                } else {
                    e = eq[q];
                    y = yq[q];
                }
                const dbl2 p = s_pr[q][lane];
                double n[2 * ROWS];
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    n[2 * r] = v[r][0] * e - p[0] * pc[r][q];
                    n[2 * r + 1] = v[r][1] * e - p[1] * pc[r][q];
                }
#pragma unroll
                for (int k = 0; k < 2 * ROWS; ++k) {
                    wt = max(wt, win_term(n[k]));
                    const double tq = n[k] * y;
                    const double rr = fma(-e, tq, n[k]);
                    v[k >> 1][k & 1] = fma(rr, y, tq);
                }
            }
            ok = __all(wt < kWinSpan);
        }
        if (!ok) {
            // the exact path (rare): one pivot's operands live at a time, re-read from LDS and
            // from the multipliers, the same operations as blk_exact
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                if (!have[r]) continue;
                const int i = i0 + r * qs;
                dbl2 xx = *reinterpret_cast<const dbl2*>(Tin + (int64_t)i * ld + jc);
                const double* m = mul + (int64_t)i * kBlkMax;
#pragma unroll 1
                for (int q = 0; q < P; ++q) {
                    const int rq = s_r[q], cq = s_c[q];
                    const double e = s_e[q], pcq = m[q];
                    const dbl2 p = s_pr[q][lane];
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        double num;
                        if (i == rq) {
                            num = (j + hh == cq) ? 1.0 : -xx[hh];
                        } else {
                            const double a = xx[hh] * e;
                            const double b = p[hh] * pcq;
                            num = (j + hh == cq) ? xx[hh] : (a - b);
                        }
                        xx[hh] = num / e;
                    }
                }
                v[r] = xx;
            }
        }
        if (j < C) {
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
                if (have[r])
                    __builtin_nontemporal_store(
                        v[r], reinterpret_cast<dbl2*>(Tout + (int64_t)(i0 + r * qs) * ld + j));
        }
    };
    const int step = ROWS * qs;
    dbl2 buf[DEPTH][ROWS];
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d)
#pragma unroll
        for (int r = 0; r < ROWS; ++r) buf[d][r] = ldrow(base + d * step + r * qs);
    int t = 0;
    for (int i0 = base; i0 < R; i0 += DEPTH * step) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int ib = i0 + d * step;
            if (ib >= R) break;
            // issue the loads DEPTH - 1 batches ahead into the set freed by the batch before
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
                buf[(d + DEPTH - 1) % DEPTH][r] = ldrow(ib + (DEPTH - 1) * step + r * qs);
            batch(buf[d], ib, t);
            ++t;
        }
    }
}

// the exact path with one pivot's operands live at a time (re-read from the header, the pivot
// rows and the row's multipliers): the same operations as blk_exact
template <int P>
__device__ __forceinline__ dbl2 fx_exact_lean(dbl2 v, int row, int j, const BlkHdr* __restrict__ h,
                                           const double* __restrict__ pr, int64_t ld,
                                           const double* __restrict__ mr) {
    const int jl = min(j, (int)ld - 2);
#pragma unroll 1
    for (int q = 0; q < P; ++q) {
        const int rq = h->r[q], cq = h->c[q];
        const double e = h->e[q], pcq = mr[q];
        const dbl2 p = *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + jl);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            double num;
            if (row == rq) {
                num = (j + hh == cq) ? 1.0 : -v[hh];
            } else {
                const double a = v[hh] * e;
                const double b = p[hh] * pcq;
                num = (j + hh == cq) ? v[hh] : (a - b);
            }
            v[hh] = num / e;
        }
    }
    return v;
}
template <int P, bool NTL, bool PF, int IWIN, int LEAN, int CSEL = 0>
__device__ __forceinline__ void fx_body(const double* Tin, double* Tout, int64_t ld,
                                                     int R, int C, const BlkHdr* __restrict__ h,
                                                     const double* __restrict__ pr,
                                                     const double* __restrict__ mul) {
    const int lane = threadIdx.x & (kWave - 1);
    int rq[P], cq[P];
    double eq[P], yq[P];
    bool allok = true;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        rq[q] = h->r[q];
        cq[q] = h->c[q];
        eq[q] = h->e[q];
        yq[q] = h->y[q];
        allok = allok && h->ok[q] != 0;
    }
    constexpr int kChunk = 2 * kWave;
    const int NW = (int)gridDim.x * kUpdWaves;
    const int w = (int)blockIdx.x * kUpdWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int qs = NW / nchunks;
    const int ch = w % nchunks;
    const int j = ch * kChunk + 2 * lane;
    const int c0 = ch * kChunk;
    dbl2 prs[P];
    bool colchunk = false;
    uint32_t cbits = 0;   // bit 2q+hh: column j+hh is pivot q's column
#pragma unroll
    for (int q = 0; q < P; ++q) {
        prs[q] = (j < C) ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j)
                         : dbl2{0.0, 0.0};
        colchunk = colchunk || (cq[q] >= c0 && cq[q] < c0 + kChunk);
        cbits |= (cq[q] == j ? 1u : 0u) << (2 * q);
        cbits |= (cq[q] == j + 1 ? 1u : 0u) << (2 * q + 1);
    }
    const bool cspecial = !allok || (!CSEL && colchunk);
    const int base = w / nchunks;
    const int tbq = blk_special_batch<P>(h, base, qs);
    int tsp = blk_next_batch<P>(tbq, -1);
    // one batch: rows i0 and i1 = i0 + qs (batch t), their loads x0 / x1 already issued
    auto batch = [&](dbl2 x0, dbl2 x1, int i0, int t) {
        const int i1 = i0 + qs;
        const bool h1 = i1 < R;
        const double* m0 = mul + (int64_t)i0 * kBlkMax;
        const double* m1 = mul + (int64_t)(h1 ? i1 : i0) * kBlkMax;
        double pc0[P], pc1[P];
        const bool special = cspecial || !h1 || t == tsp;
        if (t == tsp) tsp = blk_next_batch<P>(tbq, t);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            pc0[q] = m0[q];
            pc1[q] = m1[q];
        }
        dbl2 v0 = x0, v1 = x1;
        bool ok = false;
        auto fast = [&](auto selc) {
            constexpr bool SEL = decltype(selc)::value;
            double mn = kFdMaxAbs, mx = 0.0;
            uint32_t wt = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                double n[4];
                n[0] = v0[0] * e - prs[q][0] * pc0[q];
                n[1] = v0[1] * e - prs[q][1] * pc0[q];
                n[2] = v1[0] * e - prs[q][0] * pc1[q];
                n[3] = v1[1] * e - prs[q][1] * pc1[q];
                if (SEL) {   // the pivot column: numerator = the element itself (simplex.py:159-160)
                    const bool s0 = (cbits >> (2 * q)) & 1u, s1 = (cbits >> (2 * q + 1)) & 1u;
                    n[0] = s0 ? v0[0] : n[0];
                    n[1] = s1 ? v0[1] : n[1];
                    n[2] = s0 ? v1[0] : n[2];
                    n[3] = s1 ? v1[1] : n[3];
                }
                double rr[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (IWIN) {
                        wt = max(wt, win_term(n[k]));
                    } else {
                        mn = fmin(mn, fabs(n[k]));
                        mx = fmax(mx, fabs(n[k]));
                    }
                    const double tq = n[k] * y;               // fd_div inside its window
                    const double r = fma(-e, tq, n[k]);
                    rr[k] = fma(r, y, tq);
                }
                v0 = dbl2{rr[0], rr[1]};
                v1 = dbl2{rr[2], rr[3]};
            }
            if (IWIN)
                ok = __all(wt < kWinSpan);
            else
                ok = __all(mn >= kFdMinAbs && mx < kFdMaxAbs && v0[0] == v0[0] && v0[1] == v0[1] &&
                           v1[0] == v1[0] && v1[1] == v1[1]);
        };
        if (!special) {
            if (CSEL && colchunk)
                fast(std::integral_constant<bool, true>{});
            else
                fast(std::integral_constant<bool, false>{});
        }
        if (!ok) {
            if (PF) {
                // reloaded (this batch's elements are not written yet, even in place), so the
                // inputs need not stay live beside the chains
                const int jl = min(j, (C - 1) & ~1);
                x0 = *reinterpret_cast<const dbl2*>(Tin + (int64_t)i0 * ld + jl);
                if (h1) x1 = *reinterpret_cast<const dbl2*>(Tin + (int64_t)i1 * ld + jl);
            }
            if (LEAN) {
                v0 = fx_exact_lean<P>(x0, i0, j, h, pr, ld, m0);
                if (h1) v1 = fx_exact_lean<P>(x1, i1, j, h, pr, ld, m1);
            } else {
                v0 = blk_exact<P>(x0, i0, j, rq, cq, eq, prs, pc0);
                if (h1) v1 = blk_exact<P>(x1, i1, j, rq, cq, eq, prs, pc1);
            }
        }
        if (j < C) {
            __builtin_nontemporal_store(v0, reinterpret_cast<dbl2*>(Tout + (int64_t)i0 * ld + j));
            if (h1)
                __builtin_nontemporal_store(v1,
                                            reinterpret_cast<dbl2*>(Tout + (int64_t)i1 * ld + j));
        }
    };
    if (!PF) {
        int t = 0;
        for (int i0 = base; i0 < R; i0 += 2 * qs, ++t) {
            const int i1 = i0 + qs;
            dbl2 x0 = dbl2{0.0, 0.0}, x1 = dbl2{0.0, 0.0};
            if (j < C) {
                x0 = ld2<NTL>(Tin + (int64_t)i0 * ld + j);
                if (i1 < R) x1 = ld2<NTL>(Tin + (int64_t)i1 * ld + j);
            }
            batch(x0, x1, i0, t);
        }
        return;
    }
    // PF: the next batch's two loads are issued before this batch's arithmetic, into the other of
    // two register sets, without branches (row and column clamped into the table; a clamped row's
    // or lane's values are never stored).  The loads are inline asm with explicit waits: the
    // compiler's own vmcnt tracking waits for them at the loop edge.  In-order vmcnt (gfx9): before
    // a set is used, the ops issued after its loads are the previous batch's stores (two, as every
    // wave holds a lane j < C and only the last batch has no row i1) and the other set's loads.
    const int jc = min(j, (C - 1) & ~1);
    auto ldc = [&](int row) {
        dbl2 v;
        const double* p = Tin + (int64_t)min(row, R - 1) * ld + jc;
        if (NTL)
            asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
        else
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
        return v;
    };
    dbl2 a0 = ldc(base), a1 = ldc(base + qs);
    dbl2 b0 = ldc(base + 2 * qs), b1 = ldc(base + 3 * qs);
    asm volatile("s_waitcnt vmcnt(2)" : "+v"(a0), "+v"(a1) :: "memory");
    int t = 0;
    for (int i0 = base; i0 < R; i0 += 4 * qs, t += 2) {
        batch(a0, a1, i0, t);
        if (i0 + 2 * qs >= R) break;
        a0 = ldc(i0 + 4 * qs);
        a1 = ldc(i0 + 5 * qs);
        asm volatile("s_waitcnt vmcnt(4)" : "+v"(b0), "+v"(b1) :: "memory");
        batch(b0, b1, i0 + 2 * qs, t + 1);
        if (i0 + 4 * qs >= R) break;
        b0 = ldc(i0 + 6 * qs);
        b1 = ldc(i0 + 7 * qs);
        asm volatile("s_waitcnt vmcnt(4)" : "+v"(a0), "+v"(a1) :: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no load in flight at exit
}


template <int P, int IWIN, int LEAN, int CSEL = 0>
__global__ __launch_bounds__(kUpdBlock) void k_fx(const double* __restrict__ Tin,
                                                  double* __restrict__ Tout, int64_t ld, int R,
                                                  int C, const BlkHdr* __restrict__ h,
                                                  const double* __restrict__ mul,
                                                  const double* __restrict__ pr) {
    fx_body<P, true, true, IWIN, LEAN, CSEL>(Tin, Tout, ld, R, C, h, pr, mul);
}

}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int P = 8;
    const int R = N, C = N;
    smx_shape s{};
    s.ld = leading_dim_probe(C);
    s.rows = R - 1;
    s.n = R - 1;
    s.m = C - 1;
    s.flen = C - 1;
    s.row0 = 0;
    s.nparts = nparts_for(s.rows, s.m);
    const int64_t ld = s.ld;
    const BlkLayout L = blk_layout(R, ld, s.nparts);
    double *a, *ref, *out;
    char* blk;
    const size_t nb = (size_t)R * ld * 8;
    CK(hipMalloc(&a, nb));
    CK(hipMalloc(&ref, nb));
    CK(hipMalloc(&out, nb));
    CK(hipMalloc(&blk, L.bytes));
    double* mul = reinterpret_cast<double*>(blk + L.mul);
    double* pr = reinterpret_cast<double*>(blk + L.pr);
    BlkHdr* h = reinterpret_cast<BlkHdr*>(blk);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, (int64_t)R * ld, 1ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, pr, (int64_t)kBlkMax * ld, 2ull, -1.0,
                       1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, mul, (int64_t)R * kBlkMax, 3ull, -1.0,
                       1.0);
    hipLaunchKernelGGL(k_hdr, dim3(1), dim3(64), 0, 0, h, P, R, C, argc > 2 ? atoi(argv[2]) : 0);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nchunks = (C + 2 * kWave - 1) / (2 * kWave);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 6;
    // production: in place for even P
    CK(hipMemcpy(ref, a, nb, hipMemcpyDeviceToDevice));
    CK((hipError_t)launch_block_sweep(ref, out, s, P, blk, L, 0));
    CK(hipDeviceSynchronize());
    {
        float best = 1e30f, sum = 0.f;
        CK(hipMemcpy(out, a, nb, hipMemcpyDeviceToDevice));
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            CK((hipError_t)launch_block_sweep(out, ref + 0 * 0, s, P, blk, L, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        // restore the reference result (the timing runs wrote `out` in place from `a`)
        CK(hipMemcpy(ref, a, nb, hipMemcpyDeviceToDevice));
        CK((hipError_t)launch_block_sweep(ref, out, s, P, blk, L, 0));
        CK(hipDeviceSynchronize());
        printf("{\"variant\": \"production\", \"P\": %d, \"best_us\": %.1f, \"mean_us\": %.1f, "
               "\"gbs\": %.0f}\n", P, best * 1e3, sum / reps * 1e3, 16.0 * R * C / (best * 1e-3) / 1e9);
        fflush(stdout);
    }
    unsigned long long* dbad;
    CK(hipMalloc(&dbad, 8));
    const Var vars[] = {
        {"fx_fwin", k_fx<8, 0, 0>, 0},
        {"fx_iwin", k_fx<8, 1, 0>, 0},
        {"fx_fwin_csel", k_fx<8, 0, 0, 1>, 0},
        {"fx_iwin_csel", k_fx<8, 1, 0, 1>, 0},
        {"fx_iwin_lean_csel", k_fx<8, 1, 1, 1>, 0},
    };
    for (const Var& v : vars) {
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, (const void*)v.fn));
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)v.fn, kUpdBlock, 0));
        for (int inplace = 0; inplace < 2; ++inplace) {
            for (int bpc = 6; bpc <= 8; ++bpc) {
                const int grid = grid_for(v.fn, bpc, nchunks, v.ldsp, cus, R);
                // correctness: from a into out (out of place) or a copy in place
                CK(hipMemcpy(out, a, nb, hipMemcpyDeviceToDevice));
                hipLaunchKernelGGL(v.fn, dim3(grid), dim3(kUpdBlock), 0, 0, inplace ? out : a, out,
                                   ld, R, C, (const BlkHdr*)h, (const double*)mul, (const double*)pr);
                CK(hipDeviceSynchronize());
                CK(hipMemset(dbad, 0, 8));
                hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, ref, out, ld, R, C, dbad);
                unsigned long long bad = 0;
                CK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
                float best = 1e30f, sum = 0.f;
                if (inplace) CK(hipMemcpy(out, a, nb, hipMemcpyDeviceToDevice));
                for (int r = 0; r < reps; ++r) {
                    CK(hipEventRecord(e0, 0));
                    hipLaunchKernelGGL(v.fn, dim3(grid), dim3(kUpdBlock), 0, 0, inplace ? out : a,
                                       out, ld, R, C, (const BlkHdr*)h, (const double*)mul,
                                       (const double*)pr);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    best = ms < best ? ms : best;
                    sum += ms;
                }
                printf("{\"variant\": \"%s\", \"inplace\": %d, \"bpc\": %d, \"grid\": %d, "
                       "\"vgpr\": %d, \"occ_api\": %d, \"mismatch\": %llu, \"best_us\": %.1f, "
                       "\"mean_us\": %.1f, \"gbs\": %.0f}\n",
                       v.name, inplace, bpc, grid, fa.numRegs, occ, bad, best * 1e3,
                       sum / reps * 1e3, 16.0 * R * C / (best * 1e-3) / 1e9);
                fflush(stdout);
            }
        }
    }
    CK(hipFree(dbad));
    return 0;
}
