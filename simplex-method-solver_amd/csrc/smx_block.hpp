// smx_block.hpp -- block pivots: P consecutive Jordan steps (recalculate_matrix, simplex.py:143-177)
// applied in ONE HBM sweep of the tableau, their decisions (pick_element, :70-141) planned ahead
// from the block's input table.
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------------------------------------
// Why: one pivot reads and writes every element once (16 B), so a chain of single-pivot sweeps is
// pinned at the copy rate of HBM (16384^2: ~815 us per pivot, 95 % of the measured copy ceiling).
// But the per-element arithmetic is only two multiplies, a subtract and a division:
// tools/multipivot_probe.hip measured 3 chained updates per element in the time of 1, 4 at +7 %.
//
// Every value of T_{k+l} follows from T_k, the pivot rows and the per-row multipliers of the
// steps before it, by the update's own expression (the look-ahead's nv(), applied l times):
//     chain(x = T_k[i][j], L):  for q < L:
//         num = (i == r_q) ? (j == c_q ? 1.0 : -x) : (j == c_q ? x : x*e_q - pr_q[j]*mul[i][q])
//         x = num / e_q
//     pr_q      = row r_q of T_{k+q}        (the pivot row of step k+q, C doubles)
//     mul[i][q] = T_{k+q}[i][c_q]           (row i's pivot-column entry before step k+q)
// so chain(T_k[i][j], l) IS T_{k+l}[i][j], bit for bit (same operations on the same operands in
// the same order as l single-pivot sweeps).  A block of P pivots on T_k is then:
//   k_blk_dec(l), l = 0..P-1   one workgroup: decision l from the records of step k+l (phase 1:
//                              first positive entry of the first-negative-b row, simplex.py:72-91;
//                              phase 2: ratio arg-min, :93-141), pr_l, the f-row of T_{k+l+1}
//                              (kept in `fr`) and its first negative entry (the next entering
//                              column), and the pivot's log / label / x-history bookkeeping;
//   k_blk_cols(l + 1)          nparts workgroups: mul[i][l] for every row, then the records of
//                              step k+l+1 (first negative "-b" row, ratio candidates on the new
//                              entering column) from chains of length l+1;
//   k_blk_sweep                every element T_k -> T_{k+peff} through the peff decided steps,
//                              out of place when peff is odd and in place when it is even, so the
//                              table after d pivots is in buf[(parity + d) & 1] exactly as in the
//                              single-pivot chains.  In place is safe: each element is read and
//                              written by the same lane and nothing reads T_k after the planner.
// k_blk_cols(P) computes the records of the NEXT block's first step (chains of length P from this
// block's T_k), so a block is 2P + 1 launches.  A terminal outcome at step l latches ctl->term;
// the sweep still applies the l pivots decided before it and every later kernel does nothing.
constexpr int kBlkMax = 8;           // pivots per block (mul row stride)
constexpr int kBlkDec = 1024;        // k_blk_dec / k_blk_prime workgroup

struct BlkHdr {
    int32_t peff;                    // pivots of this block decided so far (the sweep's count)
    int32_t cf;                      // first j < fscan with fr[j] < 0 (SMX_NONE: none)
    int32_t pad[2];
    int32_t r[kBlkMax], c[kBlkMax];
    int32_t ok[kBlkMax];             // e inside the fast-division window (fd_prep)
    double e[kBlkMax], y[kBlkMax];   // pivot element and its refined reciprocal (fd_prep)
};
static_assert(sizeof(BlkHdr) <= 256, "block header");

// Scratch layout (byte offsets; smx_block_bytes): header | records [kBlkMax][nparts] |
// mul [R][kBlkMax] | pr [kBlkMax][ld] | fr [ld]
struct BlkLayout {
    int64_t parts, mul, pr, fr, bytes;
};
inline int64_t blk_align(int64_t x) { return (x + 255) / 256 * 256; }
inline BlkLayout blk_layout(int64_t R, int64_t ld, int nparts) {
    BlkLayout L;
    L.parts = 256;
    L.mul = blk_align(L.parts + (int64_t)kBlkMax * nparts * 32);
    L.pr = blk_align(L.mul + R * kBlkMax * 8);
    L.fr = blk_align(L.pr + (int64_t)kBlkMax * ld * 8);
    L.bytes = blk_align(L.fr + ld * 8);
    return L;
}

struct BlkPiv {
    int r[kBlkMax], c[kBlkMax];
    double e[kBlkMax];
};

// T_{k+L}[i][j] from x = T_k[i][j]; p[q] = pr_q[j], mq[q] = mul[i][q] (loaded by the caller, all
// before the first use, so a chain costs one memory round trip, not L)
template <int L>
__device__ __forceinline__ double blk_chain(double x, int i, int j, const BlkPiv& pv,
                                            const double* p, const double* mq) {
#pragma unroll
    for (int q = 0; q < L; ++q) {
        const double e = pv.e[q];
        double num;
        if (i == pv.r[q]) {
            num = (j == pv.c[q]) ? 1.0 : -x;
        } else {
            const double a = x * e;
            const double b = p[q] * mq[q];
            num = (j == pv.c[q]) ? x : (a - b);
        }
        x = num / e;
    }
    return x;
}

template <int L>
__device__ __forceinline__ void blk_load_col(const double* __restrict__ pr, int64_t ld, int j,
                                             double* p) {
#pragma unroll
    for (int q = 0; q < L; ++q) p[q] = pr[(int64_t)q * ld + j];
}

__device__ __forceinline__ void blk_load_piv(const BlkHdr* h, int L, BlkPiv* s_pv) {
    const int t = threadIdx.x;
    if (t < L) {
        s_pv->r[t] = h->r[t];
        s_pv->c[t] = h->c[t];
        s_pv->e[t] = h->e[t];
    }
}

// Chain start: the f-row of T into `fr` and its first negative entry (simplex.py:94-98).
__global__ __launch_bounds__(kBlkDec) void k_blk_prime(const double* __restrict__ T, int64_t ld,
                                                        int rows, int m, int fscan,
                                                        const smx_ctl* __restrict__ ctl,
                                                        char* __restrict__ blk, int64_t off_fr) {
    __shared__ int s_tmp[kBlkDec / kWave];
    if (ctl->term) return;
    const int C = m + 1;
    const double* f = T + (int64_t)rows * ld;
    double* fr = reinterpret_cast<double*>(blk + off_fr);
    int nf = SMX_NONE;
    for (int j = threadIdx.x; j < C; j += kBlkDec) {
        const double v = f[j];
        fr[j] = v;
        if (j < fscan && v < 0.0 && j < nf) nf = j;
    }
    nf = block_min_int<kBlkDec>(nf, s_tmp);
    if (threadIdx.x == 0) {
        BlkHdr* h = reinterpret_cast<BlkHdr*>(blk);
        h->cf = nf;
        h->peff = 0;
    }
}

// The records of step k+L (chains of length L from T_k) and, for L >= 1, mul[i][L-1] and the
// x-history entry of step k+L-1 (the new "-b" entry of the rows labelled x1 / x2).  Workgroup b
// of nparts covers rows b*NT + tid + q*nparts*NT (the layout of la_partial); L == P is the next
// block's first step (record slot 0).
template <int L>
__global__ __launch_bounds__(kUpdBlock) void k_blk_cols(
    const double* __restrict__ T, int64_t ld, int rows, int m, int P, int parity,
    const smx_ctl* __restrict__ ctl, char* __restrict__ blk, int64_t off_parts, int64_t off_mul,
    int64_t off_pr, double* __restrict__ xhist, int64_t log_cap) {
    constexpr int NT = kUpdBlock;
    __shared__ BlkPiv s_pv;
    __shared__ int s_cf;
    __shared__ int s_b[NT / kWave];
    __shared__ First s_f[NT / kWave];
    __shared__ Cand s_c[NT / kWave];
    if (ctl->term) return;
    const BlkHdr* h = reinterpret_cast<const BlkHdr*>(blk);
    smx_part* parts = reinterpret_cast<smx_part*>(blk + off_parts);
    double* mul = reinterpret_cast<double*>(blk + off_mul);
    const double* pr = reinterpret_cast<const double*>(blk + off_pr);
    const int tid = threadIdx.x;
    blk_load_piv(h, L, &s_pv);
    if (tid == 0) s_cf = h->cf;
    __syncthreads();
    const int cf = s_cf;
    const int cp = L > 0 ? s_pv.c[L > 0 ? L - 1 : 0] : 0;
    // x-history of step k+L-1: rows of labels x1 / x2 after it (k_blk_dec moved the labels)
    int hx0 = -1, hx1 = -1;
    int64_t hslot = 0;
    if (L > 0 && xhist != nullptr && log_cap > 0) {
        const int sp = (parity + L) & 1;
        hx0 = ctl->xpos[sp][0];
        hx1 = ctl->xpos[sp][1];
        hslot = 2 * ((ctl->npiv[sp] - 1) % log_cap);
    }
    // the pivot rows at the three columns this kernel reads (uniform across the workgroup)
    double pp[kBlkMax], pb[kBlkMax], pa[kBlkMax];
    blk_load_col<(L > 1 ? L - 1 : 0)>(pr, ld, cp, pp);
    blk_load_col<L>(pr, ld, m, pb);
    if (cf != SMX_NONE) blk_load_col<L>(pr, ld, cf, pa);
    const int b = blockIdx.x, nparts = gridDim.x;
    int nb = SMX_NONE;
    First f{SMX_NONE, 0.0};
    Cand bc = cand_none();
    for (int i = b * NT + tid; i < rows; i += nparts * NT) {
        const double* row = T + (int64_t)i * ld;
        double* mr = mul + (int64_t)i * kBlkMax;
        // every load of the row first: three strided entries and the row's multipliers
        const double xp = L > 0 ? row[cp] : 0.0;
        const double xb = row[m];
        const double xa = cf != SMX_NONE ? row[cf] : 0.0;
        double mq[kBlkMax];
#pragma unroll
        for (int q = 0; q + 1 < L; ++q) mq[q] = mr[q];
        if (L > 0) {
            mq[L > 0 ? L - 1 : 0] = blk_chain<(L > 1 ? L - 1 : 0)>(xp, i, cp, s_pv, pp, mq);
            mr[L > 0 ? L - 1 : 0] = mq[L > 0 ? L - 1 : 0];
        }
        const double bv = blk_chain<L>(xb, i, m, s_pv, pb, mq);
        if (i == hx0) xhist[hslot] = bv;
        if (i == hx1) xhist[hslot + 1] = bv;
        if (bv < 0.0 && i < nb) nb = i;                      // simplex.py:73-76
        if (cf != SMX_NONE) {
            const double a = blk_chain<L>(xa, i, cf, s_pv, pa, mq);
            if (a != 0.0) {                                 // simplex.py:112 (NaN counts)
                const double v = bv / a;                    // simplex.py:115
                if (i < f.idx) {
                    f.idx = i;
                    f.v = v;
                }
                if (!isnan(v)) {
                    const Cand x = classify(v, i);
                    if (better(x, bc)) bc = x;
                }
            }
        }
    }
    nb = wave_min_int(nb);
    f = wave_first(f);
    bc = wave_best(bc);
    const int wid = tid >> 6;
    if ((tid & 63) == 0) {
        s_b[wid] = nb;
        s_f[wid] = f;
        s_c[wid] = bc;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < NT / kWave; ++w) {
            nb = min(nb, s_b[w]);
            if (s_f[w].idx < f.idx) f = s_f[w];
            if (better(s_c[w], bc)) bc = s_c[w];
        }
        smx_part pt;
        pt.p1col = nb;
        pt.first = f.idx;
        pt.first_v = f.v;
        pt.best_cls = bc.cls;
        pt.best_i = bc.idx;
        pt.best_v = bc.v;
        const int slot = (L == P) ? 0 : L;
        parts[(int64_t)slot * nparts + b] = pt;
    }
}

// Decision L of the block (step k+L, parity slot sp = (parity + L) & 1) and everything the
// sweep and the next planning step need from it.  One workgroup.
template <int L>
__global__ __launch_bounds__(kBlkDec) void k_blk_dec(
    const double* __restrict__ T, int64_t ld, int rows, int m, int flen, int fscan, int nparts,
    int parity, smx_ctl* __restrict__ ctl, char* __restrict__ blk, int64_t off_parts,
    int64_t off_mul, int64_t off_pr, int64_t off_fr, int32_t* __restrict__ log,
    double* __restrict__ xhist, int64_t log_cap) {
    constexpr int NT = kBlkDec;
    __shared__ BlkPiv s_pv;
    __shared__ int s_tmp[NT / kWave];
    __shared__ Decision s_d;
    __shared__ int s_nb, s_cf;
    BlkHdr* h = reinterpret_cast<BlkHdr*>(blk);
    const int tid = threadIdx.x;
    if (ctl->term) {
        if (L == 0 && tid == 0) h->peff = 0;   // a later block of a stopped chain sweeps nothing
        return;
    }
    const smx_part* parts = reinterpret_cast<const smx_part*>(blk + off_parts) + (int64_t)L * nparts;
    double* mul = reinterpret_cast<double*>(blk + off_mul);
    double* pr = reinterpret_cast<double*>(blk + off_pr);
    double* fr = reinterpret_cast<double*>(blk + off_fr);
    const int sp = (parity + L) & 1;
    blk_load_piv(h, L, &s_pv);
    if (tid < kWave) {
        smx_part rec{SMX_NONE, SMX_NONE, 0.0, 3, SMX_NONE, 0.0};
        if (tid < nparts) rec = parts[tid];
        const int c = h->cf;
        int nb = wave_min_int(rec.p1col);
        First f = wave_first(First{rec.first, rec.first_v});
        Cand b = wave_best(Cand{rec.best_cls, rec.best_i, rec.best_v});
        Decision d;
        d.c = c;
        d.r = SMX_NONE;
        d.status = SMX_PIVOT;
        if (nb == SMX_NONE) {          // phase 2 (the records were built for column c)
            if (c == SMX_NONE) {
                d.status = (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;   // simplex.py:101-103
            } else if (f.idx == SMX_NONE) {
                d.status = SMX_NOT_CONVERGE;                       // simplex.py:138-139
            } else if (isnan(f.v)) {
                d.r = f.idx;                                       // simplex.py:117-121
            } else if (b.cls >= 2) {
                d.status = SMX_NOT_CONVERGE;
            } else {
                d.r = b.idx;
            }
        }
        if (tid == 0) {
            s_nb = nb;
            s_cf = c;
            s_d = d;
        }
    }
    __syncthreads();
    const int nb = s_nb;
    Decision d = s_d;
    const int C = m + 1;
    double* prl = pr + (int64_t)L * ld;
    if (nb != SMX_NONE || d.status == SMX_PIVOT) {
        // the pivot row of T_{k+L} (phase 1: also its first positive entry, simplex.py:81-85)
        const int r = nb != SMX_NONE ? nb : d.r;
        const double* row = T + (int64_t)r * ld;
        const double* mrow = mul + (int64_t)r * kBlkMax;
        double mq[kBlkMax];
#pragma unroll
        for (int q = 0; q < L; ++q) mq[q] = mrow[q];
        int p1 = SMX_NONE;
#pragma unroll 2
        for (int j = tid; j < C; j += NT) {
            double p[kBlkMax];
            blk_load_col<L>(pr, ld, j, p);
            const double v = blk_chain<L>(row[j], r, j, s_pv, p, mq);
            prl[j] = v;
            if (j < m && v > 0.0 && j < p1) p1 = j;
        }
        if (nb != SMX_NONE) {
            p1 = block_min_int<NT>(p1, s_tmp);
            d.r = nb;
            d.c = p1;
            d.status = (p1 == SMX_NONE) ? SMX_INCORRECT : SMX_PIVOT;
        }
    }
    if (d.status != SMX_PIVOT) {
        if (tid == 0) {
            ctl->sel_status = d.status;
            ctl->sel_r = d.r;
            ctl->sel_c = d.c;
            ctl->negb[sp] = nb;         // the state of T_{k+L}, where the chain stops
            ctl->negf[sp] = s_cf;
            ctl->term = 1;
            h->peff = L;
        }
        return;
    }
    __syncthreads();                    // prl complete
    const int r = d.r, c = d.c;
    const double e = prl[c];
    const double fc = fr[c];
    __syncthreads();                    // every thread has fc before fr[c] changes
    if (tid == 0) {
        // bookkeeping of the pivot (its latency overlaps the f-row pass of the other waves);
        // the x-history value of a basic label is written by k_blk_cols<L + 1>
        const FastDiv fd = fd_prep(e);
        mul[(int64_t)rows * kBlkMax + L] = fc;
        h->r[L] = r;
        h->c[L] = c;
        h->e[L] = e;
        h->y[L] = fd.y;
        h->ok[L] = fd.ok ? 1 : 0;
        const int64_t k = ctl->npiv[sp];
        if (log_cap > 0) {
            log[2 * (k % log_cap)] = r;
            log[2 * (k % log_cap) + 1] = c;
        }
        ctl->npivots = k + 1;
        ctl->npiv[sp ^ 1] = k + 1;
        ctl->sel_status = SMX_PIVOT;
        ctl->sel_r = r;
        ctl->sel_c = c;
        ctl->sel_e = e;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int code = move_label(ctl->xpos[sp][q], r, c);
            ctl->xpos[sp ^ 1][q] = code;
            if (xhist && log_cap > 0 && code < 0) xhist[2 * (k % log_cap) + q] = 0.0;  // :60-66
        }
    }
    // the f-row of T_{k+L+1} (row `rows`, never the pivot row) and its first negative entry
    int nf = SMX_NONE;
#pragma unroll 2
    for (int j = tid; j < C; j += NT) {
        const double x = fr[j];
        const double a = x * e;
        const double b = prl[j] * fc;
        const double v = ((j == c) ? x : (a - b)) / e;
        fr[j] = v;
        if (j < fscan && v < 0.0 && j < nf) nf = j;
    }
    nf = block_min_int<NT>(nf, s_tmp);
    if (tid == 0) {
        h->peff = L + 1;
        h->cf = nf;
    }
}

// The sweep: T_k -> T_{k+P} for every element (P = peff pivots of this block).  The pivot data
// is wave-uniform (scalar loads); the division takes fd_div's hoisted form when the whole wave's
// numerators lie in its window (one vote per unit and pivot), else the hardware division for
// the lanes outside it -- bit-identical either way (smx_resident.hpp).
template <int P, bool NTL>
__device__ __forceinline__ void blk_sweep_body(const double* Tin, double* Tout, int64_t ld, int R,
                                               int C, const BlkHdr* __restrict__ h,
                                               const double* __restrict__ pr,
                                               const double* __restrict__ mul) {
    const int lane = threadIdx.x & (kWave - 1);
    int rq[P], cq[P], okq[P];
    double eq[P], yq[P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
        rq[q] = h->r[q];
        cq[q] = h->c[q];
        okq[q] = h->ok[q];
        eq[q] = h->e[q];
        yq[q] = h->y[q];
    }
    constexpr int kChunk = 2 * kWave;
    constexpr int U = 2;
    const int NW = (int)gridDim.x * kUpdWaves;
    const int w = (int)blockIdx.x * kUpdWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int64_t units = (int64_t)nchunks * R;
    const int qs = NW / nchunks, rs = NW % nchunks;
    int i = w / nchunks, ch = w % nchunks;
    int ch_pr = -1;
    dbl2 prs[P];
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
            if (ii[k] < R && j < C) x[k] = ld2<NTL>(Tin + (int64_t)ii[k] * ld + j);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int row = ii[k];
            if (row >= R) continue;
            const int j = cc[k] * kChunk + 2 * lane;
            if (cc[k] != ch_pr) {
                ch_pr = cc[k];
#pragma unroll
                for (int q = 0; q < P; ++q)
                    prs[q] = (j < C) ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j)
                                     : dbl2{0.0, 0.0};
            }
            const double* mr = mul + (int64_t)row * kBlkMax;
            double pc[P];
#pragma unroll
            for (int q = 0; q < P; ++q) pc[q] = mr[q];
            dbl2 v = x[k];
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                dbl2 num;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int jj = j + hh;
                    if (row == rq[q]) {
                        num[hh] = (jj == cq[q]) ? 1.0 : -v[hh];
                    } else {
                        const double a = v[hh] * e;
                        const double b = prs[q][hh] * pc[q];
                        num[hh] = (jj == cq[q]) ? v[hh] : (a - b);
                    }
                }
                // q' = x*y ; r = fma(-e, q', x) ; fma(r, y, q')  (fd_div inside its window)
                dbl2 out;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const double t = num[hh] * y;
                    const double rr = fma(-e, t, num[hh]);
                    out[hh] = fma(rr, y, t);
                }
                const int in = (int)fd_in(num[0]) & (int)fd_in(num[1]);
                if (!(okq[q] && __all(in))) {
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh)
                        if (!(okq[q] && fd_in(num[hh]))) out[hh] = num[hh] / e;
                }
                v = out;
            }
            if (j < C)
                __builtin_nontemporal_store(v, reinterpret_cast<dbl2*>(Tout + (int64_t)row * ld + j));
        }
    }
}

template <int PMAX, bool NTL>
__global__ __launch_bounds__(kUpdBlock) void k_blk_sweep(double* b_in, double* b_other, int64_t ld,
                                                         int R, int C,
                                                         const BlkHdr* __restrict__ h,
                                                         const double* __restrict__ mul,
                                                         const double* __restrict__ pr) {
    const int peff = h->peff;
    if (peff <= 0) return;
    double* out = (peff & 1) ? b_other : b_in;
#define SMX_BLK_CASE(n)                                                           \
    if constexpr (PMAX >= n) {                                                    \
        if (peff == n) {                                                          \
            blk_sweep_body<n, NTL>(b_in, out, ld, R, C, h, pr, mul);              \
            return;                                                               \
        }                                                                         \
    }
    SMX_BLK_CASE(1)
    SMX_BLK_CASE(2)
    SMX_BLK_CASE(3)
    SMX_BLK_CASE(4)
    SMX_BLK_CASE(5)
    SMX_BLK_CASE(6)
    SMX_BLK_CASE(7)
    SMX_BLK_CASE(8)
#undef SMX_BLK_CASE
}

// End of a block chain: the state of the final table into ctl slot `parity` (first negative
// "-b" row from the next step's records, entering column from `fr`), like k_publish.
__global__ __launch_bounds__(kWave) void k_blk_publish(const char* __restrict__ blk,
                                                       int64_t off_parts, int nparts, int parity,
                                                       smx_ctl* __restrict__ ctl) {
    if (ctl->term) return;
    const smx_part* parts = reinterpret_cast<const smx_part*>(blk + off_parts);   // slot 0
    int nb = SMX_NONE;
    for (int k = threadIdx.x; k < nparts; k += kWave) nb = min(nb, parts[k].p1col);
    nb = wave_min_int(nb);
    if (threadIdx.x == 0) {
        ctl->negb[parity] = nb;
        ctl->negf[parity] = reinterpret_cast<const BlkHdr*>(blk)->cf;
        ctl->negb[parity ^ 1] = SMX_NONE;
        ctl->negf[parity ^ 1] = SMX_NONE;
    }
}

}  // namespace
