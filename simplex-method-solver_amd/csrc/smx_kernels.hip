// smx_kernels.hip -- CDNA4 (gfx950) kernels of the simplex pivot engine + the C ABI of smx.h.
//
// Hot path of jqnfxa/Simplex-Method-Solver src/simplex.py, re-designed for MI355X:
//   k_select  : pick_element partials (simplex.py:70-141), one record per workgroup
//   k_finalize: pick_element outcome (simplex.py:89, 91, 101-103, 138-141)
//   k_update  : recalculate_matrix (simplex.py:143-177) fused with the decision (every block
//               reduces the select partials itself: no extra launch, no inter-block protocol)
//               and with the NEXT step's first-negative scans of the "-b" column and f-row
//   k_reset   : first-negative scans of a freshly uploaded tableau (set-up, simplex.py:25-39)
//   k_pack / k_merge / k_update<SHARD> : the row-sharded variant (one rank per GPU)
//
// Arithmetic parity: every element is (t*e - pr*pc)/e with each op rounded on its own, exactly
// as CPython evaluates simplex.py:173-175.  This file is compiled with -ffp-contract=off and
// additionally pins `#pragma clang fp contract(off)`; fp64 division is the IEEE-correct
// div_scale/rcp/fma/div_fmas/div_fixup sequence (never a reciprocal multiply).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include "smx.h"

#pragma clang fp contract(off)

static_assert(sizeof(smx_ctl) == 128, "smx_ctl layout");
static_assert(offsetof(smx_ctl, term) == 16 && offsetof(smx_ctl, npivots) == 40 &&
                  offsetof(smx_ctl, shard_off) == 56 && offsetof(smx_ctl, xpos) == 64 &&
                  offsetof(smx_ctl, npiv) == 80 && offsetof(smx_ctl, dec) == 96,
              "smx_ctl offsets (mirrored in simplex_mi355x/_lib.py)");
static_assert(sizeof(smx_part) == 32, "smx_part layout");

namespace {

constexpr int kWave = 64;
constexpr int kSelBlock = 256;
constexpr int kUpdBlock = 256;
constexpr int kUpdWaves = kUpdBlock / kWave;
constexpr int kMaxParts = 64;

// ---------------------------------------------------------------------------------------------
// Ratio-test candidate order (simplex.py:105-141 restated as an arg-min, see oracle/numpy_oracle):
// class 0: v < 0, larger v better, ties -> larger row; class 1: v == 0 (incl. -0.0), smaller row;
// class 2: v > 0, smaller row; class 3: no candidate.  NaN ratios never enter this order.
struct Cand {
    int cls;
    int idx;
    double v;
};

__device__ __forceinline__ Cand cand_none() { return Cand{3, SMX_NONE, 0.0}; }

__device__ __forceinline__ Cand classify(double v, int idx) {
    Cand c;
    c.cls = (v < 0.0) ? 0 : ((v == 0.0) ? 1 : 2);
    c.idx = idx;
    c.v = v;
    return c;
}

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
    if (a.cls != b.cls) return a.cls < b.cls;
    if (a.cls == 0) return (a.v > b.v) || (a.v == b.v && a.idx > b.idx);
    return a.idx < b.idx;
}

__device__ __forceinline__ Cand shfl_xor_cand(const Cand& a, int mask) {
    Cand o;
    o.cls = __shfl_xor(a.cls, mask, kWave);
    o.idx = __shfl_xor(a.idx, mask, kWave);
    o.v = __shfl_xor(a.v, mask, kWave);
    return o;
}

// "first candidate" = smallest row with T[i][c] != 0, carrying its (possibly NaN) ratio
struct First {
    int idx;
    double v;
};

__device__ __forceinline__ First shfl_xor_first(const First& a, int mask) {
    First o;
    o.idx = __shfl_xor(a.idx, mask, kWave);
    o.v = __shfl_xor(a.v, mask, kWave);
    return o;
}

__device__ __forceinline__ int wave_min_int(int x) {
#pragma unroll
    for (int mask = 32; mask >= 1; mask >>= 1) x = min(x, __shfl_xor(x, mask, kWave));
    return x;
}

__device__ __forceinline__ Cand wave_best(Cand a) {
#pragma unroll
    for (int mask = 32; mask >= 1; mask >>= 1) {
        Cand o = shfl_xor_cand(a, mask);
        if (better(o, a)) a = o;
    }
    return a;
}

__device__ __forceinline__ First wave_first(First a) {
#pragma unroll
    for (int mask = 32; mask >= 1; mask >>= 1) {
        First o = shfl_xor_first(a, mask);
        if (o.idx < a.idx) a = o;
    }
    return a;
}

struct Decision {
    int status;
    int r;
    int c;
};

// The outcome of pick_element from the select partials (run by one wave; lanes cover parts).
// simplex.py:72-91 (phase 1), :94-103 (entering column / optimum), :105-141 (leaving row).
__device__ Decision decide_from_parts(const smx_ctl* ctl, const smx_part* parts, int nparts,
                                      int parity, int n, int m, int flen) {
    const int lane = threadIdx.x & (kWave - 1);
    Decision d;
    const int negb = ctl->negb[parity];
    if (negb != SMX_NONE && negb < n) {
        int p1 = SMX_NONE;
        for (int k = lane; k < nparts; k += kWave) p1 = min(p1, parts[k].p1col);
        p1 = wave_min_int(p1);
        d.r = negb;
        d.c = p1;
        d.status = (p1 == SMX_NONE) ? SMX_INCORRECT : SMX_PIVOT;
        return d;
    }
    const int c = ctl->negf[parity];
    d.c = c;
    d.r = SMX_NONE;
    if (c == SMX_NONE) {
        d.status = (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;
        return d;
    }
    First f{SMX_NONE, 0.0};
    Cand b = cand_none();
    for (int k = lane; k < nparts; k += kWave) {
        const smx_part p = parts[k];
        if (p.first < f.idx) {
            f.idx = p.first;
            f.v = p.first_v;
        }
        Cand o{p.best_cls, p.best_i, p.best_v};
        if (better(o, b)) b = o;
    }
    f = wave_first(f);
    b = wave_best(b);
    if (f.idx == SMX_NONE) {
        d.status = SMX_NOT_CONVERGE;              // first_try still set (simplex.py:138)
    } else if (isnan(f.v)) {
        d.status = SMX_PIVOT;                     // a NaN first candidate sticks (:117-121)
        d.r = f.idx;
    } else if (b.cls >= 2) {
        d.status = SMX_NOT_CONVERGE;              // min_val > 0 (simplex.py:138-139)
    } else {
        d.status = SMX_PIVOT;
        d.r = b.idx;
    }
    return d;
}

// ---------------------------------------------------------------------------------------------
// Every rank merges the P headers identically: phase decision (simplex.py:72-76), global arg-min
// of the ratio test (simplex.py:105-141) and the winning row's offset in recv.  One thread.
struct ShardDecision {
    int status, r, c, owner;
    int64_t off;
};

__device__ ShardDecision merge_headers(const double* __restrict__ recv, int nranks, int64_t ld,
                                       int m, int flen) {
    const int64_t slot = SMX_SHARD_HDR + 2 * ld;
    int gnegb = SMX_NONE, owner_b = -1;
    int gfirst = SMX_NONE, owner_f = -1;
    double fv = 0.0;
    Cand best = cand_none();
    int owner_best = -1;
    int c = SMX_NONE;
    for (int p = 0; p < nranks; ++p) {
        const double* h = recv + p * slot;
        const int nb = (int)h[0];
        if (nb < gnegb) {
            gnegb = nb;
            owner_b = p;
        }
        const int fi = (int)h[1];
        if (fi < gfirst) {
            gfirst = fi;
            fv = h[2];
            owner_f = p;
        }
        Cand o{(int)h[3], (int)h[4], h[5]};
        if (better(o, best)) {
            best = o;
            owner_best = p;
        }
        c = (int)h[6];
    }
    ShardDecision d{SMX_NOT_CONVERGE, SMX_NONE, c, -1, 0};
    if (gnegb != SMX_NONE) {                      // phase 1: the owner scanned its row
        d.r = gnegb;
        d.owner = owner_b;
        d.off = owner_b * slot + SMX_SHARD_HDR + ld;
        d.c = (int)recv[owner_b * slot + 7];
        d.status = (d.c == SMX_NONE) ? SMX_INCORRECT : SMX_PIVOT;
    } else if (c == SMX_NONE) {
        d.status = (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;
    } else if (gfirst == SMX_NONE) {
        d.status = SMX_NOT_CONVERGE;
    } else if (isnan(fv)) {
        d.status = SMX_PIVOT;
        d.r = gfirst;
        d.owner = owner_f;
        d.off = owner_f * slot + SMX_SHARD_HDR;
    } else if (best.cls >= 2) {
        d.status = SMX_NOT_CONVERGE;
    } else {
        d.status = SMX_PIVOT;
        d.r = best.idx;
        d.owner = owner_best;
        d.off = owner_best * slot + SMX_SHARD_HDR + ld;
    }
    return d;
}

// commit = false: record the selection only (smx_shard_merge, like k_finalize); commit = true:
// also count/log the pivot or latch the terminal outcome (the update kernel's block 0).
__device__ void publish_shard_decision(const ShardDecision& d, const double* recv,
                                       smx_ctl* ctl, int32_t* log, int64_t log_cap, bool commit) {
    ctl->sel_status = d.status;
    ctl->sel_r = d.r;
    ctl->sel_c = d.c;
    ctl->sel_owner = d.owner;
    ctl->shard_off = d.off;
    ctl->sel_e = (d.status == SMX_PIVOT) ? recv[d.off + d.c] : 0.0;
    if (!commit) return;
    if (d.status == SMX_PIVOT) {
        const int64_t k = ctl->npivots;   // sharded: only block 0 of the update reads/writes it
        if (log_cap > 0) {
            log[2 * (k % log_cap)] = d.r;
            log[2 * (k % log_cap) + 1] = d.c;
        }
        ctl->npivots = k + 1;
    } else {
        ctl->term = 1;
    }
}

// Every rank merges the P headers identically (one workgroup) and, in phase 1, scans the
// winning row for its first positive entry (simplex.py:81-85).
// ---------------------------------------------------------------------------------------------
// k_reset: scan the "-b" column (rows < rows_local) and the f-row (j < fscan) of a tableau.
__global__ __launch_bounds__(1024) void k_reset(const double* __restrict__ T, int64_t ld,
                                                int rows, int m, int fscan, int row0,
                                                int parity, int clear_count,
                                                smx_ctl* __restrict__ ctl) {
    __shared__ int s_b[16], s_f[16];
    const int tid = threadIdx.x;
    int nb = SMX_NONE, nf = SMX_NONE;
    for (int i = tid; i < rows; i += blockDim.x) {
        if (T[(int64_t)i * ld + m] < 0.0) {
            nb = row0 + i;
            break;
        }
    }
    const double* f = T + (int64_t)rows * ld;
    for (int j = tid; j < fscan; j += blockDim.x) {
        if (f[j] < 0.0) {
            nf = j;
            break;
        }
    }
    nb = wave_min_int(nb);
    nf = wave_min_int(nf);
    if ((tid & 63) == 0) {
        s_b[tid >> 6] = nb;
        s_f[tid >> 6] = nf;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            nb = min(nb, s_b[w]);
            nf = min(nf, s_f[w]);
        }
        ctl->negb[parity] = nb;
        ctl->negf[parity] = nf;
        ctl->negb[parity ^ 1] = SMX_NONE;
        ctl->negf[parity ^ 1] = SMX_NONE;
        ctl->term = 0;
        ctl->nla = 0;
        ctl->sel_status = SMX_IDLE;
        ctl->sel_r = SMX_NONE;
        ctl->sel_c = SMX_NONE;
        if (clear_count) ctl->npivots = 0;
        ctl->npiv[parity] = ctl->npivots;
        ctl->xpos[parity][0] = (m >= 1) ? -1 : SMX_ABSENT;   // 'x1' at column 0
        ctl->xpos[parity][1] = (m >= 2) ? -2 : SMX_ABSENT;   // 'x2' at column 1
    }
}

__global__ void k_set_xpos(smx_ctl* __restrict__ ctl, int parity, int x1, int x2) {
    if (threadIdx.x == 0) {
        ctl->xpos[parity][0] = x1;
        ctl->xpos[parity][1] = x2;
    }
}

// Label movement of one pivot (simplex.py:152): the label at column c and the one at row r swap.
__device__ __forceinline__ int move_label(int code, int r, int c) {
    if (code == -(c + 1)) return r;
    if (code == r) return -(c + 1);
    return code;
}

// ---------------------------------------------------------------------------------------------
// k_select: per-workgroup partials of pick_element.  Phase 1: first positive entry of the
// first-negative-b row, sliced over columns.  Phase 2: first candidate + best non-NaN key of the
// ratio test over the entering column, sliced over rows (two strided loads per row, spread over
// many CUs so the gather is not limited by one CU's fabric bandwidth).
__global__ __launch_bounds__(kSelBlock) void k_select(const double* __restrict__ T, int64_t ld,
                                                      int rows, int m, int row0, int parity,
                                                      smx_ctl* __restrict__ ctl,
                                                      smx_part* __restrict__ parts) {
    __shared__ int s_i[kSelBlock / kWave];
    __shared__ First s_f[kSelBlock / kWave];
    __shared__ Cand s_c[kSelBlock / kWave];
    const int tid = threadIdx.x;
    const int wid = tid >> 6;
    if (ctl->term) return;
    if (blockIdx.x == 0 && tid == 0) {
        // the slot the update of this step fills for the next step (it atomically min-s into it)
        ctl->negb[parity ^ 1] = SMX_NONE;
        ctl->negf[parity ^ 1] = SMX_NONE;
    }
    const int gtid = blockIdx.x * kSelBlock + tid;
    const int gstride = gridDim.x * kSelBlock;
    const int negb = ctl->negb[parity];
    if (negb != SMX_NONE && negb >= row0 && negb < row0 + rows) {
        // phase 1 (simplex.py:81-85): first j < m with T[r][j] > 0
        const double* rowp = T + (int64_t)(negb - row0) * ld;
        int p1 = SMX_NONE;
        for (int j = gtid; j < m; j += gstride) {
            if (rowp[j] > 0.0) {
                p1 = j;
                break;
            }
        }
        p1 = wave_min_int(p1);
        if ((tid & 63) == 0) s_i[wid] = p1;
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < kSelBlock / kWave; ++w) p1 = min(p1, s_i[w]);
            parts[blockIdx.x].p1col = p1;
        }
        return;
    }
    const int c = ctl->negf[parity];
    if (c == SMX_NONE) return;
    // phase 2 ratio test (simplex.py:111-136)
    First f{SMX_NONE, 0.0};
    Cand b = cand_none();
    for (int i = gtid; i < rows; i += gstride) {
        const double* rowp = T + (int64_t)i * ld;
        const double a = rowp[c];
        const double bb = rowp[m];
        if (a != 0.0) {                                  // simplex.py:112 (NaN counts)
            const double v = bb / a;                     // simplex.py:115
            const int gi = row0 + i;
            if (gi < f.idx) {
                f.idx = gi;
                f.v = v;
            }
            if (!isnan(v)) {
                const Cand x = classify(v, gi);
                if (better(x, b)) b = x;
            }
        }
    }
    f = wave_first(f);
    b = wave_best(b);
    if ((tid & 63) == 0) {
        s_f[wid] = f;
        s_c[wid] = b;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kSelBlock / kWave; ++w) {
            if (s_f[w].idx < f.idx) f = s_f[w];
            if (better(s_c[w], b)) b = s_c[w];
        }
        smx_part p;
        p.p1col = SMX_NONE;
        p.first = f.idx;
        p.first_v = f.v;
        p.best_cls = b.cls;
        p.best_i = b.idx;
        p.best_v = b.v;
        parts[blockIdx.x] = p;
    }
}

__global__ __launch_bounds__(kWave) void k_finalize(const smx_part* __restrict__ parts,
                                                    int nparts, int parity, int n, int m,
                                                    int flen, const double* __restrict__ T,
                                                    int64_t ld, smx_ctl* __restrict__ ctl) {
    const Decision d = decide_from_parts(ctl, parts, nparts, parity, n, m, flen);
    if (threadIdx.x == 0) {
        ctl->sel_status = d.status;
        ctl->sel_r = d.r;
        ctl->sel_c = d.c;
        ctl->sel_e = (d.status == SMX_PIVOT) ? T[(int64_t)d.r * ld + d.c] : 0.0;
    }
}

// ---------------------------------------------------------------------------------------------
// Look-ahead selection (fused chain): the whole pick_element of step k+1 (simplex.py:70-141)
// computed by ONE workgroup from T_k and step k's pivot (r, c), while the other workgroups write
// T_{k+1}.  Every entry it needs of T_{k+1} is re-derived with the update's own expression
// (nv below), so the decision is bit-identical to selecting on the materialised T_{k+1}.
__device__ __forceinline__ double nv(const double* __restrict__ T, int64_t ld, int r, int c,
                                     double e, const double* __restrict__ prow, int i, int j,
                                     double pci) {
    const double x = T[(int64_t)i * ld + j];
    double num;
    if (i == r) {
        num = (j == c) ? 1.0 : -x;
    } else {
        const double a = x * e;
        const double b = prow[j] * pci;
        num = (j == c) ? x : (a - b);
    }
    return num / e;
}

template <int NT>
__device__ __forceinline__ int block_min_int(int x, int* s_tmp) {
    x = wave_min_int(x);
    const int wid = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_tmp[wid] = x;
    __syncthreads();
    int r = s_tmp[0];
#pragma unroll
    for (int w = 1; w < NT / kWave; ++w) r = min(r, s_tmp[w]);
    return r;
}

// Fused chain: the select inputs of the NEXT step, computed by nparts workgroups from T_k and
// step k's pivot (APPLY) -- or from T_k itself to prime a chain (!APPLY).  T holds `rows` local
// constraint rows (global index row0 + i) and the f-row at local index `rows`; r_local is the
// pivot row's local index or -1 (sharded: another rank's row, prow then points into the receive
// buffer).  Workgroup b covers local rows b*NT + tid + q*nparts*NT and writes one record:
//   p1col  first row of its slice whose new "-b" entry is negative (simplex.py:72-76), or NONE
//   first/first_v, best_*  its ratio-test candidates on the new entering column (:105-141)
// and workgroup 0 stores the entering column itself (first negative new f-row coefficient,
// simplex.py:94-98) in ctl->negf[slot].  Nothing is min-ed atomically, so no slot needs a reset.
template <int NT, bool APPLY>
__device__ void la_partial(const double* __restrict__ T, int64_t ld, int rows, int m, int fscan,
                           int row0, int r_local, int c, double e,
                           const double* __restrict__ prow, smx_part* __restrict__ out, int b,
                           int nparts, smx_ctl* __restrict__ ctl, int slot) {
    __shared__ int s_tmp[NT / kWave];
    __shared__ int s_b[NT / kWave];
    __shared__ First s_f[NT / kWave];
    __shared__ Cand s_c[NT / kWave];
    const int tid = threadIdx.x;
    auto val = [&](int i, int j, double pci) -> double {
        if (APPLY) return nv(T, ld, r_local, c, e, prow, i, j, pci);
        return T[(int64_t)i * ld + j];
    };
    int nf = SMX_NONE;
    const double pcf = APPLY ? T[(int64_t)rows * ld + c] : 0.0;
    for (int j = tid; j < fscan; j += NT) {
        if (val(rows, j, pcf) < 0.0) {
            nf = j;
            break;
        }
    }
    nf = block_min_int<NT>(nf, s_tmp);
    int nb = SMX_NONE;
    First f{SMX_NONE, 0.0};
    Cand bc = cand_none();
    for (int i = b * NT + tid; i < rows; i += nparts * NT) {
        const int gi = row0 + i;
        const double pci = APPLY ? T[(int64_t)i * ld + c] : 0.0;
        const double bv = val(i, m, pci);
        if (bv < 0.0 && gi < nb) nb = gi;
        if (nf != SMX_NONE) {
            const double a = val(i, nf, pci);
            if (a != 0.0) {
                const double v = bv / a;
                if (gi < f.idx) {
                    f.idx = gi;
                    f.v = v;
                }
                if (!isnan(v)) {
                    const Cand x = classify(v, gi);
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
        out[b] = pt;
        if (b == 0) ctl->negf[slot] = nf;
    }
}

// Fused-chain decision of step k (simplex.py:70-141) from its look-ahead records and T_k: the
// phase-1 row is the minimum of the records' p1col; its first positive entry is scanned by the
// whole block on the materialised T_k (:81-85); phase 2 reduces the ratio partials (:105-141).
// `rec` / `c`: lane k's record (k < nparts <= 64) and the entering column, loaded by wave 0
// before the sweep's prefetch so the decision does not wait behind it.
template <int NT>
__device__ Decision decide_fused(const smx_part& rec, int c, int n, int m, int flen,
                                 const double* __restrict__ T, int64_t ld, int* negb_out) {
    __shared__ int s_tmp[NT / kWave];
    __shared__ Decision s_d;
    __shared__ int s_negb;
    const int tid = threadIdx.x;
    if (tid < kWave) {
        int nb = rec.p1col;
        First f{rec.first, rec.first_v};
        Cand b{rec.best_cls, rec.best_i, rec.best_v};
        nb = wave_min_int(nb);
        Decision d;
        d.c = c;
        d.r = SMX_NONE;
        if (nb == SMX_NONE) {          // phase 2 (the records were built for column c)
            f = wave_first(f);
            b = wave_best(b);
            if (c == SMX_NONE) {
                d.status = (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;
            } else if (f.idx == SMX_NONE) {
                d.status = SMX_NOT_CONVERGE;
            } else if (isnan(f.v)) {
                d.status = SMX_PIVOT;
                d.r = f.idx;
            } else if (b.cls >= 2) {
                d.status = SMX_NOT_CONVERGE;
            } else {
                d.status = SMX_PIVOT;
                d.r = b.idx;
            }
        }
        if (tid == 0) {
            s_negb = nb;
            s_d = d;
        }
    }
    __syncthreads();
    const int negb = s_negb;
    *negb_out = negb;
    if (negb == SMX_NONE) return s_d;
    // phase 1: first positive entry of the first-negative-b row of the materialised T_k
    const double* row = T + (int64_t)negb * ld;
    int p1 = SMX_NONE;
    for (int j = tid; j < m; j += NT) {
        if (row[j] > 0.0) {
            p1 = j;
            break;
        }
    }
    p1 = block_min_int<NT>(p1, s_tmp);
    Decision d;
    d.r = negb;
    d.c = p1;
    d.status = (p1 == SMX_NONE) ? SMX_INCORRECT : SMX_PIVOT;
    return d;
}

// Prime a fused chain: the look-ahead records of step `parity` from T itself.
__global__ __launch_bounds__(kUpdBlock) void k_la_prime(const double* __restrict__ T, int64_t ld,
                                                        int rows, int m, int fscan, int row0,
                                                        int parity, smx_ctl* __restrict__ ctl,
                                                        smx_part* __restrict__ parts) {
    if (ctl->term) return;
    la_partial<kUpdBlock, false>(T, ld, rows, m, fscan, row0, -1, 0, 1.0, T, parts, blockIdx.x,
                                 gridDim.x, ctl, parity);
}

// End of a fused chain: publish the next step's first-negative-b row into ctl->negb[parity]
// (the entering column is already in ctl->negf[parity]) so the unfused calls continue from it.
__global__ __launch_bounds__(kWave) void k_publish(const smx_part* __restrict__ parts, int nparts,
                                                   int parity, smx_ctl* __restrict__ ctl) {
    if (ctl->term) return;
    int nb = SMX_NONE;
    for (int k = threadIdx.x; k < nparts; k += kWave) nb = min(nb, parts[k].p1col);
    nb = wave_min_int(nb);
    if (threadIdx.x == 0) {
        ctl->negb[parity] = nb;
        ctl->negb[parity ^ 1] = SMX_NONE;
        ctl->negf[parity ^ 1] = SMX_NONE;
    }
}

// Header + candidate rows of step k+1 (layout of k_pack) from step k+1's records (`parts`, slot
// `slot`, nparts of them) and T_k with step k's pivot (r_local, c, e, prow): every value is
// nv(T_k, pivot k), i.e. exactly T_{k+1}.  Workgroup bidx of nblk; all threads of the group call.
__device__ void pack_ahead(const double* __restrict__ T, int64_t ld, int rows, int m, int row0,
                           int r_local, int c, double e, const double* __restrict__ prow,
                           const smx_ctl* __restrict__ ctl, const smx_part* __restrict__ parts,
                           int nparts, int slot, double* __restrict__ send, int bidx, int nblk) {
    __shared__ int s_rows[2];
    __shared__ int s_hdr_i[4];
    __shared__ double s_hdr_d[2];
    __shared__ int s_tmp[kUpdBlock / kWave];
    const int tid = threadIdx.x;
    const int cn = ctl->negf[slot];   // step k+1's entering column (look-ahead workgroup 0)
    if (tid < kWave) {
        int nb = SMX_NONE;
        First f{SMX_NONE, 0.0};
        Cand b = cand_none();
        for (int k = tid; k < nparts; k += kWave) {
            const smx_part p = parts[k];
            nb = min(nb, p.p1col);
            if (p.first < f.idx) {
                f.idx = p.first;
                f.v = p.first_v;
            }
            Cand o{p.best_cls, p.best_i, p.best_v};
            if (better(o, b)) b = o;
        }
        nb = wave_min_int(nb);
        f = wave_first(f);
        b = wave_best(b);
        if (nb != SMX_NONE || cn == SMX_NONE) {   // phase 1 / no entering column: no ratio test
            f = First{SMX_NONE, 0.0};
            b = cand_none();
        }
        if (tid == 0) {
            s_rows[0] = (f.idx != SMX_NONE && isnan(f.v)) ? f.idx - row0 : -1;     // row A
            s_rows[1] = (nb != SMX_NONE) ? nb - row0 : (b.cls < 3 ? b.idx - row0 : -1);
            s_hdr_i[0] = nb;
            s_hdr_i[1] = f.idx;
            s_hdr_i[2] = b.cls;
            s_hdr_i[3] = b.idx;
            s_hdr_d[0] = f.v;
            s_hdr_d[1] = b.v;
        }
    }
    __syncthreads();
    const int ra = s_rows[0], rb = s_rows[1];
    const int nb = s_hdr_i[0];
    if (bidx == 0) {
        int p1 = SMX_NONE;   // phase 1 (simplex.py:81-85) on the new values of the owner's row
        if (nb != SMX_NONE) {
            const int il = nb - row0;
            const double pci = T[(int64_t)il * ld + c];
            for (int j = tid; j < m; j += kUpdBlock) {
                if (nv(T, ld, r_local, c, e, prow, il, j, pci) > 0.0) {
                    p1 = j;
                    break;
                }
            }
            p1 = block_min_int<kUpdBlock>(p1, s_tmp);
        }
        if (tid == 0) {
            send[0] = (double)nb;
            send[1] = (double)s_hdr_i[1];
            send[2] = s_hdr_d[0];
            send[3] = (double)s_hdr_i[2];
            send[4] = (double)s_hdr_i[3];
            send[5] = s_hdr_d[1];
            send[6] = (double)cn;
            send[7] = (double)p1;
        }
    }
    const int C = m + 1;
    const double pca = ra >= 0 ? T[(int64_t)ra * ld + c] : 0.0;
    const double pcb = rb >= 0 ? T[(int64_t)rb * ld + c] : 0.0;
    for (int j = bidx * kUpdBlock + tid; j < C; j += nblk * kUpdBlock) {
        if (ra >= 0) send[SMX_SHARD_HDR + j] = nv(T, ld, r_local, c, e, prow, ra, j, pca);
        if (rb >= 0) send[SMX_SHARD_HDR + ld + j] = nv(T, ld, r_local, c, e, prow, rb, j, pcb);
    }
}

// ---------------------------------------------------------------------------------------------
// k_update: the modified Jordan step (simplex.py:149-177), out of place.
//
// Streaming shape (measured on MI355X with tools/hbm_probe.hip: a grid-wide sweep in address
// order, where every resident wave works inside one narrow moving window of the tableau, streams
// faster than per-wave private regions).  A unit is one row x one chunk of 64 lanes x 2 doubles
// (1 KiB); unit u = row * nchunks + chunk; wave w takes units w, w + NW, w + 2 NW, ... in
// batches of U (U 16-B loads in flight per lane before any arithmetic).  When NW is a multiple
// of nchunks a wave always sees the same chunk, so its pivot-row slice stays in registers.
// T[i][c] is a wave-uniform scalar load per unit.  Per element:
//     num = (i == r) ? (j == c ? 1.0 : -x)          steps 1 and 3
//                    : (j == c ? x   : x*e - pr*pc) steps 2 and 4
//     out = num / e
// which is exactly the value the reference leaves in new_table[i][j] after steps 1-4.
//
// Modes: kSingle (decision from k_select's partials), kShard (decision merged from the gathered
// shard headers, nparts = rank count), kForced (given r, c), kFused / kShardFused (as kSingle /
// kShard, plus look-ahead workgroups [0, nparts) writing the next step's records; in these modes
// forced_r = 1 when the look-ahead workgroups also sweep, and kShardFused's rank count is
// forced_c).
enum UpdMode { kSingle = 0, kShard = 1, kForced = 2, kFused = 3, kShardFused = 4 };

#ifdef SMX_TRACE
// Diagnostic build only (tools/trace_fused.hip): per-workgroup s_memrealtime stamps (100 MHz,
// chip-wide) of the last two update launches, [launch parity][block][phase]:
// 0 entry, 1 decision known, 2 look-ahead records written, 3 sweep done.
constexpr int kTraceBlocks = 4096;
__device__ unsigned long long g_trace[2][kTraceBlocks][4];
#define SMX_STAMP(ph)                                                                  \
    do {                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < kTraceBlocks)                             \
            g_trace[parity & 1][blockIdx.x][ph] = __builtin_amdgcn_s_memrealtime();    \
    } while (0)
#else
#define SMX_STAMP(ph) \
    do {              \
    } while (0)
#endif

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NTL>
__device__ __forceinline__ dbl2 ld2(const double* p) {
    if (NTL) return __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(p));
    return *reinterpret_cast<const dbl2*>(p);
}

// One batch = U units of this wave: their rows, chunks and the 16-B tableau slices.
template <int U>
struct Batch {
    int i[U], ch[U];
    dbl2 x[U];
    double pc[U];
};

// DIAG (timing only, never selectable in normal use): multiply by 1/e instead of dividing.
template <int MODE, int U, bool NTS, bool NTL, bool PIPE, bool DIAG = false>
__global__ __launch_bounds__(kUpdBlock) void k_update(
    const double* __restrict__ Tin, double* __restrict__ Tout, int64_t ld, int rows_local,
    int n, int m, int flen, int fscan, int row0, int parity, smx_ctl* __restrict__ ctl,
    const smx_part* __restrict__ parts, int nparts, int32_t* __restrict__ log,
    double* __restrict__ xhist, int64_t log_cap, const double* __restrict__ recv, int forced_r,
    int forced_c, double* __restrict__ send) {
    __shared__ int s_dec[3];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    if (MODE != kForced && ctl->term) return;
    SMX_STAMP(0);
    const int R = rows_local + 1;  // + the f-row (local row rows_local)
    const int C = m + 1;
    constexpr int kChunk = kWave * 2;                  // doubles per unit
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int64_t units = (int64_t)nchunks * R;
    // kFused: workgroups [0, nparts) compute the look-ahead records; they join the sweep only
    // when forced_r (= "look-ahead sweeps") is set: tableaux beyond the Infinity Cache, whose
    // stream needs every resident wave's loads in flight (launch_update_mode)
    constexpr bool LA = MODE == kFused || MODE == kShardFused;
    const bool la_sweep = LA && forced_r != 0;
    const int lab = (LA && !la_sweep) ? nparts : 0;
    const bool la = LA && (int)blockIdx.x < nparts;
    const bool sweeps = !la || la_sweep;
    const int NW = ((int)gridDim.x - lab) * kUpdWaves;
    const int w = sweeps ? ((int)blockIdx.x - lab) * kUpdWaves +
                               __builtin_amdgcn_readfirstlane(tid >> 6)
                         : 0;
    // unit u = i * nchunks + ch; advancing u by NW advances (i, ch) by (qs, rs)
    const int qs = NW / nchunks, rs = NW % nchunks;
    int i_cur = w / nchunks, ch_cur = w % nchunks;

    // address part of a batch: independent of the pivot, so the first batch's loads are in
    // flight while the selection decision below is still being reduced
    auto fetch = [&](Batch<U>& b) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            b.i[k] = i_cur;
            b.ch[k] = ch_cur;
            ch_cur += rs;
            i_cur += qs;
            if (ch_cur >= nchunks) {
                ch_cur -= nchunks;
                ++i_cur;
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            b.x[k] = dbl2{0.0, 0.0};
            const int j = b.ch[k] * kChunk + 2 * lane;
            if (b.i[k] < R && j < C) b.x[k] = ld2<NTL>(Tin + (int64_t)b.i[k] * ld + j);
        }
    };
    smx_part rec{SMX_NONE, SMX_NONE, 0.0, 3, SMX_NONE, 0.0};
    int negf0 = SMX_NONE;
    if (MODE == kFused && tid < kWave) {   // the decision's loads first (in-order vmcnt)
        if (tid < nparts) rec = parts[(size_t)parity * nparts + tid];
        negf0 = ctl->negf[parity];
    }
    Batch<U> cur;
    if (sweeps) fetch(cur);

    int r, c;
    const double* prow;
    if (MODE == kForced) {
        r = forced_r;
        c = forced_c;
        prow = Tin + (int64_t)r * ld;
    } else if (MODE == kSingle || MODE == kFused) {
        Decision dd;
        int negb_f = SMX_NONE;
        if (MODE == kFused)   // whole block (phase-1 row scan); parts = this step's slot
            dd = decide_fused<kUpdBlock>(rec, negf0, n, m, flen, Tin, ld, &negb_f);
        if (tid < kWave) {
            Decision d;
            if (MODE == kFused)
                d = dd;
            else
                d = decide_from_parts(ctl, parts, nparts, parity, n, m, flen);
            if (tid == 0) {
                s_dec[0] = d.status;
                s_dec[1] = d.r;
                s_dec[2] = d.c;
                if (blockIdx.x == 0) {
                    if (MODE == kFused) ctl->negb[parity] = negb_f;   // host-visible state
                    ctl->sel_status = d.status;
                    ctl->sel_r = d.r;
                    ctl->sel_c = d.c;
                    if (d.status == SMX_PIVOT) {
                        ctl->sel_e = Tin[(int64_t)d.r * ld + d.c];
                        const int64_t k = ctl->npiv[parity];
                        if (log_cap > 0) {
                            log[2 * (k % log_cap)] = d.r;
                            log[2 * (k % log_cap) + 1] = d.c;
                        }
                        ctl->npivots = k + 1;
                        ctl->npiv[parity ^ 1] = k + 1;
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int code = move_label(ctl->xpos[parity][q], d.r, d.c);
                            ctl->xpos[parity ^ 1][q] = code;
                            if (xhist && log_cap > 0 && code < 0)   // non-basic: value 0
                                xhist[2 * (k % log_cap) + q] = 0.0;
                        }
                    } else {
                        ctl->term = 1;
                    }
                }
            }
        }
        __syncthreads();
        if (s_dec[0] != SMX_PIVOT) return;
        r = __builtin_amdgcn_readfirstlane(s_dec[1]);
        c = __builtin_amdgcn_readfirstlane(s_dec[2]);
        prow = Tin + (int64_t)r * ld;
    } else {  // kShard(Fused): every block merges the P gathered headers itself
        __shared__ int64_t s_off;
        if (tid == 0) {
            const int nranks = (MODE == kShardFused) ? forced_c : nparts;
            const ShardDecision d = merge_headers(recv, nranks, ld, m, flen);
            s_dec[0] = d.status;
            s_dec[1] = d.r;
            s_dec[2] = d.c;
            s_off = d.off;
            if (blockIdx.x == 0) publish_shard_decision(d, recv, ctl, log, log_cap, true);
        }
        __syncthreads();
        if (s_dec[0] != SMX_PIVOT) return;
        r = __builtin_amdgcn_readfirstlane(s_dec[1]);
        c = __builtin_amdgcn_readfirstlane(s_dec[2]);
        prow = recv + s_off;
    }
    const double e = prow[c];
    SMX_STAMP(1);
    // history: rows whose new "-b" entry is x1 / x2 of the new tableau (find_optimum)
    int hx0 = -1, hx1 = -1;
    int64_t hslot = 0;
    if ((MODE == kSingle || MODE == kFused) && xhist != nullptr && log_cap > 0) {
        hx0 = move_label(ctl->xpos[parity][0], r, c);
        hx1 = move_label(ctl->xpos[parity][1], r, c);
        hslot = 2 * (ctl->npiv[parity] % log_cap);
    }
    // local index of the pivot row, -1 when another rank owns it (never the f-row replica,
    // whose local index rows_local may equal r - row0 for a row of the next rank)
    const int r_local = (r >= row0 && r < row0 + rows_local) ? r - row0 : -1;
    if (LA && la) {
        // this workgroup's share of step k+1's select inputs (one kernel per pivot)
        la_partial<kUpdBlock, true>(Tin, ld, rows_local, m, fscan, row0, r_local, c, e, prow,
                                    const_cast<smx_part*>(parts) + (size_t)(parity ^ 1) * nparts,
                                    blockIdx.x, nparts, ctl, parity ^ 1);
        if (MODE == kShardFused && send != nullptr) {
            // The last look-ahead workgroup to finish packs step k+1's header and candidate
            // rows into the send slot (values of T_{k+1} via nv), so a sharded pivot is this
            // kernel + the all-gather.  nparts counter atomics, not one per workgroup.
            __shared__ int s_last;
            __syncthreads();
            if (tid == 0) {
                __threadfence();   // release this workgroup's record (and negf from group 0)
                s_last = atomicAdd(&ctl->nla, 1) == nparts - 1;
            }
            __syncthreads();
            if (s_last) {
                __threadfence();   // acquire the other workgroups' records
                pack_ahead(Tin, ld, rows_local, m, row0, r_local, c, e, prow, ctl,
                           parts + (size_t)(parity ^ 1) * nparts, nparts, parity ^ 1, send, 0, 1);
                if (tid == 0) ctl->nla = 0;
            }
        }
        SMX_STAMP(2);
        if (!la_sweep) return;
    }
    int ch_pr = -1;
    dbl2 pr = dbl2{0.0, 0.0};
    const int negslot = parity ^ 1;
    int lb = SMX_NONE;   // fused next-step scan: first row with new b < 0 (this lane)
    int lf = SMX_NONE;   // fused next-step scan: first f-row column with new f < 0 (this lane)

    for (int64_t u = w; u < units; u += (int64_t)U * NW) {
#pragma unroll
        for (int k = 0; k < U; ++k)
            cur.pc[k] = (cur.i[k] < R) ? Tin[(int64_t)cur.i[k] * ld + c] : 0.0;
        Batch<U> nxt;
        if (PIPE && u + (int64_t)U * NW < units) fetch(nxt);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int i = cur.i[k];
            if (i >= R) continue;
            const int j = cur.ch[k] * kChunk + 2 * lane;
            if (cur.ch[k] != ch_pr) {
                ch_pr = cur.ch[k];
                pr = (j < C) ? *reinterpret_cast<const dbl2*>(prow + j) : dbl2{0.0, 0.0};
            }
            dbl2 o;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int jj = j + h;
                const double xv = cur.x[k][h];
                double num;
                if (i == r_local) {
                    num = (jj == c) ? 1.0 : -xv;
                } else {
                    const double a = xv * e;
                    const double b = pr[h] * cur.pc[k];
                    num = (jj == c) ? xv : (a - b);
                }
                if (DIAG)
                    o[h] = num * (1.0 / e);
                else
                    o[h] = num / e;
                if (MODE != kForced && jj < C) {
                    if ((MODE == kSingle || MODE == kFused) && jj == m) {
                        if (i == hx0) xhist[hslot] = o[h];
                        if (i == hx1) xhist[hslot + 1] = o[h];
                    }
                    if (LA) {
                        // next-step scans come from the look-ahead records
                    } else if (i < rows_local) {
                        if (jj == m && o[h] < 0.0) lb = min(lb, row0 + i);
                    } else if (jj < fscan && o[h] < 0.0) {
                        lf = min(lf, jj);
                    }
                }
            }
            if (j < C) {
                double* dst = Tout + (int64_t)i * ld + j;
                if (NTS)
                    __builtin_nontemporal_store(o, reinterpret_cast<dbl2*>(dst));
                else
                    *reinterpret_cast<dbl2*>(dst) = o;
            }
        }
        if (PIPE) {
            cur = nxt;
        } else if (u + (int64_t)U * NW < units) {
            fetch(cur);
        }
    }
    SMX_STAMP(3);
    if (MODE == kSingle || MODE == kShard) {
        lb = wave_min_int(lb);
        lf = wave_min_int(lf);
        if (lane == 0) {
            if (lb != SMX_NONE) atomicMin(&ctl->negb[negslot], lb);
            if (lf != SMX_NONE) atomicMin(&ctl->negf[negslot], lf);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Sharded exchange.  Send slot layout (doubles): [hdr SMX_SHARD_HDR][row A: ld][row B: ld]
//   hdr[0] local first-negative-b row (global) or NONE      -> row B = that row (phase 1)
//   hdr[1] first ratio candidate row (global) or NONE        -> row A = that row if its v is NaN
//   hdr[2] its ratio v
//   hdr[3] best class, hdr[4] best row (global), hdr[5] best v -> row B = best row (phase 2)
//   hdr[6] entering column c (replicated f-row => same on every rank)
//   hdr[7] phase 1: first column j < m with row B [j] > 0 (computed by the row's owner), or NONE
// FUSED: `parts` are the look-ahead records of this step (p1col = local first-negative-b row,
// global index); the rank owning that row scans it for the phase-1 column in block 0.
template <bool FUSED>
__global__ __launch_bounds__(kUpdBlock) void k_pack(const double* __restrict__ T, int64_t ld,
                                                     int rows, int m, int row0, int parity,
                                                     const smx_ctl* __restrict__ ctl,
                                                     const smx_part* __restrict__ parts,
                                                     int nparts, double* __restrict__ send) {
    __shared__ int s_rows[2];
    __shared__ int s_hdr_i[4];
    __shared__ double s_hdr_d[2];
    __shared__ int s_negb;
    __shared__ int s_tmp[kUpdBlock / kWave];
    const int tid = threadIdx.x;
    if (ctl->term) return;
    int p1f = SMX_NONE;
    if (FUSED) {
        if (tid < kWave) {
            int nb = SMX_NONE;
            for (int k = tid; k < nparts; k += kWave) nb = min(nb, parts[k].p1col);
            nb = wave_min_int(nb);
            if (tid == 0) s_negb = nb;
        }
        __syncthreads();
        const int nb = s_negb;
        if (blockIdx.x == 0 && nb != SMX_NONE) {   // simplex.py:81-85 on the owner's row
            const double* rowp = T + (int64_t)(nb - row0) * ld;
            for (int j = tid; j < m; j += kUpdBlock) {
                if (rowp[j] > 0.0) {
                    p1f = j;
                    break;
                }
            }
            p1f = block_min_int<kUpdBlock>(p1f, s_tmp);
        }
    }
    if (tid < kWave) {
        const int negb = FUSED ? s_negb : ctl->negb[parity];
        const int c = ctl->negf[parity];
        First f{SMX_NONE, 0.0};
        Cand b = cand_none();
        int p1 = SMX_NONE;   // phase 1: first column with T[negb][j] > 0 (simplex.py:81-85)
        if (FUSED) {
            p1 = p1f;
        } else if (negb != SMX_NONE) {
            for (int k = tid; k < nparts; k += kWave) p1 = min(p1, parts[k].p1col);
            p1 = wave_min_int(p1);
        }
        if (negb == SMX_NONE && c != SMX_NONE) {
            for (int k = tid; k < nparts; k += kWave) {
                const smx_part p = parts[k];
                if (p.first < f.idx) {
                    f.idx = p.first;
                    f.v = p.first_v;
                }
                Cand o{p.best_cls, p.best_i, p.best_v};
                if (better(o, b)) b = o;
            }
            f = wave_first(f);
            b = wave_best(b);
        }
        if (tid == 0) {
            s_rows[0] = (f.idx != SMX_NONE && isnan(f.v)) ? f.idx - row0 : -1;     // row A
            s_rows[1] = (negb != SMX_NONE) ? negb - row0 : (b.cls < 3 ? b.idx - row0 : -1);
            s_hdr_i[0] = negb;
            s_hdr_i[1] = f.idx;
            s_hdr_i[2] = b.cls;
            s_hdr_i[3] = b.idx;
            s_hdr_d[0] = f.v;
            s_hdr_d[1] = b.v;
            if (blockIdx.x == 0) {
                send[0] = (double)negb;
                send[1] = (double)f.idx;
                send[2] = f.v;
                send[3] = (double)b.cls;
                send[4] = (double)b.idx;
                send[5] = b.v;
                send[6] = (double)c;
                send[7] = (double)p1;
            }
        }
    }
    __syncthreads();
    const int ra = s_rows[0], rb = s_rows[1];
    const int C = m + 1;
    const int gt = blockIdx.x * kUpdBlock + tid;
    const int gs = gridDim.x * kUpdBlock;
    for (int j = gt; j < C + 1 && j < ld; j += gs) {
        if (ra >= 0) send[SMX_SHARD_HDR + j] = T[(int64_t)ra * ld + j];
        if (rb >= 0) send[SMX_SHARD_HDR + ld + j] = T[(int64_t)rb * ld + j];
    }
}

__global__ __launch_bounds__(kWave) void k_merge(const double* __restrict__ recv, int nranks,
                                                 int64_t ld, int n, int m, int flen,
                                                 smx_ctl* __restrict__ ctl,
                                                 int32_t* __restrict__ log, int64_t log_cap) {
    (void)n;
    if (ctl->term || threadIdx.x != 0) return;
    const ShardDecision d = merge_headers(recv, nranks, ld, m, flen);
    publish_shard_decision(d, recv, ctl, log, log_cap, false);
}


// ---------------------------------------------------------------------------------------------
// Overlapped sharded chain (smx_shard_run with the fused chain on): while k_update<kShardFused>
// sweeps T_k -> T_{k+1} on the solver stream, the exchange stream computes step k+1's records
// (k_shard_la) and header + candidate rows (k_pack_ahead) from T_k and step k's gathered pivot
// row with the update's own expression (nv), then all-gathers them -- so the collective runs
// under the sweep.  Both kernels re-derive step k's decision from the gathered headers
// (merge_headers is a pure function of recv) and do nothing when it is terminal.
__device__ __forceinline__ bool merged_pivot(const double* __restrict__ recv, int nranks,
                                             int64_t ld, int m, int flen, int* s_dec,
                                             int64_t* s_off) {
    if (threadIdx.x == 0) {
        const ShardDecision d = merge_headers(recv, nranks, ld, m, flen);
        s_dec[0] = d.status;
        s_dec[1] = d.r;
        s_dec[2] = d.c;
        *s_off = d.off;
    }
    __syncthreads();
    return s_dec[0] == SMX_PIVOT;
}

__global__ __launch_bounds__(kUpdBlock) void k_shard_la(const double* __restrict__ T, int64_t ld,
                                                        int rows, int m, int flen, int fscan,
                                                        int row0, const double* __restrict__ recv,
                                                        int nranks, smx_ctl* __restrict__ ctl,
                                                        smx_part* __restrict__ out, int slot) {
    __shared__ int s_dec[3];
    __shared__ int64_t s_off;
    if (ctl->term) return;
    if (!merged_pivot(recv, nranks, ld, m, flen, s_dec, &s_off)) return;
    const int r = s_dec[1], c = s_dec[2];
    const double* prow = recv + s_off;
    const int r_local = (r >= row0 && r < row0 + rows) ? r - row0 : -1;
    la_partial<kUpdBlock, true>(T, ld, rows, m, fscan, row0, r_local, c, prow[c], prow, out,
                                blockIdx.x, gridDim.x, ctl, slot);
}

__global__ __launch_bounds__(kUpdBlock) void k_pack_ahead(
    const double* __restrict__ T, int64_t ld, int rows, int m, int flen, int row0,
    const double* __restrict__ recv, int nranks, const smx_ctl* __restrict__ ctl,
    const smx_part* __restrict__ parts, int nparts, int slot, double* __restrict__ send) {
    __shared__ int s_dec[3];
    __shared__ int64_t s_off;
    if (ctl->term) return;
    if (!merged_pivot(recv, nranks, ld, m, flen, s_dec, &s_off)) return;
    const int r = s_dec[1], c = s_dec[2];
    const double* prow = recv + s_off;
    const int r_local = (r >= row0 && r < row0 + rows) ? r - row0 : -1;
    pack_ahead(T, ld, rows, m, row0, r_local, c, prow[c], prow, ctl, parts, nparts, slot, send,
               blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------------------------
// k_copy: the box's streaming read+write ceiling, measured next to the update in bench.py
// (the best shapes of tools/hbm_probe.hip: a grid-stride copy with U 16-B loads per lane).
template <int U>
__global__ void k_copy(const dbl2* __restrict__ a, dbl2* __restrict__ b, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t st = (int64_t)gridDim.x * blockDim.x;
    for (; i + (U - 1) * st < n; i += U * st) {
        dbl2 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = a[i + k * st];
#pragma unroll
        for (int k = 0; k < U; ++k) b[i + k * st] = v[k];
    }
    for (; i < n; i += st) b[i] = a[i];
}

// ---------------------------------------------------------------------------------------------
// k_batch: many small LPs, one wavefront each (the UI's workload, m = 2,
// n = 3..20, main.py:309-313).  Lane i holds row i of its LP in registers (rows 0..n, the
// f-row is lane n), so the whole get_solution loop (simplex.py:184-198) runs inside one launch:
// phase 1 by a ballot (simplex.py:72-76), the pivot row and the f-row by shuffles
// (:81-85, :94-98), the ratio test by the same wave arg-min as k_select (:105-141), and every
// element with the same (t*e - pr*pc)/e as k_update (:155-175).  Per step: (r, c), (x1, x2) of
// the new table (find_optimum, :51-68) and optionally the table itself (the Info snapshots).
template <int CMAX>
__device__ __forceinline__ double pick(const double (&x)[CMAX], int j) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < CMAX; ++q) v = (q == j) ? x[q] : v;
    return v;
}

template <int CMAX>
__global__ __launch_bounds__(256) void k_batch(
    const double* __restrict__ tabs, const int32_t* __restrict__ dims, int B, int Rmax, int ldb,
    int max_pivots, double* __restrict__ out, int32_t* __restrict__ rc,
    double* __restrict__ xv, double* __restrict__ snaps, int32_t* __restrict__ status_out,
    int32_t* __restrict__ np_out) {
    const int lane = threadIdx.x & (kWave - 1);
    const int b = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6);
    if (b >= B) return;
    const int n = dims[3 * b], m = dims[3 * b + 1], flen = dims[3 * b + 2];
    const int C = m + 1;
    const int fscan = flen < m ? flen : m;
    const bool valid = lane <= n;
    const size_t tab_elems = (size_t)Rmax * ldb;
    const double* src = tabs + (size_t)b * tab_elems + (size_t)lane * ldb;
    double x[CMAX];
#pragma unroll
    for (int q = 0; q < CMAX; ++q) x[q] = (valid && q < C) ? src[q] : 0.0;
    int p1 = (m >= 1) ? -1 : SMX_ABSENT;   // label positions of 'x1', 'x2' (simplex.py:30)
    int p2 = (m >= 2) ? -2 : SMX_ABSENT;
    int status = SMX_PIVOT;
    int np = 0;
    for (int step = 0; step < max_pivots; ++step) {
        const double bval = pick<CMAX>(x, m);
        const unsigned long long neg = __ballot(lane < n && bval < 0.0);
        int r = SMX_NONE, c = SMX_NONE;
        if (neg) {                                           // phase 1 (simplex.py:72-91)
            r = __ffsll((long long)neg) - 1;
#pragma unroll
            for (int q = 0; q < CMAX; ++q) {
                const double v = __shfl(x[q], r, kWave);
                if (q < m && c == SMX_NONE && v > 0.0) c = q;
            }
            if (c == SMX_NONE) {
                status = SMX_INCORRECT;
                break;
            }
        } else {
#pragma unroll
            for (int q = 0; q < CMAX; ++q) {                 // simplex.py:94-98
                const double v = __shfl(x[q], n, kWave);
                if (q < fscan && c == SMX_NONE && v < 0.0) c = q;
            }
            if (c == SMX_NONE) {
                status = (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;
                break;
            }
            const double a = pick<CMAX>(x, c);               // simplex.py:111-136
            First f{SMX_NONE, 0.0};
            Cand bc = cand_none();
            if (lane < n && a != 0.0) {
                const double v = bval / a;
                f.idx = lane;
                f.v = v;
                if (!isnan(v)) bc = classify(v, lane);
            }
            f = wave_first(f);
            bc = wave_best(bc);
            if (f.idx == SMX_NONE) {
                status = SMX_NOT_CONVERGE;
                break;
            }
            if (isnan(f.v)) {
                r = f.idx;
            } else if (bc.cls >= 2) {
                status = SMX_NOT_CONVERGE;
                break;
            } else {
                r = bc.idx;
            }
        }
        // the Jordan step (simplex.py:149-177); every right-hand side is the OLD table
        const double pc = pick<CMAX>(x, c);
        const double e = __shfl(pc, r, kWave);
#pragma unroll
        for (int q = 0; q < CMAX; ++q) {
            const double pr = __shfl(x[q], r, kWave);
            double num;
            if (lane == r) {
                num = (q == c) ? 1.0 : -x[q];
            } else {
                const double t1 = x[q] * e;
                const double t2 = pr * pc;
                num = (q == c) ? x[q] : (t1 - t2);
            }
            x[q] = num / e;
        }
        p1 = move_label(p1, r, c);
        p2 = move_label(p2, r, c);
        const double bnew = pick<CMAX>(x, m);
        const double x1 = (p1 >= 0) ? __shfl(bnew, p1, kWave) : 0.0;
        const double x2 = (p2 >= 0) ? __shfl(bnew, p2, kWave) : 0.0;
        const size_t hs = (size_t)b * max_pivots + step;
        if (lane == 0) {
            rc[2 * hs] = r;
            rc[2 * hs + 1] = c;
            xv[2 * hs] = x1;
            xv[2 * hs + 1] = x2;
        }
        if (snaps && valid) {
            double* dst = snaps + hs * tab_elems + (size_t)lane * ldb;
#pragma unroll
            for (int q = 0; q < CMAX; ++q)
                if (q < C) dst[q] = x[q];
        }
        ++np;
    }
    if (valid) {
        double* dst = out + (size_t)b * tab_elems + (size_t)lane * ldb;
#pragma unroll
        for (int q = 0; q < CMAX; ++q)
            if (q < C) dst[q] = x[q];
    }
    if (lane == 0) {
        status_out[b] = status;
        np_out[b] = np;
    }
}
// ---------------------------------------------------------------------------------------------
inline int nparts_for(int rows, int m) {
    const int work = rows > m ? rows : m;
    int p = (work + kSelBlock - 1) / kSelBlock;
    if (p < 1) p = 1;
    if (p > kMaxParts) p = kMaxParts;
    return p;
}

inline int fscan_of(const smx_shape& s) { return s.flen < s.m ? s.flen : s.m; }

inline bool shape_ok(const smx_shape* s) {
    if (!s) return false;
    if (s->m < 0 || s->rows < 0 || s->n < s->rows || s->ld < s->m + 1) return false;
    if ((s->ld & 1) != 0) return false;                   // 16-B aligned double2 rows
    if (((s->m + 1) & 1) && s->ld < s->m + 2) return false;  // odd C: vector tail in padding
    if ((s->m + 1) > 2 && (s->ld & 3) != 0) return false;    // VEC = 4 variants: 32-B lanes
    if (s->nparts < 1 || s->nparts > kMaxParts) return false;
    return true;
}

inline hipStream_t S(void* p) { return reinterpret_cast<hipStream_t>(p); }

int launch_select(const double* T, const smx_shape& s, int parity, smx_ctl* ctl, smx_part* parts,
                  hipStream_t st) {
    hipLaunchKernelGGL(k_select, dim3(s.nparts), dim3(kSelBlock), 0, st, T, s.ld, s.rows, s.m,
                       s.row0, parity, ctl, parts);
    return (int)hipGetLastError();
}

template <bool FUSED>
int launch_pack(const double* T, const smx_shape& s, int parity, const smx_ctl* ctl,
                const smx_part* parts, double* send, hipStream_t st) {
    int blocks = (int)((s.m + 2 + kUpdBlock - 1) / kUpdBlock);
    if (blocks > 64) blocks = 64;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_pack<FUSED>, dim3(blocks), dim3(kUpdBlock), 0, st, T, s.ld, s.rows, s.m,
                       s.row0, parity, ctl, parts, s.nparts, send);
    return (int)hipGetLastError();
}

// Fused chain helpers: prime the look-ahead records of step `parity` from T; publish at the end.
int launch_prime(const double* T, const smx_shape& s, int parity, smx_ctl* ctl, smx_part* parts,
                 hipStream_t st) {
    const int fscan = s.flen < s.m ? s.flen : s.m;
    hipLaunchKernelGGL(k_la_prime, dim3(s.nparts), dim3(kUpdBlock), 0, st, T, s.ld, s.rows, s.m,
                       fscan, s.row0, parity, ctl, parts + (size_t)parity * s.nparts);
    return (int)hipGetLastError();
}

int launch_publish(const smx_shape& s, int parity, smx_ctl* ctl, const smx_part* parts,
                   hipStream_t st) {
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(kWave), 0, st, parts + (size_t)parity * s.nparts,
                       s.nparts, parity, ctl);
    return (int)hipGetLastError();
}

// ---- update-kernel variants (rows per unit TR, doubles per lane VEC, non-temporal stores) -----
struct UpdVariant {
    int u, nts, ntl, pipe;
};
constexpr UpdVariant kVariants[] = {{2, 1, 0, 0}, {2, 1, 1, 0}, {2, 1, 0, 1}, {2, 1, 1, 1},
                                    {1, 1, 0, 1}, {1, 1, 1, 1}, {4, 1, 0, 0}, {4, 1, 0, 1},
                                    {2, 0, 0, 0}, {1, 1, 0, 0},
                                    // diagnostics (reciprocal multiply: timing only)
                                    {2, 1, 1, 0}, {1, 1, 1, 1}};
constexpr int kFirstDiagVariant = 10;
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
// Defaults from tools/tune_update.py on MI355X at 16384^2 (profiles/r01_tune_sweep*.jsonl).
// Variant -1 = automatic: U=2 with non-temporal stores and loads (1) for tableaux that stream
// from HBM; plain loads (0) when one buffer is at most kCacheTable bytes, where the ping-pong
// pair stays in the 256 MB Infinity Cache and a non-temporal load only adds latency
// (profiles/r01_sweep_small.jsonl: 1024^2 11.1 vs 13.1 us per fused pivot; from 2048^2 on the
// non-temporal variant is as fast or faster).
int g_variant = -1;       // smx_tune_set overrides
constexpr int kLargeVariant = 1, kSmallVariant = 0;
constexpr int64_t kCacheTable = 16ll << 20;
constexpr int64_t kLaSweepTable = 256ll << 20;
// Sharded fused update: its last look-ahead workgroup packs the next step (one workgroup reading
// two rows) only when the local sweep is long enough to hide that (2048^2 world 1: 27.2 vs
// 19.0 us per update; 16384^2 world 1: 812 us either way); smaller shards use k_pack<true>.
constexpr int64_t kFoldPackTable = 64ll << 20;
inline bool folds_pack(const smx_shape& s) {
    return (int64_t)(s.rows + 1) * s.ld * 8 >= kFoldPackTable;
}
int g_blocks_per_cu = 0;  // 0: kDefaultBpc, capped by the occupancy API (see blocks_per_cu)
constexpr int kDefaultBpc = 5;

using UpdFn = void (*)(const double*, double*, int64_t, int, int, int, int, int, int, int,
                       smx_ctl*, const smx_part*, int, int32_t*, double*, int64_t, const double*,
                       int, int, double*);

template <int MODE>
UpdFn upd_fn(int v) {
    switch (v) {
        case 0: return k_update<MODE, 2, true, false, false>;
        case 1: return k_update<MODE, 2, true, true, false>;
        case 2: return k_update<MODE, 2, true, false, true>;
        case 3: return k_update<MODE, 2, true, true, true>;
        case 4: return k_update<MODE, 1, true, false, true>;
        case 5: return k_update<MODE, 1, true, true, true>;
        case 6: return k_update<MODE, 4, true, false, false>;
        case 7: return k_update<MODE, 4, true, false, true>;
        case 8: return k_update<MODE, 2, false, false, false>;
        case 9: return k_update<MODE, 1, true, false, false>;
        case 10: return k_update<MODE, 2, true, true, false, true>;
        default: return k_update<MODE, 1, true, true, true, true>;
    }
}

int variant_for(const smx_shape& s) {
    if (g_variant >= 0) return g_variant;
    return (int64_t)(s.rows + 1) * s.ld * 8 <= kCacheTable ? kSmallVariant : kLargeVariant;
}

// Resident blocks per CU for a kernel, cached.  The grid is exactly CUs x this, so every block
// is resident at once and the balanced unit ranges finish together (no second residency round).
int blocks_per_cu(const void* fn) {
    if (g_blocks_per_cu > 0) return g_blocks_per_cu;
    struct Entry {
        const void* fn;
        int dev;
        int bpc;
    };
    static Entry cache[128];
    static int ncache = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    for (int i = 0; i < ncache; ++i)
        if (cache[i].fn == fn && cache[i].dev == dev) return cache[i].bpc;
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, fn, kUpdBlock, 0) != hipSuccess ||
        bpc < 1)
        bpc = 4;
    // ROCm 7.2 over-reports by one block/CU for 256-thread kernels above 80 SGPRs
    // (MI355X_MICROARCH.md, residency): keep one block of margin below the API's answer.
    if (bpc > 1) bpc -= 1;
    if (bpc > kDefaultBpc) bpc = kDefaultBpc;
    if (ncache < 128) cache[ncache++] = Entry{fn, dev, bpc};
    return bpc;
}

int num_cus() {
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (!cus[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v < 1)
            v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}

// Grid = resident blocks, trimmed so the wave count is a multiple of the chunks per row (then
// every wave keeps one pivot-row slice for the whole sweep).
int update_grid(const smx_shape& s, const void* fn, int reserved) {
    const int64_t R = s.rows + 1;
    const int64_t nchunks = (s.m + 1 + 2 * kWave - 1) / (2 * kWave);
    const int64_t units = nchunks * R;
    int64_t blocks = (int64_t)num_cus() * blocks_per_cu(fn) - reserved;
    if (blocks < 1) blocks = 1;
    // waves = a multiple of lcm(nchunks, waves per block) when that keeps >= 3/4 of them
    int64_t g = nchunks, h = kUpdWaves;
    while (h) {
        const int64_t t = g % h;
        g = h;
        h = t;
    }
    const int64_t lcm = nchunks / g * kUpdWaves;
    const int64_t waves = blocks * kUpdWaves;
    if (waves >= lcm && (waves - waves % lcm) * 4 >= waves * 3) blocks = (waves - waves % lcm) / kUpdWaves;
    const int64_t need = (units + kUpdWaves - 1) / kUpdWaves;
    if (blocks > need) blocks = need;
    if (blocks < 1) blocks = 1;
    return (int)blocks + reserved;
}

template <int MODE>
int launch_update_mode(const double* Tin, double* Tout, const smx_shape& s, int parity,
                       smx_ctl* ctl, const smx_part* parts, int32_t* log, double* xhist,
                       int64_t log_cap, const double* recv, int fr, int fc, hipStream_t st,
                       int reserve = 0, double* send = nullptr) {
    const int v = variant_for(s);
    UpdFn fn = upd_fn<MODE>(v);
    // kFused: the first nparts workgroups compute the look-ahead records; within the Infinity
    // Cache they are reserved (their extra round trips would be the critical path), beyond it
    // they sweep too (profiles/r01_sweep_small.jsonl)
    constexpr bool LA = MODE == kFused || MODE == kShardFused;
    const bool la_sweep = LA && (int64_t)(s.rows + 1) * s.ld * 8 > kLaSweepTable;
    // reserve: resident slots left free for kernels of another stream (overlapped shard chain)
    int grid = update_grid(s, (const void*)fn, (LA && !la_sweep ? s.nparts : 0) + reserve) -
               reserve;
    if (grid < s.nparts) grid = s.nparts;
    if (grid < 1) grid = 1;
    if (LA) fr = la_sweep ? 1 : 0;   // kShardFused: fc = rank count (caller)
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kUpdBlock), 0, st, Tin,
                       Tout, s.ld, s.rows, s.n, s.m, s.flen, fscan_of(s), s.row0, parity, ctl,
                       parts, s.nparts, log, xhist, log_cap, recv, fr, fc, send);
    return (int)hipGetLastError();
}

int launch_update(const double* Tin, double* Tout, const smx_shape& s, int parity, smx_ctl* ctl,
                  const smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
                  hipStream_t st) {
    return launch_update_mode<kSingle>(Tin, Tout, s, parity, ctl, parts, log, xhist, log_cap,
                                       nullptr, 0, 0, st);
}

// Chains (smx_tune_fused): 0 select + update; 1 one fused kernel per pivot (default); 2 as 1, and
// the sharded chain overlaps the next step's look-ahead + all-gather with the sweep on a second
// stream -- correct, but slower on this stack: the two cross-stream waits per step cost more than
// the all-gather they hide (profiles/r01_shard_overlap_trace.txt).
int g_fused = 1;

int launch_chain(double* buf0, double* buf1, const smx_shape& s, int parity, int k, smx_ctl* ctl,
                 smx_part* parts, int32_t* log, double* xhist, int64_t log_cap, hipStream_t st) {
    if (g_fused && k > 0) {
        // prime the records of the first step, one fused kernel per pivot, publish the next
        int err = launch_prime(parity ? buf1 : buf0, s, parity, ctl, parts, st);
        if (err) return err;
        for (int step = 0; step < k; ++step) {
            const int p = (parity + step) & 1;
            err = launch_update_mode<kFused>(p ? buf1 : buf0, p ? buf0 : buf1, s, p, ctl, parts,
                                             log, xhist, log_cap, nullptr, 0, 0, st);
            if (err) return err;
        }
        return launch_publish(s, (parity + k) & 1, ctl, parts, st);
    }
    for (int step = 0; step < k; ++step) {
        const int p = (parity + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        int err = launch_select(tin, s, p, ctl, parts, st);
        if (err) return err;
        err = launch_update(tin, tout, s, p, ctl, parts, log, xhist, log_cap, st);
        if (err) return err;
    }
    return 0;
}

struct Graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

}  // namespace

// =============================================================================================
extern "C" {

int smx_version(char* buf, int len) {
    const char* v = "smx 0.1 gfx950 fp64 (select, finalize, update<single|shard|forced>, reset, "
                    "pack, merge)";
    if (buf && len > 0) {
        strncpy(buf, v, (size_t)len - 1);
        buf[len - 1] = 0;
    }
    return 8;
}

int smx_nparts_for(int32_t rows, int32_t m) { return nparts_for(rows, m); }

int smx_tune_set(int32_t variant, int32_t blocks_per_cu_override) {
    if (variant >= kNumVariants) return (int)hipErrorInvalidValue;
    if (variant >= kFirstDiagVariant) {   // wrong-bits timing variants: explicit opt-in only
        const char* env = getenv("SMX_ALLOW_DIAG");
        if (!env || env[0] != '1') return (int)hipErrorInvalidValue;
    }
    if (variant >= 0 || variant == -2) g_variant = variant >= 0 ? variant : -1;
    if (blocks_per_cu_override >= 0) g_blocks_per_cu = blocks_per_cu_override;
    return 0;
}

int smx_tune_fused(int32_t on) {
    const int prev = g_fused;
    if (on >= 0) g_fused = on > 2 ? 2 : on;
    return prev;
}

int smx_tune_get(int32_t* variant, int32_t* blocks_per_cu_override, int32_t* nvariants,
                 int32_t* units_in_flight, int32_t* vec, int32_t* nt) {
    if (variant) *variant = g_variant;
    if (blocks_per_cu_override) *blocks_per_cu_override = g_blocks_per_cu;
    if (nvariants) *nvariants = kNumVariants;
    const int gv = g_variant >= 0 ? g_variant : kLargeVariant;   // auto: report the HBM one
    if (units_in_flight) *units_in_flight = kVariants[gv].u;
    if (vec) *vec = 2;
    if (nt) *nt = kVariants[gv].nts | (kVariants[gv].ntl << 1) | (kVariants[gv].pipe << 2);
    return 0;
}

int smx_reset(const double* T, const smx_shape* shape, int32_t parity, int32_t clear_count,
              smx_ctl* ctl, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_reset, dim3(1), dim3(1024), 0, S(stream), T, shape->ld, shape->rows,
                       shape->m, fscan_of(*shape), shape->row0, parity & 1, clear_count, ctl);
    return (int)hipGetLastError();
}

int smx_select(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
               smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_select(T, *shape, parity & 1, ctl, parts, S(stream));
}

int smx_finalize(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                 const smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kWave), 0, S(stream), parts, shape->nparts,
                       parity & 1, shape->n, shape->m, shape->flen, T, shape->ld, ctl);
    return (int)hipGetLastError();
}

int smx_update(const double* Tin, double* Tout, const smx_shape* shape, int32_t parity,
               smx_ctl* ctl, const smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
               void* stream) {
    if (!shape_ok(shape) || Tin == Tout) return (int)hipErrorInvalidValue;
    return launch_update(Tin, Tout, *shape, parity & 1, ctl, parts, log, xhist, log_cap,
                         S(stream));
}

int smx_set_xpos(smx_ctl* ctl, int32_t parity, int32_t x1code, int32_t x2code, void* stream) {
    hipLaunchKernelGGL(k_set_xpos, dim3(1), dim3(kWave), 0, S(stream), ctl, parity & 1, x1code,
                       x2code);
    return (int)hipGetLastError();
}

int smx_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
            smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
            void* stream) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 0) return (int)hipErrorInvalidValue;
    return launch_chain(buf0, buf1, *shape, parity & 1, k, ctl, parts, log, xhist, log_cap,
                        S(stream));
}

int smx_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
                  void* stream, float* host_update_ms, float* host_total_ms) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 1 || !host_update_ms || !host_total_ms)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    const int p0 = parity & 1;
    hipEvent_t* ev = new hipEvent_t[2 * (size_t)k + 1];
    int err = 0;
    for (int i = 0; i < 2 * k + 1; ++i) {
        if (hipEventCreate(&ev[i]) != hipSuccess) {
            for (int j = 0; j < i; ++j) (void)hipEventDestroy(ev[j]);
            delete[] ev;
            return (int)hipErrorOutOfMemory;
        }
    }
    (void)hipEventRecord(ev[2 * k], st);
    if (g_fused) err = launch_prime(p0 ? buf1 : buf0, *shape, p0, ctl, parts, st);
    for (int step = 0; step < k && !err; ++step) {
        const int p = (p0 + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        if (g_fused) {
            (void)hipEventRecord(ev[2 * step], st);
            err = launch_update_mode<kFused>(tin, tout, *shape, p, ctl, parts, log, xhist,
                                             log_cap, nullptr, 0, 0, st);
            (void)hipEventRecord(ev[2 * step + 1], st);
            continue;
        }
        err = launch_select(tin, *shape, p, ctl, parts, st);
        if (err) break;
        (void)hipEventRecord(ev[2 * step], st);
        err = launch_update(tin, tout, *shape, p, ctl, parts, log, xhist, log_cap, st);
        (void)hipEventRecord(ev[2 * step + 1], st);
    }
    if (!err && g_fused) err = launch_publish(*shape, (p0 + k) & 1, ctl, parts, st);
    if (!err) err = (int)hipEventSynchronize(ev[2 * k - 1]);
    if (!err) {
        for (int step = 0; step < k; ++step)
            (void)hipEventElapsedTime(&host_update_ms[step], ev[2 * step], ev[2 * step + 1]);
        (void)hipEventElapsedTime(host_total_ms, ev[2 * k], ev[2 * k - 1]);
    }
    for (int i = 0; i < 2 * k + 1; ++i) (void)hipEventDestroy(ev[i]);
    delete[] ev;
    return err;
}

int smx_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                     int32_t k, smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist,
                     int64_t log_cap, void* stream, void** graph_out) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 1 || !graph_out) return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    Graph* g = new Graph();
    hipError_t err = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    if (err != hipSuccess) {
        delete g;
        return (int)err;
    }
    int lerr = launch_chain(buf0, buf1, *shape, parity & 1, k, ctl, parts, log, xhist, log_cap,
                            st);
    err = hipStreamEndCapture(st, &g->graph);
    if (lerr || err != hipSuccess) {
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return lerr ? lerr : (int)err;
    }
    err = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    if (err != hipSuccess) {
        (void)hipGraphDestroy(g->graph);
        delete g;
        return (int)err;
    }
    *graph_out = g;
    return 0;
}

int smx_graph_launch(void* graph, void* stream) {
    if (!graph) return (int)hipErrorInvalidValue;
    return (int)hipGraphLaunch(static_cast<Graph*>(graph)->exec, S(stream));
}

int smx_graph_destroy(void* graph) {
    if (!graph) return 0;
    Graph* g = static_cast<Graph*>(graph);
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    delete g;
    return 0;
}

int smx_update_forced(const double* Tin, double* Tout, const smx_shape* shape, int32_t r,
                      int32_t c, void* stream) {
    if (!shape_ok(shape) || Tin == Tout) return (int)hipErrorInvalidValue;
    if (r < 0 || r >= shape->rows || c < 0 || c > shape->m) return (int)hipErrorInvalidValue;
    return launch_update_mode<kForced>(Tin, Tout, *shape, 0, nullptr, nullptr, nullptr, nullptr,
                                       0, nullptr, r, c, S(stream));
}

int smx_shard_pack(const double* T, const smx_shape* shape, int32_t parity, const smx_ctl* ctl,
                   const smx_part* parts, double* send, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_pack<false>(T, *shape, parity & 1, ctl, parts, send, S(stream));
}

int smx_shard_merge(const double* recv, int32_t nranks, const smx_shape* shape,
                    int32_t parity, smx_ctl* ctl, int32_t* log, int64_t log_cap, void* stream) {
    (void)parity;
    if (!shape_ok(shape) || nranks < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_merge, dim3(1), dim3(kWave), 0, S(stream), recv, nranks, shape->ld,
                       shape->n, shape->m, shape->flen, ctl, log, log_cap);
    return (int)hipGetLastError();
}

int smx_shard_update(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                     const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                     int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || Tin == Tout || nranks < 1) return (int)hipErrorInvalidValue;
    smx_shape sh = *shape;
    sh.nparts = nranks;   // the update kernel's partial count is the rank count in shard mode
    return launch_update_mode<kShard>(Tin, Tout, sh, parity & 1, ctl, nullptr, log, nullptr,
                                      log_cap, recv, 0, 0, S(stream));
}


int smx_batch_solve(const double* tabs, const int32_t* dims, int32_t B, int32_t Rmax,
                    int32_t ldb, int32_t max_pivots, double* out, int32_t* rc, double* xv,
                    double* snaps, int32_t* status, int32_t* npivots, void* stream) {
    if (B < 0 || Rmax < 1 || Rmax > kWave || ldb < 1 || ldb > 64 || max_pivots < 0)
        return (int)hipErrorInvalidValue;
    if (B == 0) return 0;
    const dim3 grid((B + 3) / 4), block(256);
    hipStream_t st = S(stream);
    if (ldb <= 4)
        hipLaunchKernelGGL(k_batch<4>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else if (ldb <= 8)
        hipLaunchKernelGGL(k_batch<8>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else if (ldb <= 16)
        hipLaunchKernelGGL(k_batch<16>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else if (ldb <= 32)
        hipLaunchKernelGGL(k_batch<32>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else
        hipLaunchKernelGGL(k_batch<64>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    return (int)hipGetLastError();
}


// ---- native RCCL shard driver: the all-gather on the solver's own stream --------------------
// (torch.distributed would run it on its own NCCL stream: one cross-stream event wait per pivot,
// ~14 us measured; here the whole pivot -- select, pack, ncclAllGather, update -- is one
// stream-ordered sequence that can also be captured in a hipGraph.)
static int nccl_err(ncclResult_t r) { return r == ncclSuccess ? 0 : -1000 - (int)r; }

int smx_comm_unique_id(void* id_out) {
    if (!id_out) return (int)hipErrorInvalidValue;
    ncclUniqueId id;
    const int err = nccl_err(ncclGetUniqueId(&id));
    if (!err) memcpy(id_out, &id, sizeof(id));
    return err;
}

int smx_comm_init(void** comm_out, int32_t nranks, const void* id, int32_t rank) {
    if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return (int)hipErrorInvalidValue;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const int err = nccl_err(ncclCommInitRank(&comm, nranks, uid, rank));
    if (!err) *comm_out = comm;
    return err;
}

int smx_comm_destroy(void* comm) {
    if (!comm) return 0;
    return nccl_err(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)));
}

namespace {
// Fused sharded chain, per pivot: one ncclAllGather -> k_update<kShardFused> (merge, sweep, the
// records of step k+1, and -- by its last look-ahead workgroup -- step k+1's header and candidate
// rows in `send`).  Primed by k_la_prime + k_pack<true>, closed by k_publish.  e_upd: 2k events
// around the updates.
int shard_chain_fused(double* buf0, double* buf1, const smx_shape& s, int parity, int k,
                      smx_ctl* ctl, smx_part* parts, double* send, double* recv, int nranks,
                      ncclComm_t comm, int32_t* log, int64_t log_cap, hipEvent_t* e_upd,
                      hipStream_t st) {
    double* T0 = parity ? buf1 : buf0;
    const bool fold = folds_pack(s);
    int err = launch_prime(T0, s, parity, ctl, parts, st);
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    for (int step = 0; step < k && !err; ++step) {
        const int p = (parity + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        if (step == 0 || !fold)
            err = launch_pack<true>(tin, s, p, ctl, parts + (size_t)p * s.nparts, send, st);
        if (!err) err = nccl_err(ncclAllGather(send, recv, slot, ncclFloat64, comm, st));
        if (err) break;
        if (e_upd) (void)hipEventRecord(e_upd[2 * step], st);
        err = launch_update_mode<kShardFused>(tin, tout, s, p, ctl, parts, log, nullptr, log_cap,
                                              recv, 0, nranks, st, 0, fold ? send : nullptr);
        if (e_upd) (void)hipEventRecord(e_upd[2 * step + 1], st);
    }
    if (!err) err = launch_publish(s, (parity + k) & 1, ctl, parts, st);
    return err;
}

// The two halves of an overlapped sharded step (also exported for the P-rank simulation tests):
// ahead = step k+1's records (s.nparts of them, slot parity^1) and, if `pack`, its header and
// candidate rows into `send`, from T_k and step k's gathered headers; sweep = the update of step
// k without look-ahead workgroups, leaving `reserve` resident slots free.
int launch_ahead(const double* T, const smx_shape& s, int parity, const double* recv,
                 int nranks, smx_ctl* ctl, smx_part* parts, double* send, bool pack,
                 hipStream_t st) {
    smx_part* pn = parts + (size_t)(parity ^ 1) * s.nparts;
    hipLaunchKernelGGL(k_shard_la, dim3(s.nparts), dim3(kUpdBlock), 0, st, T, s.ld, s.rows, s.m,
                       s.flen, fscan_of(s), s.row0, recv, nranks, ctl, pn, parity ^ 1);
    if (pack)
        hipLaunchKernelGGL(k_pack_ahead, dim3(s.nparts), dim3(kUpdBlock), 0, st, T, s.ld, s.rows,
                           s.m, s.flen, s.row0, recv, nranks, ctl, pn, s.nparts, parity ^ 1,
                           send);
    return (int)hipGetLastError();
}

int launch_sweep(const double* Tin, double* Tout, const smx_shape& s, int parity,
                 const double* recv, int nranks, smx_ctl* ctl, int32_t* log, int64_t log_cap,
                 int reserve, hipStream_t st) {
    smx_shape sy = s;
    sy.nparts = 0;   // no look-ahead workgroups
    return launch_update_mode<kShardFused>(Tin, Tout, sy, parity, ctl, nullptr, log, nullptr,
                                           log_cap, recv, 0, nranks, st, reserve);
}

// The exchange stream and two events of the overlapped chain, created once per device.
struct Overlap {
    hipStream_t s2 = nullptr;
    hipEvent_t ev_sweep = nullptr, ev_gather = nullptr;
};

int overlap_for_device(Overlap** out) {
    static Overlap cache[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return (int)hipErrorInvalidDevice;
    Overlap& o = cache[dev];
    if (!o.s2) {
        hipError_t e = hipStreamCreateWithFlags(&o.s2, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&o.ev_sweep, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&o.ev_gather, hipEventDisableTiming);
        if (e != hipSuccess) return (int)e;
    }
    *out = &o;
    return 0;
}

constexpr int kOverlapParts = 16;   // look-ahead workgroups of the overlapped chain

// Overlapped sharded chain.  recv holds two gather slots (step parity).  Per step k:
//   S2: wait(T_k ready) -> k_shard_la (records of k+1) -> k_pack_ahead -> all-gather into
//       recv[(k+1)&1] -> record ev_gather
//   S1: k_update<kShardFused> without look-ahead workgroups (T_k -> T_{k+1}, pivot from
//       recv[k&1]) -> wait(ev_gather) -> record ev_sweep
// S1 waiting for the gather before the next sweep also orders S2's reads of T_k before the
// sweep that overwrites it.  The last step computes the records of step k (for a continuation)
// but no pack/gather.
int shard_chain_overlap(double* buf0, double* buf1, const smx_shape& s, int parity, int k,
                        smx_ctl* ctl, smx_part* parts, double* send, double* recv, int nranks,
                        ncclComm_t comm, int32_t* log, int64_t log_cap, hipEvent_t* e_upd,
                        hipStream_t st) {
    Overlap* o = nullptr;
    int err = overlap_for_device(&o);
    if (err) return err;
    smx_shape sx = s;
    sx.nparts = s.nparts < kOverlapParts ? s.nparts : kOverlapParts;
    const int npx = sx.nparts;
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    const size_t rsz = (size_t)nranks * slot;
    double* T0 = parity ? buf1 : buf0;
    err = launch_prime(T0, sx, parity, ctl, parts, st);
    if (!err) err = launch_pack<true>(T0, sx, parity, ctl, parts + (size_t)parity * npx, send, st);
    if (!err) err = nccl_err(ncclAllGather(send, recv + (size_t)parity * rsz, slot, ncclFloat64,
                                           comm, st));
    if (!err) err = (int)hipEventRecord(o->ev_sweep, st);
    for (int step = 0; step < k && !err; ++step) {
        const int p = (parity + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        const double* rc = recv + (size_t)p * rsz;
        double* rn = recv + (size_t)(p ^ 1) * rsz;
        const bool more = step + 1 < k;
        err = (int)hipStreamWaitEvent(o->s2, o->ev_sweep, 0);
        if (!err) err = launch_ahead(tin, sx, p, rc, nranks, ctl, parts, send, more, o->s2);
        if (!err && more)
            err = nccl_err(ncclAllGather(send, rn, slot, ncclFloat64, comm, o->s2));
        if (!err) err = (int)hipEventRecord(o->ev_gather, o->s2);
        if (err) break;
        if (e_upd) (void)hipEventRecord(e_upd[2 * step], st);
        err = launch_sweep(tin, tout, s, p, rc, nranks, ctl, log, log_cap, npx, st);
        if (e_upd) (void)hipEventRecord(e_upd[2 * step + 1], st);
        if (!err) err = (int)hipStreamWaitEvent(st, o->ev_gather, 0);
        if (!err) err = (int)hipEventRecord(o->ev_sweep, st);
    }
    if (!err) err = launch_publish(sx, (parity + k) & 1, ctl, parts, st);
    return err;
}

int shard_pivot(double* tin, double* tout, const smx_shape& s, int p, smx_ctl* ctl,
                smx_part* parts, double* send, double* recv, int nranks, ncclComm_t comm,
                int32_t* log, int64_t log_cap, hipEvent_t e0, hipEvent_t e1, hipStream_t st) {
    int err = launch_select(tin, s, p, ctl, parts, st);
    if (err) return err;
    err = smx_shard_pack(tin, &s, p, ctl, parts, send, st);
    if (err) return err;
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    err = nccl_err(ncclAllGather(send, recv, slot, ncclFloat64, comm, st));
    if (err) return err;
    if (e0) (void)hipEventRecord(e0, st);
    err = smx_shard_update(tin, tout, recv, nranks, &s, p, ctl, log, log_cap, st);
    if (e1) (void)hipEventRecord(e1, st);
    return err;
}
}  // namespace

int smx_shard_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  smx_ctl* ctl, smx_part* parts, double* send, double* recv, int32_t nranks,
                  void* comm, int32_t* log, int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || !comm || nranks < 1 || k < 0) return (int)hipErrorInvalidValue;
    if (g_fused == 2 && k > 0)
        return shard_chain_overlap(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                   nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap,
                                   nullptr, S(stream));
    if (g_fused && k > 0)
        return shard_chain_fused(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                 nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap,
                                 nullptr, S(stream));
    for (int step = 0; step < k; ++step) {
        const int p = (parity + step) & 1;
        const int err = shard_pivot(p ? buf1 : buf0, p ? buf0 : buf1, *shape, p, ctl, parts,
                                    send, recv, nranks, reinterpret_cast<ncclComm_t>(comm), log,
                                    log_cap, nullptr, nullptr, S(stream));
        if (err) return err;
    }
    return 0;
}

int smx_shard_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                        int32_t k, smx_ctl* ctl, smx_part* parts, double* send, double* recv,
                        int32_t nranks, void* comm, int32_t* log, int64_t log_cap, void* stream,
                        float* host_update_ms, float* host_total_ms) {
    if (!shape_ok(shape) || !comm || nranks < 1 || k < 1 || !host_update_ms || !host_total_ms)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    hipEvent_t* ev = new hipEvent_t[2 * (size_t)k + 1];
    for (int i = 0; i < 2 * k + 1; ++i) {
        if (hipEventCreate(&ev[i]) != hipSuccess) {
            for (int j = 0; j < i; ++j) (void)hipEventDestroy(ev[j]);
            delete[] ev;
            return (int)hipErrorOutOfMemory;
        }
    }
    (void)hipEventRecord(ev[2 * k], st);
    int err = 0;
    if (g_fused == 2)
        err = shard_chain_overlap(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                  nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap, ev,
                                  st);
    else if (g_fused)
        err = shard_chain_fused(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap, ev, st);
    for (int step = 0; step < k && !err && !g_fused; ++step) {
        const int p = (parity + step) & 1;
        err = shard_pivot(p ? buf1 : buf0, p ? buf0 : buf1, *shape, p, ctl, parts, send, recv,
                          nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap, ev[2 * step],
                          ev[2 * step + 1], st);
    }
    if (!err) err = (int)hipEventSynchronize(ev[2 * k - 1]);
    if (!err) {
        for (int step = 0; step < k; ++step)
            (void)hipEventElapsedTime(&host_update_ms[step], ev[2 * step], ev[2 * step + 1]);
        (void)hipEventElapsedTime(host_total_ms, ev[2 * k], ev[2 * k - 1]);
    }
    for (int i = 0; i < 2 * k + 1; ++i) (void)hipEventDestroy(ev[i]);
    delete[] ev;
    return err;
}

int smx_shard_fused_prime(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                          smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_prime(T, *shape, parity & 1, ctl, parts, S(stream));
}

int smx_shard_fused_begin(const double* T, const smx_shape* shape, int32_t parity,
                          const smx_ctl* ctl, const smx_part* parts, double* send, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_pack<true>(T, *shape, parity & 1, ctl,
                             parts + (size_t)(parity & 1) * shape->nparts, send, S(stream));
}

int smx_shard_fused_finish(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                           const smx_shape* shape, int32_t parity, smx_ctl* ctl, smx_part* parts,
                           double* send, int32_t* log, int64_t log_cap, void* ev_before,
                           void* ev_after, void* stream) {
    if (!shape_ok(shape) || Tin == Tout || nranks < 1) return (int)hipErrorInvalidValue;
    if (ev_before) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_before), S(stream));
    const int err = launch_update_mode<kShardFused>(Tin, Tout, *shape, parity & 1, ctl, parts,
                                                    log, nullptr, log_cap, recv, 0, nranks,
                                                    S(stream), 0,
                                                    folds_pack(*shape) ? send : nullptr);
    if (ev_after) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_after), S(stream));
    return err;
}

int smx_shard_folds_pack(const smx_shape* shape) {
    return shape_ok(shape) && folds_pack(*shape) ? 1 : 0;
}

int smx_shard_ahead(const double* T, const smx_shape* shape, int32_t parity, const double* recv,
                    int32_t nranks, smx_ctl* ctl, smx_part* parts, double* send, void* stream) {
    if (!shape_ok(shape) || nranks < 1) return (int)hipErrorInvalidValue;
    return launch_ahead(T, *shape, parity & 1, recv, nranks, ctl, parts, send, true, S(stream));
}

int smx_shard_sweep(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                    const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                    int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || Tin == Tout || nranks < 1) return (int)hipErrorInvalidValue;
    return launch_sweep(Tin, Tout, *shape, parity & 1, recv, nranks, ctl, log, log_cap, 0,
                        S(stream));
}

int smx_copy_probe(const double* src, double* dst, int64_t ndoubles, int32_t variant,
                   void* stream) {
    if (!src || !dst || ndoubles < 2 || (ndoubles & 1) || variant < 0 || variant > 1)
        return (int)hipErrorInvalidValue;
    const int64_t n2 = ndoubles / 2;
    const auto* a = reinterpret_cast<const dbl2*>(src);
    auto* b = reinterpret_cast<dbl2*>(dst);
    if (variant == 0)
        hipLaunchKernelGGL(k_copy<4>, dim3(num_cus()), dim3(256), 0, S(stream), a, b, n2);
    else
        hipLaunchKernelGGL(k_copy<1>, dim3(num_cus()), dim3(1024), 0, S(stream), a, b, n2);
    return (int)hipGetLastError();
}

int smx_fused_publish(const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                      const smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_publish(*shape, parity & 1, ctl, parts, S(stream));
}

int smx_shard_begin(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                    smx_part* parts, double* send, void* stream) {
    int err = smx_select(T, shape, parity, ctl, parts, stream);
    if (err) return err;
    return smx_shard_pack(T, shape, parity, ctl, parts, send, stream);
}

int smx_shard_finish(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                     const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                     int64_t log_cap, void* ev_before, void* ev_after, void* stream) {
    if (ev_before) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_before), S(stream));
    const int err = smx_shard_update(Tin, Tout, recv, nranks, shape, parity, ctl, log, log_cap,
                                     stream);
    if (ev_after) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_after), S(stream));
    return err;
}

}  // extern "C"
