// smx_lookahead.hpp -- the fused chain's look-ahead: next-step records from T_k, decision, prime/publish, pack
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

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
__device__ __forceinline__ int block_min_int_dpp(int x, int* s_tmp) {
    x = wave_min_int_dpp(x);
    const int wid = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_tmp[wid] = x;
    __syncthreads();
    int r = s_tmp[0];
#pragma unroll
    for (int w = 1; w < NT / kWave; ++w) r = min(r, s_tmp[w]);
    return r;
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

}  // namespace
