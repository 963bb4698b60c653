// smx_shard.hpp -- row-sharded exchange: k_pack, k_merge, the overlapped chain's k_shard_la / k_pack_ahead
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

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

}  // namespace
