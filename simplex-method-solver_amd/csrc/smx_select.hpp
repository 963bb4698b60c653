// smx_select.hpp -- k_reset, k_select, k_finalize (pick_element, simplex.py:70-141)
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

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

}  // namespace
