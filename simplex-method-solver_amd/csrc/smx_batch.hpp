// smx_batch.hpp -- k_copy (copy-ceiling probe) and k_batch (many small LPs, one wavefront each)
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

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

}  // namespace
