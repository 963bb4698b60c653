// smx_window.hpp -- the window planner of block pivots: the decisions of a block's P pivots
// (pick_element, simplex.py:70-141) from a window of the first columns of every row, kept current
// pivot by pivot (recalculate_matrix's per-element rule, simplex.py:155-175), instead of chains of
// up to P update steps re-derived per value from the block's input table (the register form,
// k_blk_step in smx_block.hpp).
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

// Why.  The register-form planner's step derives every value it reads -- the pivot row at the
// columns it scans, the entering column of every row -- as a chain of up to D update steps from
// the block's input table T_k: a 20-pivot step is ~4 dependent memory round trips plus chains of
// ~75 ns per step on one wave per SIMD, and it ran on 64 workgroups at 16384 rows (a quarter of
// the chip), 16.3 us per pivot on average at 20 pivots per block.  But the pivot
// decisions only ever read a few columns: the "-b" column (phase 1, the ratio test, simplex.py:
// 73-76, 115), the entering column (the first negative f-row entry, simplex.py:94-98, at the low
// column indices on these LPs: 16384^2 over 220 pivots never past column 27, config 5 never past
// 13; tests/golden/bench16k.json, config5.json) and the phase-1 row's first positive entry.
// So the window planner keeps T_{k+D} at the first kWin - 1 columns and the "-b" column of every
// row (and the f-row) in a [2][R][kWin] scratch buffer -- one row per wave, one column per lane --
// and each step applies its pivot to the whole window with the reference's own expression: one
// update step per value, every row and column in parallel over 256 workgroups of four waves.
// A step is then two dependent memory round trips (the records, then the pivot row's window) and
// one element update, whatever D is.  The pivot rows at every column, which the sweep needs, are
// computed ONCE per block after its last step (k_blk_prows: per column the P pivot rows through
// the pivots before them).  Values outside the window (an entering or phase-1 column past it)
// fall back to chains from T_k (win_colvals / win_chain), so every table is handled; the window
// only decides how often that slow path runs.  Same operations on the same operands in the same
// order as the single-pivot sweeps: the same bits (tests/test_gpu_block.py runs every case with
// both planners, and with windows of 2..64 columns to drive the fallbacks).
// (kWin = 64 window slots per row, one wave's lanes: smx_block.hpp, beside the scratch layout)
constexpr int kWinMaxG = 256;     // planner workgroups at most (the records merge: kBlkPartsMax)
// Eight waves per workgroup: 2,048 waves at 16384 rows, eight rows each (one batch), two per
// SIMD.  (Four waves of 16 rows: the row pass, a dependent chain of shuffles, divisions and
// stores per batch on one wave per SIMD, took 4.2 us of a 12 us step, profiles/r06g/.)
constexpr int kWinNT = 512;
constexpr int kWinWaves = kWinNT / kWave;
constexpr int kWinBatch = 8;      // rows of a wave updated together (two batches in flight)
static_assert(kWinMaxG <= kBlkPartsMax, "window planner records");

// Rows per wave and workgroups of a window step for `rows` constraint rows: four waves per
// workgroup, at most kWinMaxG workgroups (16384 rows: 16 per wave on 256 workgroups)
__host__ __device__ __forceinline__ int win_rpw(int rows) {
    const int w = kWinMaxG * kWinWaves;
    const int r = (rows + w - 1) / w;
    return r < 1 ? 1 : r;
}
__host__ __device__ __forceinline__ int win_groups(int rows) {
    const int per = win_rpw(rows) * kWinWaves;
    const int g = (rows + per - 1) / per;
    return g < 1 ? 1 : g;
}

// Column of window slot k when nwin slots are in use (C = m + 1 columns): the first nwin - 1
// columns, then the "-b" column m; every column of a table of at most nwin; -1: an unused slot
__host__ __device__ __forceinline__ int win_col(int k, int nwin, int C) {
    if (k >= nwin) return -1;
    if (C <= nwin) return k < C ? k : -1;
    return k < nwin - 1 ? k : C - 1;
}
// Window slot of column j (0 <= j < C), -1 outside the window
__host__ __device__ __forceinline__ int win_slot(int j, int nwin, int C) {
    if (C <= nwin) return j;
    return j < nwin - 1 ? j : (j == C - 1 ? nwin - 1 : -1);
}

// One step of the reference's update on one value x = T_{k+q}[i][j] (simplex.py:155-175): the
// pivot row (prow) -x / e, or 1 / e at the pivot column (pcol); elsewhere x / e in the pivot
// column, (x e - p mq) / e off it, with p = T_{k+q}[r_q][j] and mq = T_{k+q}[i][c_q] -- two
// products, a difference and a division, each rounded, no FMA
__device__ __forceinline__ double win_upd(double x, bool prow, bool pcol, double p, double mq,
                                          double e) {
    const double a = x * e;
    const double b = p * mq;
    const double num = prow ? (pcol ? 1.0 : -x) : (pcol ? x : (a - b));
    return num / e;
}

// The fallback for a column outside the window (and k_blk_prows' whole job): the values of
// column j after the block's first D pivots, from T_k, step by step.  out(q, v) receives
// v = T_{k+q}[r_q][j] (pivot row q as it was pivoted, q < D), and xo[k] = T_{k+D}[xr[k]][j] for NX
// more rows.  The pivot rows' values are carried through the pivots before theirs (a row pivoted
// twice takes the pivot-row rule at its first step) with the multipliers mul[row][q] =
// T_{k+q}[row][c_q] that each step stored for every row.  A rolled loop over the pivots with the
// rows in a shift register (x[0] is always the next pivot row's value), so the code stays one
// step's worth (the fully unrolled triangle made the planner kernel ~57 k instructions and its
// launches instruction-fetch bound: 18.7 us per step, profiles/r06c/).
template <int NX, class OUT>
__device__ __forceinline__ void win_colvals(const double* __restrict__ T, int64_t ld, int j,
                                            int D, const BlkPiv& pv,
                                            const double* __restrict__ mul, const int* xr,
                                            OUT out, double* xo) {
    double x[kBlkMax];
    double xx[NX > 0 ? NX : 1];
#pragma unroll
    for (int p = 0; p < kBlkMax; ++p) x[p] = p < D ? T[(int64_t)pv.r[p] * ld + j] : 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k) xx[k] = T[(int64_t)xr[k] * ld + j];
#pragma unroll 1
    for (int q = 0; q < D; ++q) {
        const double p = x[0];   // T_{k+q}[r_q][j]: updated by the q pivots before it
        out(q, p);
        const int rq = pv.r[q];
        const bool pc = j == pv.c[q];
        const double e = pv.e[q];
#pragma unroll
        for (int s = 1; s < kBlkMax; ++s) {
            const int t = q + s;   // the row of pivot t, not pivoted yet
            if (t < D)
                x[s] = win_upd(x[s], pv.r[t] == rq, pc, p, mul[(int64_t)pv.r[t] * kBlkMax + q], e);
        }
#pragma unroll
        for (int k = 0; k < NX; ++k)
            xx[k] = win_upd(xx[k], xr[k] == rq, pc, p, mul[(int64_t)xr[k] * kBlkMax + q], e);
#pragma unroll
        for (int s = 0; s + 1 < kBlkMax; ++s) x[s] = x[s + 1];
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) xo[k] = xx[k];
}

// T_{k+D}[i][j] from T_k through the first D pivots, pj[q] = T_{k+q}[r_q][j] (win_colvals)
__device__ __forceinline__ double win_chain(const double* __restrict__ T, int64_t ld, int i, int j,
                                            int D, const BlkPiv& pv, const double* pj,
                                            const double* __restrict__ mul) {
    double x = T[(int64_t)i * ld + j];
#pragma unroll 1
    for (int q = 0; q < D; ++q)
        x = win_upd(x, i == pv.r[q], j == pv.c[q], pj[q], mul[(int64_t)i * kBlkMax + q], pv.e[q]);
    return x;
}

// One pivot of the block (step L: decide block step D = L - 1, apply it to the window, build the
// records of step L).  Grid: win_groups(rows) workgroups of kWinNT threads; wave w owns
// constraint rows [w rpw, (w + 1) rpw).  W = the window, [2][rows + 1][kWin] by step parity.
__global__ __launch_bounds__(kWinNT) void k_blk_wstep(
    const double* __restrict__ T, int64_t ld, int rows, int m, int flen, int fscan, int P, int L,
    int parity, int bn, int nwin, int rpw, int fromT, smx_ctl* __restrict__ ctl,
    BlkHdr* __restrict__ h,
    smx_part* __restrict__ parts, double* __restrict__ mul, double* __restrict__ W,
    int32_t* __restrict__ log, double* __restrict__ xhist, int64_t log_cap) {
    __shared__ BlkPiv s_pv;
    __shared__ Decision s_d;
    __shared__ int s_nb, s_cfD;
    __shared__ double s_e, s_fc, s_prcf;
    __shared__ double s_colc[kBlkMax], s_colf[kBlkMax];   // pivot rows at c / cf (fallbacks)
    __shared__ int s_tmp[kWinWaves];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
    const int b = blockIdx.x, G = gridDim.x;
    const int D = L - 1;
    const int sp = (parity + D) & 1;   // step parity of block step D
    const int C = m + 1;
    const int64_t WR = (int64_t)rows + 1;
    const int jl = win_col(lane, nwin, C);   // this lane's column
    double* __restrict__ Wn = W + (int64_t)(sp ^ 1) * WR * kWin;   // T_{k+L}
    // T_{k+D} at the window: the window of the step before, or at a chain's first step the table
    // itself at the window's columns (no fill pass)
    const double* __restrict__ So = fromT ? T : W + (int64_t)sp * WR * kWin;
    const int64_t sld = fromT ? ld : kWin;
    const int sj = fromT ? max(jl, 0) : lane;
    // Every load of the prologue is unconditional (rows and columns clamped, results masked): a
    // load behind a branch leaves the compiler unable to count the loads in flight, and it then
    // waits for all of them -- the decision behind the whole row prefetch (profiles/r06h/).
    auto wold = [&](int i) -> double {
        const double v = So[(int64_t)i * sld + sj];
        return jl >= 0 ? v : 0.0;
    };
    // Everything that does not depend on the decision is loaded with the decision's operands
    // (one round trip): the stop flag, the pivots so far, the f-row's window, this wave's first
    // rows.  The records go first: a wave's loads return in order, and behind the window rows
    // (8 MB over the chip at 16384 rows) the decision waited ~2 us longer (profiles/r06f/).  On
    // a stopped chain those loads read stale scratch and are discarded.
    SMX_BLK_STAMP(0);
    const int stopped = ctl->term;
    constexpr int RU = kBlkPartsMax / kWave;
    smx_part rp[RU];
    int cD = SMX_NONE;
    if (wid == 0) {
        cD = h->cfs[blk_slot(D, P, bn)];
        const smx_part* __restrict__ slot = parts + (int64_t)blk_slot(D, P, bn) * G;
#pragma unroll
        for (int u = 0; u < RU; ++u) rp[u] = slot[min(lane + u * kWave, G - 1)];
#pragma unroll
        for (int u = 0; u < RU; ++u)
            if (lane + u * kWave >= G) rp[u] = smx_part{SMX_NONE, SMX_NONE, 0.0, 3, SMX_NONE, 0.0};
    }
    asm volatile("" ::: "memory");   // (issue order only: nothing waits here)
    blk_load_pivots(h, D, &s_pv);
    const double fo = wold(rows);
    const int i0 = (b * kWinWaves + wid) * rpw;
    const int i1 = min(rows, i0 + rpw);
    // this wave's first two batches of rows (the row pass keeps two batches in flight)
    double xv[kWinBatch], xn[kWinBatch];
#pragma unroll
    for (int u = 0; u < kWinBatch; ++u) {
        xv[u] = wold(i0 + u < i1 ? i0 + u : rows);
        xn[u] = wold(i0 + kWinBatch + u < i1 ? i0 + kWinBatch + u : rows);
    }
    if (wid == 0) {
        // the decision of step D from its records (every workgroup, identically; the order of
        // the merges is immaterial: total orders)
        const int c = cD;
        int nb;
        First f;
        Cand bb;
        {
            int n0 = SMX_NONE;
            First fi{SMX_NONE, 0.0};
            Cand bq = cand_none();
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                n0 = min(n0, rp[u].p1col);
                fi = first_sel(rp[u].first < fi.idx, First{rp[u].first, rp[u].first_v}, fi);
                const Cand o{rp[u].best_cls, rp[u].best_i, rp[u].best_v};
                bq = cand_sel(better(o, bq), o, bq);
            }
            nb = wave_min_int_dpp(n0);
            f = wave_first_dpp(fi);
            bb = wave_best_dpp(bq);
        }
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
            } else if (bb.cls >= 2) {
                d.status = SMX_NOT_CONVERGE;
            } else {
                d.r = bb.idx;
            }
        } else {
            d.r = nb;                  // phase 1: the column comes from row r below
            d.c = SMX_NONE;
        }
        if (tid == 0) {
            s_nb = nb;
            s_d = d;
            s_cfD = c;
        }
    }
    // A barrier for the LDS hand-off only: __syncthreads() would first wait for every wave's
    // outstanding loads -- the whole row prefetch (profiles/r06g/: the decision at ~4.5 us)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    SMX_BLK_STAMP(1);
    if (stopped) {
        if (D == 0 && b == 0 && tid == 0) h->peff = 0;   // a later block of a stopped chain
        return;
    }
    const int nb = s_nb;
    Decision d = s_d;
    auto terminal = [&](const Decision& dd) {
        if (b == 0 && tid == 0) {
            ctl->sel_status = dd.status;
            ctl->sel_r = dd.r;
            ctl->sel_c = dd.c;
            ctl->negb[sp] = nb;        // the state of T_{k+D}, where the chain stops
            ctl->negf[sp] = s_cfD;
            ctl->term = 1;
            h->peff = D;
        }
    };
    if (d.status != SMX_PIVOT) {
        terminal(d);
        return;
    }
    const int r = d.r;
    const double pw = wold(r);   // T_{k+D}[r][jl]
    int c = d.c;
    if (nb != SMX_NONE) {
        // phase 1: first j < m with T_{k+D}[r][j] > 0 (simplex.py:81-85); the lanes hold the
        // window's columns in increasing order (the "-b" lane is excluded by j < m)
        const unsigned long long bal = __ballot(jl >= 0 && jl < m && pw > 0.0);
        int p1 = bal ? win_col(__ffsll((long long)bal) - 1, nwin, C) : SMX_NONE;
        if (p1 == SMX_NONE && C > nwin) {
            // the columns past the window, T_{k+D}[r][j] from T_k (rounds with early exit; the
            // same minimum in every workgroup)
            for (int j0 = nwin - 1; j0 < m && p1 == SMX_NONE; j0 += kWinNT) {
                const int j = j0 + tid;
                int mine = SMX_NONE;
                if (j < m) {
                    double xo[1];
                    const int xr[1] = {r};
                    win_colvals<1>(T, ld, j, D, s_pv, mul, xr, [](int, double) {}, xo);
                    if (xo[0] > 0.0) mine = j;
                }
                p1 = block_min_int_dpp<kWinNT>(mine, s_tmp);
            }
        }
        if (p1 == SMX_NONE) {
            d.c = SMX_NONE;
            d.status = SMX_INCORRECT;  // simplex.py:88-89
            terminal(d);
            return;
        }
        c = p1;
    }
    // the pivot element and the f-row's multiplier: from the window, or through the pivots so far
    // from T_k when column c lies outside it
    const int cs = __builtin_amdgcn_readfirstlane(win_slot(c, nwin, C));
    double e, fc;
    if (cs >= 0) {
        e = readlane_d(pw, cs);
        fc = readlane_d(fo, cs);
    } else {
        if (tid == 0) {
            const int xr[2] = {r, rows};
            double xo[2];
            win_colvals<2>(T, ld, c, D, s_pv, mul, xr, [&](int q, double v) { s_colc[q] = v; }, xo);
            s_e = xo[0];
            s_fc = xo[1];
        }
        __syncthreads();
        e = s_e;
        fc = s_fc;
    }
    SMX_BLK_STAMP(2);
    // the f-row after this pivot (never the pivot row) and the next entering column: first
    // j < fscan with f_{k+L}[j] < 0 (simplex.py:94-98)
    const double fn = jl >= 0 ? win_upd(fo, false, jl == c, pw, fc, e) : 0.0;
    int cf;
    {
        const unsigned long long bal = __ballot(jl >= 0 && jl < fscan && fn < 0.0);
        cf = bal ? win_col(__ffsll((long long)bal) - 1, nwin, C) : SMX_NONE;
        if (cf == SMX_NONE && C > nwin) {
            for (int j0 = nwin - 1; j0 < fscan && cf == SMX_NONE; j0 += kWinNT) {
                const int j = j0 + tid;
                int mine = SMX_NONE;
                if (j < fscan) {
                    double xo[2];
                    const int xr[2] = {r, rows};
                    win_colvals<2>(T, ld, j, D, s_pv, mul, xr, [](int, double) {}, xo);
                    if (win_upd(xo[1], false, j == c, xo[0], fc, e) < 0.0) mine = j;
                }
                cf = block_min_int_dpp<kWinNT>(mine, s_tmp);
            }
        }
    }
    SMX_BLK_STAMP(3);
    const int cfs = __builtin_amdgcn_readfirstlane(cf != SMX_NONE ? win_slot(cf, nwin, C) : -1);
    if (cf != SMX_NONE && cfs < 0) {
        // the records' column outside the window: the pivot rows there, T_{k+D}[r][cf] too
        if (tid == 0) {
            const int xr[1] = {r};
            double xo[1];
            win_colvals<1>(T, ld, cf, D, s_pv, mul, xr, [&](int q, double v) { s_colf[q] = v; }, xo);
            s_prcf = xo[0];
        }
        __syncthreads();
    }
    // bookkeeping of this pivot (workgroup 0): the plan, the log, the labels (simplex.py:152)
    const int hx0 = move_label(ctl->xpos[sp][0], r, c);
    const int hx1 = move_label(ctl->xpos[sp][1], r, c);
    const int64_t kpiv = ctl->npiv[sp];
    if (b == 0 && tid == 0) {
        const FastDiv fd = fd_prep(e);
        mul[(int64_t)rows * kBlkMax + D] = fc;
        h->r[D] = r;
        h->c[D] = c;
        h->e[D] = e;
        h->y[D] = fd.y;
        h->ok[D] = fd.ok ? 1 : 0;
        h->peff = D + 1;
        h->cfs[blk_slot(L, P, bn)] = cf;
        if (log_cap > 0) {
            log[2 * (kpiv % log_cap)] = r;
            log[2 * (kpiv % log_cap) + 1] = c;
        }
        ctl->npivots = kpiv + 1;
        ctl->npiv[sp ^ 1] = kpiv + 1;
        ctl->sel_status = SMX_PIVOT;
        ctl->sel_r = r;
        ctl->sel_c = c;
        ctl->sel_e = e;
        ctl->xpos[sp ^ 1][0] = hx0;
        ctl->xpos[sp ^ 1][1] = hx1;
        if (xhist && log_cap > 0) {                  // non-basic labels: 0 (simplex.py:60-66)
            if (hx0 < 0) xhist[2 * (kpiv % log_cap)] = 0.0;
            if (hx1 < 0) xhist[2 * (kpiv % log_cap) + 1] = 0.0;
        }
    }
    if (b == 0 && wid == 0 && jl >= 0) Wn[(int64_t)rows * kWin + lane] = fn;
    SMX_BLK_STAMP(4);
    const int64_t hslot = 2 * (kpiv % (log_cap > 0 ? log_cap : 1));
    const bool want_x = xhist && log_cap > 0;
    // The row pass: every row of the wave through this pivot at the window's columns, its
    // multiplier T_{k+D}[i][c] stored for the sweep, and the records of step L on column cf.
    // A batch's rows are independent: their multipliers (lane cs), updates and stores are issued
    // together, then lane u takes row u's "-b" and entering-column entries (ds_bpermute) and adds
    // it to its own partial record; the wave's partials are reduced once at the end (DPP).  (Row by
    // row with scalar read-backs and a record update per row, one dependent division chain after
    // another, the pass took 9.2 us of a 15.3 us step at 16 rows per wave, profiles/r06e/.)
    const int ms = __builtin_amdgcn_readfirstlane(win_slot(m, nwin, C));
    double* __restrict__ mT = blk_mulT(mul, rows + 1);
    const FastDiv efd = fd_prep(e);
    const double ey = efd.y;
    const bool eok = efd.ok;
    BlkRec R{SMX_NONE, First{SMX_NONE, 0.0}, cand_none()};
    for (int ib = i0; ib < i1; ib += kWinBatch) {
        // fallbacks (columns outside the window): lane u derives row ib + u's value from T_k
        double mcv = 0.0, acv = 0.0;
        if (cs < 0 && lane < kWinBatch && ib + lane < i1)
            mcv = win_chain(T, ld, ib + lane, c, D, s_pv, s_colc, mul);
        if (cfs < 0 && cf != SMX_NONE && lane < kWinBatch && ib + lane < i1)
            acv = win_chain(T, ld, ib + lane, cf, D, s_pv, s_colf, mul);
        double mc[kWinBatch], nv[kWinBatch];
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) mc[u] = __shfl(cs >= 0 ? xv[u] : mcv, cs >= 0 ? cs : u);
        // the hoisted-reciprocal division while every numerator of the batch lies inside the
        // exponent window (win_term; the planner chains' argument, smx_block.hpp blk_chain_fd),
        // else the batch again with the IEEE division: the same bits either way
        uint32_t wt = 0;
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            const double a = xv[u] * e;
            const double bq = pw * mc[u];
            const bool pc = jl == c;
            const double num = (ib + u == r) ? (pc ? 1.0 : -xv[u]) : (pc ? xv[u] : (a - bq));
            wt = max(wt, win_term(num));
            const double tq = num * ey;
            const double rr = fma(-e, tq, num);
            nv[u] = fma(rr, ey, tq);
        }
        if (!eok || !__all(jl < 0 || wt < kWinSpan)) {
#pragma unroll
            for (int u = 0; u < kWinBatch; ++u)
                nv[u] = win_upd(xv[u], ib + u == r, jl == c, pw, mc[u], e);
        }
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u)
            if (ib + u < i1 && jl >= 0) Wn[(int64_t)(ib + u) * kWin + lane] = nv[u];
        // the next batch in flight while this one's records are built
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            xv[u] = xn[u];
            const int i2 = ib + 2 * kWinBatch + u;
            xn[u] = wold(i2 < i1 ? i2 : rows);
        }
        double myc = 0.0, mybv = 0.0, mya = 0.0;
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            const double bvu = __shfl(nv[u], ms);
            const double au = cfs >= 0 ? __shfl(nv[u], cfs) : 0.0;
            const bool mine = lane == u;
            myc = mine ? mc[u] : myc;
            mybv = mine ? bvu : mybv;
            mya = mine ? au : mya;
        }
        const int i = ib + lane;
        if (lane < kWinBatch && i < i1) {
            if (cf != SMX_NONE && cfs < 0)
                mya = win_upd(acv, i == r, cf == c, s_prcf, myc, e);
            mul[(int64_t)i * kBlkMax + D] = myc;
            mT[(int64_t)D * (rows + 1) + i] = myc;
            if (want_x) {
                if (i == hx0) xhist[hslot] = mybv;
                if (i == hx1) xhist[hslot + 1] = mybv;
            }
            blk_rec_add(R, i, mybv, cf != SMX_NONE, mya);
        }
    }
    SMX_BLK_STAMP(5);
    {
        // the workgroup's record: DPP per wave, then wave 0 merges the eight (total orders)
        __shared__ BlkRec s_r[kWinWaves];
        const int n0 = wave_min_int_dpp(R.nb);
        const First f0 = wave_first_dpp(R.f);
        const Cand c0 = wave_best_dpp(R.bc);
        if (lane == 0) s_r[wid] = BlkRec{n0, f0, c0};
        // LDS only: the row pass's stores need not land before the record goes out (the kernel's
        // end waits for them anyway)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (tid == 0) {
            BlkRec a = s_r[0];
            for (int w = 1; w < kWinWaves; ++w) {
                a.nb = min(a.nb, s_r[w].nb);
                if (s_r[w].f.idx < a.f.idx) a.f = s_r[w].f;
                if (better(s_r[w].bc, a.bc)) a.bc = s_r[w].bc;
            }
            smx_part pt;
            pt.p1col = a.nb;
            pt.first = a.f.idx;
            pt.first_v = a.f.v;
            pt.best_cls = a.bc.cls;
            pt.best_i = a.bc.idx;
            pt.best_v = a.bc.v;
            parts[(int64_t)blk_slot(L, P, bn) * G + b] = pt;
        }
    }
    SMX_BLK_STAMP(7);
}

// After a block's last planner step: the pivot rows at every column, pr[q][j] = T_{k+q}[r_q][j]
// (the sweep's and the pivot-column pass's operands), and the sweep's per-row flags (blk_rflags)
// when the block applied all P of its pivots.  Every column is one quad of lanes: lane k of the
// quad holds the pivot rows s = 4u + k (u < kQ) of that column; step q takes pivot row q's value
// from its lane (ds_bpermute) and every lane applies pivot q to its later pivot rows, with the
// pivot rows' multipliers (mul[r_s][q]) and the reciprocals in LDS.  (One column per thread with a
// global load per element update took 45.7 us per 20-pivot block at 16384^2, with the
// multipliers in LDS 34.7 us, profiles/r06d/, r06f/: one wave per SIMD on a quarter of the chip,
// each lane a 190-step triangle.)  The division is the hoisted-reciprocal sequence while every
// numerator of the wave stays inside the exponent window (win_term, one vote), else the columns
// again with the IEEE division: the same bits either way (smx_block.hpp blk_chain_fd).
constexpr int kProwsNT = kUpdBlock;
constexpr int kProwsQ = kBlkMax / 4;   // pivot rows per lane
__global__ __launch_bounds__(kProwsNT) void k_blk_prows(const double* __restrict__ T, int64_t ld,
                                                        int rows, int m, int P,
                                                        const BlkHdr* __restrict__ h,
                                                        double* __restrict__ mul,
                                                        double* __restrict__ pr) {
    __shared__ BlkPiv s_pv;
    __shared__ double s_mp[kBlkMax][kBlkMax];   // [pivot row s][step q]: mul[r_s][q]
    __shared__ int s_ok;
    const int peff = h->peff;
    if (peff <= 0) return;
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    if (tid < peff) {
        s_pv.r[tid] = h->r[tid];
        s_pv.c[tid] = h->c[tid];
        s_pv.e[tid] = h->e[tid];
        s_pv.y[tid] = fd_prep(h->e[tid]).y;
    }
    if (tid == 0) s_ok = 1;
    __syncthreads();
    if (tid < peff && !fd_prep(s_pv.e[tid]).ok) s_ok = 0;   // (ordered by the barrier below)
    for (int t = tid; t < peff * peff; t += kProwsNT) {
        const int sr = t / peff, q = t % peff;
        s_mp[sr][q] = mul[(int64_t)s_pv.r[sr] * kBlkMax + q];
    }
    __syncthreads();
    const bool allok = s_ok != 0;
    const int C = m + 1;
    const int k = lane & 3;              // this lane's pivot rows: s = 4 u + k
    const int qbase = lane & ~3;         // the quad's first lane
    const int64_t ncol = (int64_t)gridDim.x * (kProwsNT / 4);
    for (int64_t j0 = (int64_t)blockIdx.x * (kProwsNT / 4); j0 < C; j0 += ncol) {
        const int jq = (int)j0 + (tid >> 2);
        const int j = jq < C ? jq : C - 1;   // (tail quads redo the last column)
        double x0[kProwsQ];
#pragma unroll
        for (int u = 0; u < kProwsQ; ++u) {
            const int sr = 4 * u + k;
            x0[u] = sr < peff ? T[(int64_t)s_pv.r[sr] * ld + j] : 0.0;
        }
        for (int exact = 0; exact < 2; ++exact) {
            double x[kProwsQ];
#pragma unroll
            for (int u = 0; u < kProwsQ; ++u) x[u] = x0[u];
            uint32_t wt = 0;
#pragma unroll 1
            for (int q = 0; q < peff; ++q) {
                // T_{k+q}[r_q][j]: slot q / 4 of quad lane q % 4 (updated by the q pivots before)
                const int uq = q >> 2;
                double mine = x[0];
#pragma unroll
                for (int u = 1; u < kProwsQ; ++u)
                    if (u == uq) mine = x[u];
                const double p = __shfl(mine, qbase | (q & 3));
                if (k == 0 && jq < C) pr[(int64_t)q * ld + j] = p;
                const int rq = s_pv.r[q];
                const bool pc = j == s_pv.c[q];
                const double e = s_pv.e[q], y = s_pv.y[q];
#pragma unroll
                for (int u = 0; u < kProwsQ; ++u) {
                    const int sr = 4 * u + k;
                    if (sr > q && sr < peff) {
                        const double a = x[u] * e;
                        const double b = p * s_mp[sr][q];
                        const bool prow = s_pv.r[sr] == rq;
                        const double num = prow ? (pc ? 1.0 : -x[u]) : (pc ? x[u] : (a - b));
                        if (exact) {
                            x[u] = num / e;
                        } else {
                            wt = max(wt, win_term(num));
                            const double tq = num * y;
                            const double rr = fma(-e, tq, num);
                            x[u] = fma(rr, y, tq);
                        }
                    }
                }
            }
            if (!exact && allok && __all(wt < kWinSpan)) break;   // every quotient exact
        }
    }
    if (peff != P) return;
    int32_t* fl = blk_rflags(mul, rows + 1);
    const int nt = (int)gridDim.x * kProwsNT;
    for (int i = (int)blockIdx.x * kProwsNT + tid; i <= rows; i += nt) {
        const double* mr = mul + (int64_t)i * kBlkMax;
        bool bnd = true, zero = false, piv = false;
#pragma unroll
        for (int q = 0; q < kBlkMax; ++q) {
            if (q < P) {
                const double v = mr[q];
                bnd = bnd && bnd_or_zero(v);
                zero = zero || (dbits(v) << 1) == 0;
                piv = piv || i == s_pv.r[q];
            }
        }
        fl[i] = blk_rflag(piv, bnd, zero);
    }
}

}  // namespace
