// smx_plan.hpp -- the persistent planner: ONE launch decides all P pivots of a block
// (pick_element, simplex.py:70-141, for block steps 0..P-1) instead of P launches of k_blk_step.
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------------------------------------
// Why: a k_blk_step launch is ~4 dependent memory round trips plus a kernel boundary (launch gap
// ~1.4 us, the records re-read from memory by the next launch): 13-16 us per pivot at 16384^2,
// the planner's ~18 us per pivot at P = 20 next to a ~70 us share of the sweep.  Here the same
// G workgroups (blk_parts_of) stay resident for the whole block, every thread owning ONE row:
//   * step L's records go out as tagged 8-B granules (st_sc1: payload and tag in one store, the
//     resident loop's form), and step L+1 polls them -- no kernel boundary between steps;
//   * a row's multipliers mul[i][0..D) and its cached T_{k+D}[i][m] / T_{k+D}[i][cf] stay in
//     registers across steps (the launch form re-reads them: the transposed copy mT and the
//     column caches);
//   * the pivot list (r, c, e) and the next entering column live in LDS, identical in every
//     workgroup (every workgroup reaches the same decisions), so no header is re-read;
//   * what other workgroups do read within the launch -- the pivot-row and f-row slices, the
//     pivot row's multipliers -- is stored write-through (agent-scope relaxed stores, sc1) and
//     drained (s_waitcnt vmcnt(0)) before the workgroup's record, and loaded with agent-scope
//     loads (MI355X_MICROARCH.md: sc1 payload -> drain -> sc1 flag; no release / acquire fence).
// Same decisions, same operations on the same operands in the same order as k_blk_step (the
// chains, the fast-division window, the scans): the same bits (tests/test_gpu_block.py runs the
// block suites with smx_tune_block_persist(1) against the launch form and the C oracle).
// Eligible: unsharded, unpipelined chains with at most one row per thread (rows <= G x 256: up to
// 65,536 rows).  Tags: (pepoch << 8) | step, pepoch = launches of this scratch so far (BlkHdr,
// bumped by workgroup 0 at the end of every launch), so a graph replay never meets its own
// previous replay's granules.  Every spin is bounded (g_plan_spin_ticks): on a timeout the chain
// stops with ctl->dec[0][0] |= kResTimeout, like the resident loop.

constexpr int kPlanRecWords = 8;                 // a record as 8 granules of 32-bit payload
__device__ int64_t g_plan_spin_ticks = 2000000000;   // 20 s of s_memrealtime (100 MHz)

__device__ __forceinline__ double ld_ag(const double* p) {
    return bitsd(ld_sc1(reinterpret_cast<const uint64_t*>(p)));
}
__device__ __forceinline__ void st_ag(double* p, double v) {
    st_sc1(reinterpret_cast<uint64_t*>(p), dbits(v));
}

// blk_chain_fd / blk_chain / blk_pv_regs with runtime step bounds (steps q0 <= q < q1), loops
// unrolled to NM with uniform guards: one kernel body serves every step of a block (a body per
// step, as k_blk_step has, made the persistent kernels' compile time quadratic in P)
template <int NM>
__device__ __forceinline__ double plan_chain_fd(double x, int i, int j, const BlkPiv& pv,
                                                const double* p, const double* mq, uint32_t& wt,
                                                int q0, int q1) {
#pragma unroll
    for (int q = 0; q < NM; ++q) {
        if (q < q0 || q >= q1) continue;
        const double e = pv.e[q];
        const double a = x * e;
        const double b = p[q] * mq[q];
        const bool jc = j == pv.c[q];
        const double num = (i == pv.r[q]) ? (jc ? 1.0 : -x) : (jc ? x : (a - b));
        wt = max(wt, win_term(num));
        const double t = num * pv.y[q];
        const double r = fma(-e, t, num);
        x = fma(r, pv.y[q], t);
    }
    return x;
}
template <int NM>
__device__ __forceinline__ double plan_chain(double x, int i, int j, const BlkPiv& pv,
                                             const double* p, const double* mq, int q0, int q1) {
#pragma unroll
    for (int q = 0; q < NM; ++q) {
        if (q < q0 || q >= q1) continue;
        const double e = pv.e[q];
        const double a = x * e;
        const double b = p[q] * mq[q];
        const bool jc = j == pv.c[q];
        const double num = (i == pv.r[q]) ? (jc ? 1.0 : -x) : (jc ? x : (a - b));
        x = num / e;
    }
    return x;
}
template <int NM>
__device__ __forceinline__ BlkPiv plan_pv_regs(const BlkPiv& s, int n, bool* allok) {
    BlkPiv v;
#pragma unroll
    for (int q = 0; q < NM; ++q) {
        v.r[q] = q < n ? s.r[q] : -1;
        v.c[q] = q < n ? s.c[q] : -1;
        v.e[q] = q < n ? s.e[q] : 1.0;
    }
#pragma unroll
    for (int q = 0; q < NM; ++q) {
        blk_pin(v.r[q]);
        blk_pin(v.c[q]);
        blk_pin(v.e[q]);
    }
    bool ok = true;
#pragma unroll
    for (int q = 0; q < NM; ++q) {
        const FastDiv f = fd_prep(v.e[q]);
        v.y[q] = f.y;
        ok = ok && (q >= n || f.ok);
    }
    *allok = ok;
    return v;
}

__device__ __forceinline__ void plan_rec_put(uint64_t* d, const smx_part& pt, uint32_t tag) {
    const uint64_t t = (uint64_t)tag << 32;
    const uint64_t fv = dbits(pt.first_v), bv = dbits(pt.best_v);
    st_sc1(d + 0, t | (uint32_t)pt.p1col);
    st_sc1(d + 1, t | (uint32_t)pt.first);
    st_sc1(d + 2, t | (uint32_t)fv);
    st_sc1(d + 3, t | (uint32_t)(fv >> 32));
    st_sc1(d + 4, t | (uint32_t)pt.best_cls);
    st_sc1(d + 5, t | (uint32_t)pt.best_i);
    st_sc1(d + 6, t | (uint32_t)bv);
    st_sc1(d + 7, t | (uint32_t)(bv >> 32));
}

// One wave: the G records of a step from their granules, polled until every tag is `want` (all
// loads of a round in flight together), then merged like blk_merge_records.  false: timed out.
__device__ __forceinline__ bool plan_merge_granules(const uint64_t* __restrict__ xr, int G,
                                                    uint32_t want, int& nb, First& f, Cand& bb) {
    constexpr int U = kBlkPartsMax / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    uint64_t w[U][kPlanRecWords];
    const int64_t t0 = rt_now();
    bool done = false;
    for (;;) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = lane + u * kWave;
#pragma unroll
            for (int q = 0; q < kPlanRecWords; ++q)
                w[u][q] = k < G ? ld_sc1(xr + (int64_t)k * kPlanRecWords + q)
                                : ((uint64_t)want << 32);
        }
        bool ok = true;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < kPlanRecWords; ++q) ok = ok && (uint32_t)(w[u][q] >> 32) == want;
        if (__all(ok)) {
            done = true;
            break;
        }
        if (rt_now() - t0 > g_plan_spin_ticks) break;
        __builtin_amdgcn_s_sleep(1);
    }
    int n = SMX_NONE;
    First fi{SMX_NONE, 0.0};
    Cand b = cand_none();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (lane + u * kWave >= G) continue;
        const int p1 = (int)(uint32_t)w[u][0];
        const int first = (int)(uint32_t)w[u][1];
        const double fv = bitsd((w[u][2] & 0xffffffffull) | (w[u][3] << 32));
        const Cand o{(int)(uint32_t)w[u][4], (int)(uint32_t)w[u][5],
                     bitsd((w[u][6] & 0xffffffffull) | (w[u][7] << 32))};
        n = min(n, p1);
        if (first < fi.idx) fi = First{first, fv};
        if (better(o, b)) b = o;
    }
    nb = wave_min_int_dpp(n);
    f = wave_first_dpp(fi);
    bb = wave_best_dpp(b);
    return done;
}

struct PlanArgs {
    const double* T;
    int64_t ld;
    int rows, m, flen, fscan, P, parity, bn;
    smx_ctl* ctl;
    BlkHdr* h;
    smx_part* parts;
    double *mul, *pr, *fr;
    int32_t* log;
    double* xhist;
    int64_t log_cap;
    uint64_t* xr;
    uint32_t epoch;
    int64_t kpiv0;
};

// Per-workgroup state shared by the steps (LDS): identical in every workgroup
struct PlanSh {
    BlkPiv pv;                   // the block's pivots so far: local row, column, element
    double col[3][kBlkMax];      // pr_q at the columns c, m, cf of the current step
    int tmp[kBlkNT / kWave];
    Decision d;
    int nb, cdec, cnext;         // step D's first negative "-b" row and records' column; step
                                 // L's entering column (the records' column of step L)
    int stop;                    // 2: a hand-off timed out
    double e, fc, pm, pa;
};

// Block step D = L - 1 (L = 1..P at run time; NM = P bounds the unrolled loops): decide it, build
// the records of step L.  mq / cb / ca / hx0 / hx1: this thread's row state across steps.
// true: the launch ends here.
template <int NM>
__device__ __forceinline__ bool blk_pstep(const PlanArgs& a, PlanSh& S, const int L,
                                          double (&mq)[NM], double& cb, double& ca, int& hx0,
                                          int& hx1) {
    constexpr int NT = kBlkNT;
    const int D = L - 1;
    const int tid = threadIdx.x;
    const int b = blockIdx.x, G = gridDim.x;
    const int P = a.P, rows = a.rows, m = a.m, flen = a.flen, fscan = a.fscan, bn = a.bn;
    const int64_t ld = a.ld;
    const double* __restrict__ T = a.T;
    double* __restrict__ mul = a.mul;
    double* __restrict__ pr = a.pr;
    smx_ctl* __restrict__ ctl = a.ctl;
    const int sp = (a.parity + D) & 1;
    const int C = m + 1;
    SMX_BLK_STAMP(0);
    if (tid < kWave) {
        // the decision of step D from its records: the previous launch's (D = 0, in `parts`) or
        // this launch's step D granules (every workgroup, identically)
        const int c = D == 0 ? a.h->cfs[blk_slot(0, P, bn)] : S.cnext;
        int nb;
        First f;
        Cand bb;
        bool ok = true;
        if (D == 0)
            blk_merge_records(a.parts + (int64_t)blk_slot(0, P, bn) * G, G, nb, f, bb);
        else
            ok = plan_merge_granules(a.xr + (int64_t)(D & 1) * kBlkPartsMax * kPlanRecWords, G,
                                     (a.epoch << 8) | (uint32_t)D, nb, f, bb);
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
            d.r = nb;                  // phase 1: the column comes from the row scan below
            d.c = SMX_NONE;
        }
        if (tid == 0) {
            S.nb = nb;
            S.d = d;
            S.cdec = c;
            S.stop = ok ? 0 : 2;
        }
    }
    __syncthreads();
    SMX_BLK_STAMP(1);
    if (S.stop == 2) {   // a workgroup's record never came: leave, report it (like k_resident)
        if (tid == 0) {
            atomicOr(&ctl->dec[0][0], kResTimeout);
            ctl->term = 1;
        }
        return true;
    }
    const int nb = S.nb;
    Decision d = S.d;
    auto terminal = [&](const Decision& dd) {
        if (b == 0 && tid == 0) {
            ctl->sel_status = dd.status;
            ctl->sel_r = dd.r;
            ctl->sel_c = dd.c;
            ctl->negb[sp] = nb;        // the state of T_{k+D}, where the chain stops
            ctl->negf[sp] = S.cdec;
            ctl->term = 1;
            a.h->peff = D;
        }
    };
    if (d.status != SMX_PIVOT) {
        terminal(d);
        return true;
    }
    const int r = d.r;             // pivot row (unsharded: local = global)
    double mqr[NM];                // the pivot row's multipliers (its owner stored them)
#pragma unroll
    for (int q = 0; q < NM; ++q) mqr[q] = q < D ? ld_ag(mul + (int64_t)r * kBlkMax + q) : 0.0;
#pragma unroll
    for (int q = 0; q < NM; ++q) blk_pin(mqr[q]);
    bool okD = true;
    const BlkPiv pvD = plan_pv_regs<NM>(S.pv, D, &okD);
    auto prv = [&](int j) -> double {   // T_{k+D}[r][j]
        double x = T[(int64_t)r * ld + j];
        double p[NM];
#pragma unroll
        for (int q = 0; q < NM; ++q) p[q] = q < D ? ld_ag(pr + (int64_t)q * ld + j) : 0.0;
#pragma unroll
        for (int q = 0; q < NM; ++q) blk_pin(p[q]);
        blk_pin(x);
        uint32_t wt = 0;
        const double v = plan_chain_fd<NM>(x, r, j, pvD, p, mqr, wt, 0, D);
        if (okD && __all(wt < kWinSpan)) return v;
        return plan_chain<NM>(x, r, j, pvD, p, mqr, 0, D);
    };
    const double* fo = a.fr + (int64_t)sp * ld;          // f-row of T_{k+D}
    double* fn = a.fr + (int64_t)(sp ^ 1) * ld;          // f-row of T_{k+L}
    double* prD = pr + (int64_t)D * ld;
    int c, cf;
    double e, fc;
    if (nb == SMX_NONE) {
        // phase 2: row r's operands for the pivot element, the "-b" column, this thread's slice
        // column and its first-round scan column in ONE round trip (blk_step_body's fast path)
        c = d.c;
        const double* Tr = T + (int64_t)r * ld;
        const int Sw = ((C + G - 1) / G + 1) & ~1;
        const int s0 = b * Sw, s1 = min(C, s0 + Sw);
        constexpr int NSC = NT >= 128 ? 1 : 128 / NT;
        constexpr int NJ = 2 + NSC;
        int jj[NJ];
        jj[0] = (tid & 1) ? m : c;
        jj[1] = s0 + tid;
#pragma unroll
        for (int k = 0; k < NSC; ++k) jj[2 + k] = tid + k * NT;
        double x[NJ], pq[NJ][NM], fv[NJ];
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
            const int jc = min(jj[u], C - 1);
            x[u] = Tr[jc];
            fv[u] = ld_ag(fo + jc);
#pragma unroll
            for (int q = 0; q < NM; ++q) pq[u][q] = q < D ? ld_ag(pr + (int64_t)q * ld + jc) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
            blk_pin(x[u]);
            blk_pin(fv[u]);
#pragma unroll
            for (int q = 0; q < NM; ++q) blk_pin(pq[u][q]);
        }
        double v[NJ];
        uint32_t wt = 0;
#pragma unroll
        for (int u = 0; u < NJ; ++u)
            v[u] = plan_chain_fd<NM>(x[u], r, jj[u], pvD, pq[u], mqr, wt, 0, D);
        if (!okD || !__all(wt < kWinSpan)) {
            SMX_BLK_FALLBACK(0);
#pragma unroll
            for (int u = 0; u < NJ; ++u)
                v[u] = plan_chain<NM>(x[u], r, jj[u], pvD, pq[u], mqr, 0, D);
        }
        e = blk_readlane(v[0], 0);
        fc = blk_readlane(fv[0], 0);
        SMX_BLK_STAMP(2);
        if (jj[1] < s1) {
            st_ag(prD + jj[1], v[1]);
            st_ag(fn + jj[1], blk_fnew(fv[1], v[1], jj[1], c, e, fc));
        }
        for (int j = s0 + tid + NT; j < s1; j += NT) {
            const double vv = prv(j);
            st_ag(prD + j, vv);
            st_ag(fn + j, blk_fnew(ld_ag(fo + j), vv, j, c, e, fc));
        }
        SMX_BLK_STAMP(3);
        int mine = SMX_NONE;
#pragma unroll
        for (int k = NJ - 1; k >= 2; --k)
            if (jj[k] < fscan && blk_fnew(fv[k], v[k], jj[k], c, e, fc) < 0.0) mine = jj[k];
        cf = block_min_int_dpp<NT>(mine, S.tmp);
        if (cf != SMX_NONE) {
            if (tid == cf % NT) {
#pragma unroll
                for (int k = 2; k < NJ; ++k)
                    if (k - 2 == cf / NT) {
                        S.pa = v[k];
#pragma unroll
                        for (int q = 0; q < NM; ++q)
                            if (q < D) S.col[2][q] = pq[k][q];
                    }
            }
        } else {
            for (int j0 = NSC * NT; j0 < fscan && cf == SMX_NONE; j0 += kBlkScan) {
                int mn = SMX_NONE;
#pragma unroll 4
                for (int k = 0; k < 4; ++k) {
                    const int j = j0 + k * NT + tid;
                    if (j < fscan && blk_fnew(ld_ag(fo + j), prv(j), j, c, e, fc) < 0.0 && j < mn)
                        mn = j;
                }
                cf = block_min_int_dpp<NT>(mn, S.tmp);
            }
            if (tid == 0) {
                S.pa = cf != SMX_NONE ? prv(cf) : 0.0;
                if (cf != SMX_NONE)
                    for (int q = 0; q < D; ++q) S.col[2][q] = ld_ag(pr + (int64_t)q * ld + cf);
            }
        }
        if (tid < 2) {   // lane 0 holds column c's operands, lane 1 column m's
            if (tid == 1) S.pm = v[0];
#pragma unroll
            for (int q = 0; q < NM; ++q)
                if (q < D) S.col[tid][q] = pq[0][q];
        }
        SMX_BLK_STAMP(4);
    } else {
        // phase 1: first j < m with T_{k+D}[r][j] > 0 (simplex.py:81-85), early exit by rounds
        int p1 = SMX_NONE;
        for (int j0 = 0; j0 < m && p1 == SMX_NONE; j0 += kBlkScan) {
            int mine = SMX_NONE;
#pragma unroll 4
            for (int k = 0; k < 4; ++k) {
                const int j = j0 + k * NT + tid;
                if (j < m && prv(j) > 0.0 && j < mine) mine = j;
            }
            p1 = block_min_int_dpp<NT>(mine, S.tmp);
        }
        if (p1 == SMX_NONE) {
            d.c = SMX_NONE;
            d.status = SMX_INCORRECT;   // simplex.py:88-89
            terminal(d);
            return true;
        }
        d.c = p1;
        c = d.c;
        if (tid == 0) {
            S.e = prv(c);
            S.fc = ld_ag(fo + c);
            S.pm = prv(m);
        }
        __syncthreads();
        SMX_BLK_STAMP(2);
        e = S.e;
        fc = S.fc;
        {
            const int Sw = ((C + G - 1) / G + 1) & ~1;
            const int s1 = min(C, (b + 1) * Sw);
            for (int j = b * Sw + tid; j < s1; j += NT) {
                const double v = prv(j);
                st_ag(prD + j, v);
                st_ag(fn + j, blk_fnew(ld_ag(fo + j), v, j, c, e, fc));
            }
        }
        SMX_BLK_STAMP(3);
        cf = SMX_NONE;
        for (int j0 = 0; j0 < fscan && cf == SMX_NONE; j0 += kBlkScan) {
            int mine = SMX_NONE;
#pragma unroll 4
            for (int k = 0; k < 4; ++k) {
                const int j = j0 + k * NT + tid;
                if (j < fscan && blk_fnew(ld_ag(fo + j), prv(j), j, c, e, fc) < 0.0 && j < mine)
                    mine = j;
            }
            cf = block_min_int_dpp<NT>(mine, S.tmp);
        }
        SMX_BLK_STAMP(4);
        if (tid == 0) S.pa = cf != SMX_NONE ? prv(cf) : 0.0;
        if (tid < D) {
            S.col[0][tid] = ld_ag(pr + (int64_t)tid * ld + c);
            S.col[1][tid] = ld_ag(pr + (int64_t)tid * ld + m);
            if (cf != SMX_NONE) S.col[2][tid] = ld_ag(pr + (int64_t)tid * ld + cf);
        }
    }
    // the labels after this pivot (simplex.py:152), identically in every workgroup
    hx0 = move_label(hx0, r, c);
    hx1 = move_label(hx1, r, c);
    const int64_t kpiv = a.kpiv0 + D;
    if (b == 0 && tid == 0) {
        const FastDiv fd = fd_prep(e);
        mul[(int64_t)rows * kBlkMax + D] = fc;
        if (L == P) {   // the f-row's sweep flag: never a pivot row; its multipliers are the fc's
            bool bnd = bnd_or_zero(fc), zero = (dbits(fc) << 1) == 0;
            for (int q = 0; q < D; ++q) {
                const double v = mul[(int64_t)rows * kBlkMax + q];
                bnd = bnd && bnd_or_zero(v);
                zero = zero || (dbits(v) << 1) == 0;
            }
            blk_rflags(mul, rows + 1)[rows] = blk_rflag(false, bnd, zero);
        }
        a.h->r[D] = r;
        a.h->c[D] = c;
        a.h->e[D] = e;
        a.h->y[D] = fd.y;
        a.h->ok[D] = fd.ok ? 1 : 0;
        a.h->peff = D + 1;
        a.h->cfs[blk_slot(L, P, bn)] = cf;
        if (a.log_cap > 0) {
            a.log[2 * (kpiv % a.log_cap)] = r;
            a.log[2 * (kpiv % a.log_cap) + 1] = c;
        }
        ctl->npivots = kpiv + 1;
        ctl->npiv[sp ^ 1] = kpiv + 1;
        ctl->sel_status = SMX_PIVOT;
        ctl->sel_r = r;
        ctl->sel_c = c;
        ctl->sel_e = e;
        ctl->xpos[sp ^ 1][0] = hx0;
        ctl->xpos[sp ^ 1][1] = hx1;
        if (a.xhist && a.log_cap > 0) {              // non-basic labels: 0 (simplex.py:60-66)
            if (hx0 < 0) a.xhist[2 * (kpiv % a.log_cap)] = 0.0;
            if (hx1 < 0) a.xhist[2 * (kpiv % a.log_cap) + 1] = 0.0;
        }
    }
    __syncthreads();   // S.pa / S.pm / S.col of the scans are written before this
    if (tid == 0) {
        S.pv.r[D] = r;
        S.pv.c[D] = c;
        S.pv.e[D] = e;
        S.col[1][D] = S.pm;
        S.col[2][D] = S.pa;
        S.cnext = cf;
    }
    __syncthreads();
    SMX_BLK_STAMP(5);
    const int64_t hslot = 2 * (kpiv % (a.log_cap > 0 ? a.log_cap : 1));
    bool okL = true;
    const BlkPiv pvL = plan_pv_regs<NM>(S.pv, L, &okL);
    double colv[3][NM];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int q = 0; q < NM; ++q) colv[k][q] = q < L ? S.col[k][q] : 0.0;
#pragma unroll
        for (int q = 0; q < NM; ++q) blk_pin(colv[k][q]);
    }
    // the row pass: this thread's row i, its multipliers and cached columns from registers
    const bool reuse_c = D > 0 && c == S.cdec;   // phase 2: c is the column of step D's records
    BlkRec R{SMX_NONE, First{SMX_NONE, 0.0}, cand_none()};
    const int i = b * NT + tid;
    if (i < rows) {
        const double* row = T + (int64_t)i * ld;
        const double xc = reuse_c ? ca : row[c];
        const double xb = D > 0 ? cb : row[m];
        const double xa = cf != SMX_NONE ? row[cf] : 0.0;
        double x3[3] = {xc, xb, xa};
#pragma unroll
        for (int k = 0; k < 3; ++k) blk_pin(x3[k]);
        uint32_t wt = 0;
        // x3[1]: T_{k+D}[i][m] (cached) from step 1 on -- one step; T_k[i][m] at step 0
        const double md = reuse_c ? x3[0] : plan_chain_fd<NM>(x3[0], i, c, pvL, colv[0], mq, wt, 0, D);
#pragma unroll
        for (int q = 0; q < NM; ++q)
            if (q == D) mq[q] = md;
        double bv = plan_chain_fd<NM>(x3[1], i, m, pvL, colv[1], mq, wt, D > 0 ? D : 0, L);
        double av = cf != SMX_NONE ? plan_chain_fd<NM>(x3[2], i, cf, pvL, colv[2], mq, wt, 0, L)
                                   : 0.0;
        if (!okL || !__all(wt < kWinSpan)) {   // some numerator outside the window
            SMX_BLK_FALLBACK(1);
            if (!reuse_c) {
                const double m2 = plan_chain<NM>(x3[0], i, c, pvL, colv[0], mq, 0, D);
#pragma unroll
                for (int q = 0; q < NM; ++q)
                    if (q == D) mq[q] = m2;
            }
            bv = plan_chain<NM>(x3[1], i, m, pvL, colv[1], mq, D > 0 ? D : 0, L);
            av = cf != SMX_NONE ? plan_chain<NM>(x3[2], i, cf, pvL, colv[2], mq, 0, L) : 0.0;
        }
        double mD = 0.0;
#pragma unroll
        for (int q = 0; q < NM; ++q)
            if (q == D) mD = mq[q];
        st_ag(mul + (int64_t)i * kBlkMax + D, mD);   // read as mqr should row i pivot later
        // the transposed copy, for the sweep's pivot-column pass (blk_fixcols; after this launch)
        blk_mulT(mul, rows + 1)[(int64_t)D * (rows + 1) + i] = mD;
        cb = bv;
        ca = av;
        if (L == P) {   // the sweep's per-row flag (blk_rflags)
            bool bnd = true, zero = false, piv = false;
#pragma unroll
            for (int q = 0; q < NM; ++q) {
                if (q >= L) continue;
                bnd = bnd && bnd_or_zero(mq[q]);
                zero = zero || (dbits(mq[q]) << 1) == 0;
                piv = piv || i == pvL.r[q];
            }
            blk_rflags(mul, rows + 1)[i] = blk_rflag(piv, bnd, zero);
        }
        if (a.xhist && a.log_cap > 0) {
            if (i == hx0) a.xhist[hslot] = bv;
            if (i == hx1) a.xhist[hslot + 1] = bv;
        }
        blk_rec_add(R, i, bv, cf != SMX_NONE, av);
    }
    SMX_BLK_STAMP(6);
    // every store another workgroup reads (slices, multipliers) has landed before the record
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const smx_part pt = blk_rec_reduce(R);
    if (tid == 0) {
        if (L < P)
            plan_rec_put(a.xr + ((int64_t)(L & 1) * kBlkPartsMax + b) * kPlanRecWords, pt,
                         (a.epoch << 8) | (uint32_t)L);
        else   // the next block's first step: read by the next launch
            a.parts[(int64_t)blk_slot(L, P, bn) * G + b] = pt;
    }
    SMX_BLK_STAMP(7);
    return false;
}

// The P planner steps of one block (unsharded, unpipelined; rows <= gridDim.x * kBlkNT)
template <int P>
__global__ __launch_bounds__(kBlkNT) void k_blk_plan(const double* __restrict__ T, int64_t ld,
                                                     int rows, int m, int flen, int fscan,
                                                     int parity, int bn,
                                                     smx_ctl* __restrict__ ctl,
                                                     BlkHdr* __restrict__ h,
                                                     smx_part* __restrict__ parts,
                                                     double* __restrict__ mul,
                                                     double* __restrict__ pr,
                                                     double* __restrict__ fr,
                                                     int32_t* __restrict__ log,
                                                     double* __restrict__ xhist, int64_t log_cap,
                                                     uint64_t* __restrict__ xr) {
    __shared__ PlanSh S;
    if (ctl->term) {   // a stopped chain: nothing to plan (a later block of a stopped chain)
        if (blockIdx.x == 0 && threadIdx.x == 0) h->peff = 0;
        return;
    }
    const uint32_t epoch = (h->pepoch + 1u) & 0xffffffu;
    const PlanArgs a{T, ld, rows, m, flen, fscan, P, parity, bn, ctl, h, parts, mul, pr, fr,
                     log, xhist, log_cap, xr, epoch, ctl->npiv[parity]};
    double mq[P];
#pragma unroll
    for (int q = 0; q < P; ++q) mq[q] = 0.0;
    double cb = 0.0, ca = 0.0;
    int hx0 = ctl->xpos[parity][0], hx1 = ctl->xpos[parity][1];
    for (int L = 1; L <= P; ++L)
        if (blk_pstep<P>(a, S, L, mq, cb, ca, hx0, hx1)) break;
    // every workgroup has read pepoch: the last step waited for every workgroup's records of
    // the step before (P >= 2); at P = 1 no granule is used
    if (blockIdx.x == 0 && threadIdx.x == 0) h->pepoch = epoch;
}

}  // namespace
