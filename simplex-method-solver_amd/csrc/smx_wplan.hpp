// smx_wplan.hpp -- the window planner as ONE persistent launch per block (k_blk_wplan).
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

// Why.  The launch form of the window planner (k_blk_wstep, smx_window.hpp) pays per step a
// kernel boundary (~1.5 us plus the dirty bytes it leaves: the window it rewrites, 8 MB at 16384
// rows, MI355X_MICROARCH.md "boundary"), a full read and write of that window, and the record
// round trip after every boundary: ~13.7 us per step at 16384^2 (profiles/r06l/).  Here every
// workgroup keeps its rows' window in REGISTERS for the whole block and the steps hand off
// through tagged 8-byte granules ({32-bit payload, 32-bit tag}, relaxed agent-scope = sc1 stores
// and loads, the resident loop's protocol, smx_resident.hpp).  Per step:
//   * every workgroup publishes its record (4 granules) and its CANDIDATE pivot row -- the row
//     its record would nominate (phase 1: its first row with a negative "-b"; phase 2: its
//     ratio-test winner, or its first candidate when that ratio is NaN) -- with that row's window
//     and multipliers (each wave stages its own candidate's window in LDS; the merging wave
//     publishes the workgroup's);
//   * one wave per workgroup polls all records, decides (every workgroup identically), then
//     fetches the winner's window from the owning workgroup's candidate slot -- one more round
//     trip, the bytes already published.  Where the owner's candidate is another row (a NaN first
//     candidate in another wave, the block's first step) the owner publishes the pivot row on
//     demand instead.  (One candidate per wave cost 2,048 x 1.4 KB of write-through granules per
//     step -- ~70 MB per block that the following sweep paid for in HBM traffic: 469 vs 440 us
//     per 24-pivot sweep at 8192^2, profiles/r06r/.)
//   * every wave applies the pivot to its rows in registers.
// No window traffic, no boundary; the pivots, multipliers, log and x-history go out as in the
// launch form (plain stores, read after the kernel).  Co-residency: one workgroup per CU (G <=
// CUs, launched only then); every spin is bounded (g_res_spin_ticks): a workgroup that times out
// latches kResTimeout in ctl->dec[0][0], stops the chain and leaves at its next barrier, so the
// grid always drains, and the host reports it.
// A record travels as 4 granules (16 B of payload): the three row indices in 16 bits each
// (0xFFFF = none; eligible tables have at most 32,768 rows), the best candidate's class, whether
// the first candidate's ratio is NaN (the only use of its value, the decision's simplex.py:117-121
// test) and the best candidate's ratio.
constexpr int kWpRecG = 4;
constexpr int kWpRowG = 2 * kWin + 2 * kBlkMax;       // on-demand pivot row: window, multipliers
constexpr int kWpCandG = 2 + 2 * kWin + 2 * kBlkMax;  // a candidate: row, window, multipliers
constexpr int kWpMaxRpw = 16;                         // rows per wave in registers (32,768 rows)

// The pivot rows at every column (the sweep's operands, k_blk_prows' job) are built inside the
// launch when every workgroup's column slice fits one wave: ceil(C / G) <= 64 columns
__host__ __device__ __forceinline__ int wp_cols_per_group(int C, int G) { return (C + G - 1) / G; }
__host__ __device__ __forceinline__ bool wp_inpr(int C, int G) {
    return wp_cols_per_group(C, G) <= kWave;
}

// scratch (uint64 granules): records [2 parities][kWinMaxG][kWpRecG], on-demand pivot rows
// [2][kWpRowG], candidates [2][G][kWpCandG] (blk_xg_used(G) of them)
static_assert((2 * kWinMaxG * kWpRecG + 2 * kWpRowG + 2 * kWinMaxG * kWpCandG) * 8 ==
                  kBlkXgBytes,
              "granule scratch");

__device__ __forceinline__ uint32_t wp_idx16(int i) { return i == SMX_NONE ? 0xFFFFu : (uint32_t)i; }
__device__ __forceinline__ int wp_idx(uint32_t v) { return v == 0xFFFFu ? SMX_NONE : (int)v; }
__device__ __forceinline__ uint32_t wp_pack1(const BlkRec& a, int g) {
    if (g == 0) return wp_idx16(a.nb) | (wp_idx16(a.f.idx) << 16);
    if (g == 1)
        return wp_idx16(a.bc.idx) | ((uint32_t)a.bc.cls << 16) |
               ((a.f.idx != SMX_NONE && isnan(a.f.v)) ? 1u << 18 : 0u);
    const uint64_t v = dbits(a.bc.v);
    return g == 2 ? (uint32_t)v : (uint32_t)(v >> 32);
}
__device__ __forceinline__ smx_part wp_unpack(const uint64_t* w) {
    smx_part pt;
    pt.p1col = wp_idx((uint32_t)w[0] & 0xFFFFu);
    pt.first = wp_idx((uint32_t)w[0] >> 16);
    pt.first_v = ((uint32_t)w[1] >> 18) & 1u ? __builtin_nan("") : 0.0;
    pt.best_i = wp_idx((uint32_t)w[1] & 0xFFFFu);
    pt.best_cls = (int)(((uint32_t)w[1] >> 16) & 3u);
    pt.best_v = bitsd(((w[3] & 0xFFFFFFFFull) << 32) | (w[2] & 0xFFFFFFFFull));
    return pt;
}
constexpr uint64_t kWpTagMask = 0xFFFFFFFF00000000ull;
__device__ __forceinline__ bool wp_tagged(uint64_t w, uint64_t tag) { return (w & kWpTagMask) == tag; }
__device__ __forceinline__ double wp_val(uint64_t lo, uint64_t hi) {
    return bitsd((hi << 32) | (lo & 0xFFFFFFFFull));
}
__device__ __forceinline__ void wp_put(uint64_t* p, uint64_t tag, double v) {
    const uint64_t bits = dbits(v);
    st_sc1(p, tag | (uint32_t)bits);
    st_sc1(p + 1, tag | (uint32_t)(bits >> 32));
}
// Branches a step almost never takes (fallbacks for columns outside the window, the exact
// division's redo, time-outs, terminal steps): laid out after the hot path
#define WP_COLD(x) __builtin_expect(!!(x), 0)
// s_sleep operand between two polls of a hand-off (x 64 cycles; a build knob for power A/Bs)
#ifndef WP_POLL_SLEEP
#define WP_POLL_SLEEP 1
#endif

// The row a record would nominate as the pivot row if it won the decision
__device__ __forceinline__ int wp_nominee(int nb, const First& f, const Cand& bc) {
    return nb != SMX_NONE ? nb
         : (f.idx != SMX_NONE && isnan(f.v)) ? f.idx
         : (bc.cls < 2 ? bc.idx : SMX_NONE);
}

// Records of the 8 waves (lanes 0..7 of wave 0, one each): merged in every lane of the group
template <int CTRL>
__device__ __forceinline__ BlkRec wp_rec_dpp(const BlkRec& a) {
    BlkRec o;
    o.nb = dpp_i<CTRL>(a.nb);
    o.f = dpp_first<CTRL>(a.f);
    o.bc = dpp_cand<CTRL>(a.bc);
    return o;
}
__device__ __forceinline__ BlkRec wp_rec_merge(BlkRec a, const BlkRec& o) {
    a.nb = min(a.nb, o.nb);
    a.f = first_sel(o.f.idx < a.f.idx, o.f, a.f);
    a.bc = cand_sel(better(o.bc, a.bc), o.bc, a.bc);
    return a;
}

// The pivot-row values of column j after the block's first D pivots (win_colvals with the
// multipliers of pivot rows from `mp` -- LDS, [pivot][step] -- and extra rows' from `xm`)
template <int NX, class OUT>
__device__ __forceinline__ void wp_colvals(const double* __restrict__ T, int64_t ld, int j, int D,
                                           const BlkPiv& pv, const double (*mp)[kBlkMax],
                                           const int* xr, const double (*xm)[kBlkMax], OUT out,
                                           double* xo) {
    double x[kBlkMax];
    double xx[NX > 0 ? NX : 1];
#pragma unroll
    for (int p = 0; p < kBlkMax; ++p) x[p] = p < D ? T[(int64_t)pv.r[p] * ld + j] : 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k) xx[k] = T[(int64_t)xr[k] * ld + j];
#pragma unroll 1
    for (int q = 0; q < D; ++q) {
        const double p = x[0];
        out(q, p);
        const int rq = pv.r[q];
        const bool pc = j == pv.c[q];
        const double e = pv.e[q];
#pragma unroll
        for (int s = 1; s < kBlkMax; ++s) {
            const int t = q + s;
            if (t < D) x[s] = win_upd(x[s], pv.r[t] == rq, pc, p, mp[t][q], e);
        }
#pragma unroll
        for (int k = 0; k < NX; ++k) xx[k] = win_upd(xx[k], xr[k] == rq, pc, p, xm[k][q], e);
#pragma unroll
        for (int s = 0; s + 1 < kBlkMax; ++s) x[s] = x[s + 1];
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) xo[k] = xx[k];
}

// One block of P planner steps in one launch.  Grid: win_groups(rows) workgroups of kWinNT
// threads (<= one per CU), wave w owns rows [w rpw, (w + 1) rpw) (rpw <= kWpMaxRpw).  xg: the
// granule scratch, zeroed by k_blk_start at every chain's start (tags are unique within a chain:
// done + L + 1, `done` = pivots of the chain before this block).  The decisions, the arithmetic
// and every output are the launch form's (k_blk_wstep), step for step.
__global__ __launch_bounds__(kWinNT) void k_blk_wplan(
    const double* __restrict__ T, int64_t ld, int rows, int m, int flen, int fscan, int P,
    int parity, int bn, int done, int nwin, int rpw, smx_ctl* __restrict__ ctl,
    BlkHdr* __restrict__ h, smx_part* __restrict__ parts, double* __restrict__ mul,
    double* __restrict__ pr, uint64_t* __restrict__ xg, int32_t* __restrict__ log,
    double* __restrict__ xhist, int64_t log_cap) {
    __shared__ BlkPiv s_pv;                      // the block's pivots so far (r, c, e)
    __shared__ double s_mp[kBlkMax + 1][kBlkMax]; // [pivot t][step q]: mul[r_t][q]
    // the fallbacks' extra rows: [0] the current pivot row's multipliers, [1] the f-row's (fc_q)
    __shared__ double s_xm[2][kBlkMax];
    // this workgroup's rows' multipliers [wave][row][step] (the candidates' and the on-demand
    // pivot rows' multipliers come from here, not from a global round trip)
    __shared__ double s_mrow[kWinWaves][kWpMaxRpw][kBlkMax];
    __shared__ Decision s_d;
    __shared__ int s_nb, s_bail;
    __shared__ double s_e, s_fc, s_prcf;
    __shared__ double s_colc[kBlkMax], s_colf[kBlkMax];
    __shared__ int s_tmp[kWinWaves];
    __shared__ BlkRec s_r[kWinWaves];
    __shared__ double s_pw[kWave];               // the pivot row's window
    __shared__ double s_rv[kWinWaves][3][kWinBatch];   // row pass: "-b", entering, multiplier
    __shared__ double s_prv[kBlkMax][kWave];     // pivot rows at this workgroup's column slice
    __shared__ double s_cw[kWinWaves][kWave];    // each wave's candidate row's window
    __shared__ int s_wc[kWinWaves];              // each wave's candidate row
    __shared__ int s_gcand;                      // the workgroup's published candidate row
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
    const int b = blockIdx.x, G = gridDim.x;
    const int C = m + 1;
    const int jl = win_col(lane, nwin, C);
    const int jc = max(jl, 0);
    uint64_t* __restrict__ rec = xg;                                    // [2][kWinMaxG][kWpRecG]
    uint64_t* __restrict__ prg = rec + 2 * (int64_t)kWinMaxG * kWpRecG;  // [2][kWpRowG]
    uint64_t* __restrict__ cand = prg + 2 * (int64_t)kWpRowG;           // [2][waves][kWpCandG]
    const int64_t spin = g_res_spin_ticks;
    const int gw = b * kWinWaves + wid;   // this wave's index in the grid
    const int i0 = gw * rpw;
    const int i1 = min(rows, i0 + rpw);
    constexpr int RU = kBlkPartsMax / kWave;
    // The block's first records (built by the previous launch), the chain state, this wave's
    // rows and the f-row at the window's columns from the table itself (T_k)
    const int stopped = ctl->term;
    smx_part rp[RU];
    if (wid == 0) {
        const smx_part* __restrict__ slot = parts + (int64_t)blk_slot(0, P, bn) * G;
#pragma unroll
        for (int u = 0; u < RU; ++u) rp[u] = slot[min(lane + u * kWave, G - 1)];
    }
    int cf = h->cfs[blk_slot(0, P, bn)];   // the entering column of block step 0
    int hx0 = ctl->xpos[parity][0], hx1 = ctl->xpos[parity][1];
    int64_t kpiv = ctl->npiv[parity];
    asm volatile("" ::: "memory");
    double x[kWpMaxRpw];
#pragma unroll
    for (int u = 0; u < kWpMaxRpw; ++u) {
        if (u < rpw) {
            const double v = T[(int64_t)(i0 + u < i1 ? i0 + u : rows) * ld + jc];
            x[u] = jl >= 0 ? v : 0.0;
        } else {
            x[u] = 0.0;
        }
    }
    double fo;
    {
        const double v = T[(int64_t)rows * ld + jc];
        fo = jl >= 0 ? v : 0.0;
    }
    if (tid == 0) s_bail = 0;
    if (WP_COLD(stopped)) {
        if (b == 0 && tid == 0) h->peff = 0;   // a later block of a stopped chain
        return;
    }
    const int ms = __builtin_amdgcn_readfirstlane(win_slot(m, nwin, C));
    double* __restrict__ mT = blk_mulT(mul, rows + 1);
    const bool want_x = xhist && log_cap > 0;
    auto bail = [&](int D) {
        // a hand-off that never came (a workgroup not resident or stalled): stop the chain; the
        // host reports it (device.py sync_state, RESIDENT_TIMEOUT)
        atomicOr(&ctl->dec[0][0], kResTimeout);
        ctl->term = 1;
        if (b == 0) h->peff = D;
        s_bail = 1;
    };
    if (tid == 0) s_gcand = SMX_NONE;   // the workgroup's published candidate (none yet)
    // The pivot rows at this workgroup's column slice [jb, jb + CPW) (wave 1, lane = column):
    // pivot row q's values T_{k+q}[r_q][j] from T_k[r_q][j] through the pivots before it, with
    // pivot row q's multipliers (s_mp[q]) and the earlier pivot rows' values there (s_prv) --
    // k_blk_prows' chains, one row per step, run while wave 0 polls the next step's records.
    const bool inpr = wp_inpr(C, G);
    const int CPW = wp_cols_per_group(C, G);
    const int jpr = b * CPW + lane;
    const bool prlane = inpr && wid == 1 && lane < CPW && jpr < C;
    double prx = 0.0;   // T_k[r_q][jpr] of the latest pivot row, loaded when it was decided
    auto prow_at = [&](int q) {
        double v = prx;
#pragma unroll 1
        for (int t = 0; t < q; ++t)
            v = win_upd(v, s_pv.r[q] == s_pv.r[t], jpr == s_pv.c[t], s_prv[t][lane], s_mp[q][t],
                        s_pv.e[t]);
        s_prv[q][lane] = v;
        pr[(int64_t)q * ld + jpr] = v;
    };
    auto xrow = [&](int u) {   // x[u] for a uniform u
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < kWpMaxRpw; ++k)
            if (k == u) v = x[k];
        return v;
    };
#pragma unroll 1
    for (int L = 1; L <= P; ++L) {
        SMX_BLK_STAMP(0);
        const int D = L - 1;
        const int sp = (parity + D) & 1;
        const uint64_t tagD = (uint64_t)(uint32_t)(done + D + 1) << 32;
        const uint64_t tagL = (uint64_t)(uint32_t)(done + L + 1) << 32;
        // ---- the records of step D: from memory at D = 0, else the granules of step D --------
        if (prlane && D > 0) prow_at(D - 1);
        if (wid == 0) {
            if (D > 0) {
                // every record at once (RU x 4 granule loads per lane in flight), again until all
                // carry step D's tag
                const uint64_t* src = rec + (int64_t)(D & 1) * kWinMaxG * kWpRecG;
                uint64_t w[RU][kWpRecG];
                const int64_t t0 = rt_now();
                for (;;) {
#pragma unroll
                    for (int u = 0; u < RU; ++u)
#pragma unroll
                        for (int g = 0; g < kWpRecG; ++g)
                            w[u][g] = ld_sc1(src + (int64_t)min(lane + u * kWave, G - 1) * kWpRecG + g);
                    bool ok = true;
#pragma unroll
                    for (int u = 0; u < RU; ++u)
#pragma unroll
                        for (int g = 0; g < kWpRecG; ++g) ok = ok && wp_tagged(w[u][g], tagD);
                    if (__all(ok)) break;
                    if (WP_COLD(rt_now() - t0 > spin)) {
                        bail(D);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(WP_POLL_SLEEP);
                }
#pragma unroll
                for (int u = 0; u < RU; ++u) rp[u] = wp_unpack(w[u]);
            }
#pragma unroll
            for (int u = 0; u < RU; ++u)
                if (lane + u * kWave >= G) rp[u] = smx_part{SMX_NONE, SMX_NONE, 0.0, 3, SMX_NONE, 0.0};
            const int c = cf;
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
            const int nb = wave_min_int_dpp(n0);
            const First f = wave_first_dpp(fi);
            const Cand bb = wave_best_dpp(bq);
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
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // (LDS hand-off only)
        SMX_BLK_STAMP(1);
        if (WP_COLD(s_bail)) return;
        const int nb = s_nb;
        Decision d = s_d;
        auto terminal = [&](const Decision& dd) {
            if (b == 0 && tid == 0) {
                ctl->sel_status = dd.status;
                ctl->sel_r = dd.r;
                ctl->sel_c = dd.c;
                ctl->negb[sp] = nb;        // the state of T_{k+D}, where the chain stops
                ctl->negf[sp] = cf;
                ctl->term = 1;
                h->peff = D;
            }
        };
        if (WP_COLD(d.status != SMX_PIVOT)) {
            terminal(d);
            return;
        }
        const int r = d.r;
        if (prlane) prx = T[(int64_t)r * ld + jpr];
        // ---- the pivot row: the owner's candidate slot, or published on demand -----------------
        uint64_t* __restrict__ prow = prg + (int64_t)(L & 1) * kWpRowG;
        if (WP_COLD(r >= i0 && r < i1 && (D == 0 || s_gcand != r))) {
            const int u = r - i0;
            wp_put(prow + 2 * lane, tagL, xrow(u));
            if (lane < D) wp_put(prow + 2 * kWin + 2 * lane, tagL, s_mrow[wid][u][lane]);
        }
        if (wid == 0) {
            const bool wm = lane < D;   // row r's multipliers, for the fallbacks' chains
            const int64_t t0 = rt_now();
            uint64_t lo = 0, hi = 0, mlo = 0, mhi = 0;
            bool demand = D == 0;
            if (!demand) {
                const uint64_t* cs_ =
                    cand + ((int64_t)(D & 1) * G + r / (rpw * kWinWaves)) * kWpCandG;
                for (;;) {
                    const uint64_t rg = ld_sc1(cs_);
                    lo = ld_sc1(cs_ + 2 + 2 * lane);
                    hi = ld_sc1(cs_ + 3 + 2 * lane);
                    mlo = ld_sc1(cs_ + 2 + 2 * kWin + 2 * lane);
                    mhi = ld_sc1(cs_ + 3 + 2 * kWin + 2 * lane);
                    const uint32_t rtag = __builtin_amdgcn_readfirstlane((uint32_t)(rg >> 32));
                    const uint32_t rrow = __builtin_amdgcn_readfirstlane((uint32_t)rg);
                    if (rtag == (uint32_t)(tagD >> 32)) {
                        if (rrow != (uint32_t)r) {   // the owner's candidate is another row
                            demand = true;
                            break;
                        }
                        const bool ok = wp_tagged(lo, tagD) && wp_tagged(hi, tagD) &&
                                        (!wm || (wp_tagged(mlo, tagD) && wp_tagged(mhi, tagD)));
                        if (__all(ok)) break;
                    }
                    if (WP_COLD(rt_now() - t0 > spin)) {
                        bail(D);   // (the workgroup leaves at the barrier below)
                        break;
                    }
                    __builtin_amdgcn_s_sleep(WP_POLL_SLEEP);
                }
            }
            if (WP_COLD(demand)) {
                for (;;) {
                    lo = ld_sc1(prow + 2 * lane);
                    hi = ld_sc1(prow + 2 * lane + 1);
                    mlo = ld_sc1(prow + 2 * kWin + 2 * lane);
                    mhi = ld_sc1(prow + 2 * kWin + 2 * lane + 1);
                    const bool ok = wp_tagged(lo, tagL) && wp_tagged(hi, tagL) &&
                                    (!wm || (wp_tagged(mlo, tagL) && wp_tagged(mhi, tagL)));
                    if (__all(ok)) break;
                    if (WP_COLD(rt_now() - t0 > spin)) {
                        bail(D);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(WP_POLL_SLEEP);
                }
            }
            s_pw[lane] = wp_val(lo, hi);
            if (wm) {
                const double mv = wp_val(mlo, mhi);
                s_mp[D][lane] = mv;
                s_xm[0][lane] = mv;
            }
            if (lane == 0) s_pv.r[D] = r;   // (c, e below, before anything reads them)
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        SMX_BLK_STAMP(2);
        if (WP_COLD(s_bail)) return;
        const double pw = jl >= 0 ? s_pw[lane] : 0.0;   // T_{k+D}[r][jl]
        int c = d.c;
        if (nb != SMX_NONE) {
            // phase 1: first j < m with T_{k+D}[r][j] > 0 (simplex.py:81-85)
            const unsigned long long bal = __ballot(jl >= 0 && jl < m && pw > 0.0);
            int p1 = bal ? win_col(__ffsll((long long)bal) - 1, nwin, C) : SMX_NONE;
            if (WP_COLD(p1 == SMX_NONE && C > nwin)) {
                const int xr[1] = {r};
                for (int j0 = nwin - 1; j0 < m && p1 == SMX_NONE; j0 += kWinNT) {
                    const int j = j0 + tid;
                    int mine = SMX_NONE;
                    if (j < m) {
                        double xo[1];
                        wp_colvals<1>(T, ld, j, D, s_pv, s_mp, xr, s_xm, [](int, double) {}, xo);
                        if (xo[0] > 0.0) mine = j;
                    }
                    p1 = block_min_int_dpp<kWinNT>(mine, s_tmp);
                }
            }
            if (WP_COLD(p1 == SMX_NONE)) {
                d.c = SMX_NONE;
                d.status = SMX_INCORRECT;  // simplex.py:88-89
                terminal(d);
                return;
            }
            c = p1;
        }
        // the pivot element and the f-row's multiplier
        const int cs = __builtin_amdgcn_readfirstlane(win_slot(c, nwin, C));
        double e, fc;
        if (__builtin_expect(cs >= 0, 1)) {
            e = readlane_d(pw, cs);
            fc = readlane_d(fo, cs);
        } else {
            if (tid == 0) {
                const int xr[2] = {r, rows};
                double xo[2];
                wp_colvals<2>(T, ld, c, D, s_pv, s_mp, xr, s_xm,
                              [&](int q, double v) { s_colc[q] = v; }, xo);
                s_e = xo[0];
                s_fc = xo[1];
            }
            __syncthreads();
            e = s_e;
            fc = s_fc;
        }
        // the f-row after this pivot and the next entering column
        const double fn = jl >= 0 ? win_upd(fo, false, jl == c, pw, fc, e) : 0.0;
        int cfn;
        {
            const unsigned long long bal = __ballot(jl >= 0 && jl < fscan && fn < 0.0);
            cfn = bal ? win_col(__ffsll((long long)bal) - 1, nwin, C) : SMX_NONE;
            if (WP_COLD(cfn == SMX_NONE && C > nwin)) {
                const int xr[2] = {r, rows};
                for (int j0 = nwin - 1; j0 < fscan && cfn == SMX_NONE; j0 += kWinNT) {
                    const int j = j0 + tid;
                    int mine = SMX_NONE;
                    if (j < fscan) {
                        double xo[2];
                        wp_colvals<2>(T, ld, j, D, s_pv, s_mp, xr, s_xm, [](int, double) {}, xo);
                        if (win_upd(xo[1], false, j == c, xo[0], fc, e) < 0.0) mine = j;
                    }
                    cfn = block_min_int_dpp<kWinNT>(mine, s_tmp);
                }
            }
        }
        SMX_BLK_STAMP(3);
        const int cfs = __builtin_amdgcn_readfirstlane(cfn != SMX_NONE ? win_slot(cfn, nwin, C) : -1);
        if (WP_COLD(cfn != SMX_NONE && cfs < 0)) {
            if (tid == 0) {
                const int xr[1] = {r};
                double xo[1];
                wp_colvals<1>(T, ld, cfn, D, s_pv, s_mp, xr, s_xm,
                              [&](int q, double v) { s_colf[q] = v; }, xo);
                s_prcf = xo[0];
            }
            __syncthreads();
        }
        // bookkeeping of this pivot (workgroup 0), the labels in every workgroup (simplex.py:152)
        hx0 = move_label(hx0, r, c);
        hx1 = move_label(hx1, r, c);
        if (b == 0 && tid == 0) {
            const FastDiv fd = fd_prep(e);
            mul[(int64_t)rows * kBlkMax + D] = fc;
            h->r[D] = r;
            h->c[D] = c;
            h->e[D] = e;
            h->y[D] = fd.y;
            h->ok[D] = fd.ok ? 1 : 0;
            h->peff = D + 1;
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
            if (want_x) {                          // non-basic labels: 0 (simplex.py:60-66)
                if (hx0 < 0) xhist[2 * (kpiv % log_cap)] = 0.0;
                if (hx1 < 0) xhist[2 * (kpiv % log_cap) + 1] = 0.0;
            }
            if (L == P) h->cfs[blk_slot(L, P, bn)] = cfn;
        }
        SMX_BLK_STAMP(4);
        const int64_t hslot = 2 * (kpiv % (log_cap > 0 ? log_cap : 1));
        // the row pass (registers): every row of the wave through the pivot, its multiplier
        // stored for the sweep, the records of step L on column cfn (k_blk_wstep's pass)
        const FastDiv efd = fd_prep(e);
        const double ey = efd.y;
        const bool eok = efd.ok;
        BlkRec R{SMX_NONE, First{SMX_NONE, 0.0}, cand_none()};
        // (one instantiation per batch size: tables of at most 8,192 rows hold 4 rows per wave,
        // and an 8-row batch would compute 4 of them for nothing)
        auto rowpass = [&](auto nbc) {
            constexpr int NB = decltype(nbc)::value;
            constexpr int UBMAX = NB < kWinBatch ? NB : kWpMaxRpw;
#pragma unroll
            for (int ub = 0; ub < UBMAX; ub += NB) {
                if (ub == 0 || WP_COLD(ub < rpw)) {   // (a second batch from 16,385 rows on)
                    const int ib = i0 + ub;
                    double mcv = 0.0, acv = 0.0;
                    if (WP_COLD(cs < 0) && lane < NB && ib + lane < i1)
                        mcv = win_chain(T, ld, ib + lane, c, D, s_pv, s_colc, mul);
                    if (WP_COLD(cfs < 0 && cfn != SMX_NONE) && lane < NB && ib + lane < i1)
                        acv = win_chain(T, ld, ib + lane, cfn, D, s_pv, s_colf, mul);
                    // row u's multiplier T_{k+D}[ib + u][c]: lane cs of x (uniform), or the chain
                    double mc[NB], nv[NB];
                    if (__builtin_expect(cs >= 0, 1)) {
#pragma unroll
                        for (int u = 0; u < NB; ++u) mc[u] = readlane_d(x[ub + u], cs);
                    } else {
#pragma unroll
                        for (int u = 0; u < NB; ++u) mc[u] = __shfl(mcv, u);
                    }
                    // lane u of the wave will take row u's multiplier (lane cs's old value), "-b"
                    // entry (lane ms's new value) and entering-column entry (lane cfs's): handed over
                    // through LDS by those three lanes, 8 writes each (read-lane + select chains cost
                    // ~100 instructions per batch)
                    if (__builtin_expect(cs >= 0, 1) && lane == cs) {
#pragma unroll
                        for (int u = 0; u < NB; ++u) s_rv[wid][2][u] = x[ub + u];
                    }
                    // the pivot row (one row of the grid) takes its own rule below, off the fast path
                    const bool pc = jl == c;
                    double num[NB];
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const double a = x[ub + u] * e;
                        const double bq = pw * mc[u];
                        num[u] = pc ? x[ub + u] : (a - bq);
                    }
                    if (WP_COLD((unsigned)(r - ib) < (unsigned)NB)) {
#pragma unroll
                        for (int u = 0; u < NB; ++u)
                            if (ib + u == r) num[u] = pc ? 1.0 : -x[ub + u];
                    }
                    uint32_t wt = 0;
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        wt = max(wt, win_term(num[u]));
                        const double tq = num[u] * ey;
                        const double rr = fma(-e, tq, num[u]);
                        nv[u] = fma(rr, ey, tq);
                    }
                    if (WP_COLD(!eok || !__all(jl < 0 || wt < kWinSpan))) {
#pragma unroll
                        for (int u = 0; u < NB; ++u)
                            nv[u] = win_upd(x[ub + u], ib + u == r, jl == c, pw, mc[u], e);
                    }
                    // (lanes outside the window, jl < 0, hold zeros that stay zeros; nothing reads
                    // them unmasked)
#pragma unroll
                    for (int u = 0; u < NB; ++u) x[ub + u] = nv[u];
                    if (lane == ms) {
#pragma unroll
                        for (int u = 0; u < NB; ++u) s_rv[wid][0][u] = nv[u];
                    }
                    if (cfs >= 0 && lane == cfs) {
#pragma unroll
                        for (int u = 0; u < NB; ++u) s_rv[wid][1][u] = nv[u];
                    }
                    const int l8 = lane & (NB - 1);
                    const double mybv = s_rv[wid][0][l8];
                    double mya = cfs >= 0 ? s_rv[wid][1][l8] : 0.0;
                    const double myc = __builtin_expect(cs >= 0, 1) ? s_rv[wid][2][l8] : mcv;
                    const int i = ib + lane;
                    if (lane < NB && i < i1) {
                        if (WP_COLD(cfn != SMX_NONE && cfs < 0))
                            mya = win_upd(acv, i == r, cfn == c, s_prcf, myc, e);
                        mul[(int64_t)i * kBlkMax + D] = myc;
                        mT[(int64_t)D * (rows + 1) + i] = myc;
                        s_mrow[wid][ub + lane][D] = myc;
                        if (want_x) {
                            if (i == hx0) xhist[hslot] = mybv;
                            if (i == hx1) xhist[hslot + 1] = mybv;
                        }
                        blk_rec_add(R, i, mybv, cfn != SMX_NONE, mya);
                    }
                }
            }
        };
        if (rpw <= kWinBatch / 2)
            rowpass(std::integral_constant<int, kWinBatch / 2>{});
        else
            rowpass(std::integral_constant<int, kWinBatch>{});
        SMX_BLK_STAMP(5);
        SMX_BLK_STAMP_WMAX(6);
        // ---- the records of step L: granules (L < P) or memory (the next block's first) -------
        {
            // the wave's record: only lanes 0..7 hold rows (one per batch row), three DPP steps
            R = wp_rec_merge(R, wp_rec_dpp<kDppXor1>(R));
            R = wp_rec_merge(R, wp_rec_dpp<kDppXor2>(R));
            R = wp_rec_merge(R, wp_rec_dpp<kDppHalfMirror>(R));
            const int n0 = __builtin_amdgcn_readfirstlane(R.nb);
            const First f0{__builtin_amdgcn_readfirstlane(R.f.idx), readlane_d(R.f.v, 0)};
            const Cand c0 = readlane_cand(R.bc, 0);
            if (L < P) {
                // this wave's candidate pivot row for step L, staged in LDS (see the header)
                const int cr = wp_nominee(n0, f0, c0);
                if (cr != SMX_NONE) s_cw[wid][lane] = xrow(cr - i0);
                if (lane == 0) s_wc[wid] = cr;
            }
            if (lane == 0) s_r[wid] = BlkRec{n0, f0, c0};
            if (tid == 0) {
                s_pv.c[D] = c;
                s_pv.e[D] = e;
                s_xm[1][D] = fc;
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            SMX_BLK_STAMP(8);
            if (wid == 0) {
                // the eight waves' records: lane k < 8 takes wave k's, three DPP steps merge them
                BlkRec a = s_r[lane & (kWinWaves - 1)];
                a = wp_rec_merge(a, wp_rec_dpp<kDppXor1>(a));
                a = wp_rec_merge(a, wp_rec_dpp<kDppXor2>(a));
                a = wp_rec_merge(a, wp_rec_dpp<kDppHalfMirror>(a));
                if (L < P) {
                    if (lane < kWpRecG)
                        st_sc1(rec + ((int64_t)(L & 1) * kWinMaxG + b) * kWpRecG + lane,
                               tagL | wp_pack1(a, lane));
                    // the workgroup's candidate: the staged window of the wave that holds it,
                    // when that wave nominated the same row (else none: on demand)
                    int gc = wp_nominee(a.nb, a.f, a.bc);
                    const int wg = gc != SMX_NONE ? (gc - b * kWinWaves * rpw) / rpw : 0;
                    if (gc != SMX_NONE && s_wc[wg] != gc) gc = SMX_NONE;
                    uint64_t* __restrict__ cd = cand + ((int64_t)(L & 1) * G + b) * kWpCandG;
                    if (gc != SMX_NONE) {
                        wp_put(cd + 2 + 2 * lane, tagL, s_cw[wg][lane]);
                        if (lane < L)
                            wp_put(cd + 2 + 2 * kWin + 2 * lane, tagL,
                                   s_mrow[wg][gc - (b * kWinWaves + wg) * rpw][lane]);
                    }
                    if (lane == 0) {
                        st_sc1(cd, tagL | (uint32_t)(gc == SMX_NONE ? 0xFFFFFFFFu : (uint32_t)gc));
                        s_gcand = gc;   // (read after the next step's decision barrier)
                    }
                } else if (lane == 0) {
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
        }
        SMX_BLK_STAMP(7);
        fo = fn;
        cf = cfn;
        ++kpiv;
    }
    if (!inpr) return;   // (k_blk_prows builds the pivot rows and the flags)
    // the block's last pivot row, then the sweep's per-row flags (k_blk_prows' second job): this
    // wave's rows from their multipliers in LDS, the f-row (workgroup 0) from fc_q
    if (prlane) prow_at(P - 1);
    int32_t* __restrict__ fl = blk_rflags(mul, rows + 1);
    if (lane < rpw && i0 + lane < i1) {
        bool bnd = true, zero = false, piv = false;
#pragma unroll 1
        for (int q = 0; q < P; ++q) {
            const double v = s_mrow[wid][lane][q];
            bnd = bnd && bnd_or_zero(v);
            zero = zero || (dbits(v) << 1) == 0;
            piv = piv || i0 + lane == s_pv.r[q];
        }
        fl[i0 + lane] = blk_rflag(piv, bnd, zero);
    }
    if (b == 0 && tid == 0) {
        bool bnd = true, zero = false;
#pragma unroll 1
        for (int q = 0; q < P; ++q) {
            const double v = s_xm[1][q];
            bnd = bnd && bnd_or_zero(v);
            zero = zero || (dbits(v) << 1) == 0;
        }
        fl[rows] = blk_rflag(false, bnd, zero);
    }
}

}  // namespace
