// smx_resident.hpp -- k_resident: the whole get_solution pivot loop (simplex.py:184-198) in ONE
// persistent launch for tableaux that fit on chip.
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------------------------------------
// Why: below ~4096^2 a pivot is latency-bound, not HBM-bound (1024^2: 16.8 MB of traffic = 2.1 us
// at 8 TB/s, but ~11 us per fused launch: five dependent memory round trips plus the launch gap).
// MI355X has 256 CUs x 160 KiB of LDS = 40 MiB on chip, so a tableau up to ~2048^2 can stay in
// LDS for the whole solve: workgroup g (one per CU, 16 waves) owns constraint rows
// [g*rpw, (g+1)*rpw) and a replica of the f-row; the only per-pivot traffic between CUs is one
// 32-B record per workgroup and one pivot row.  Per pivot s (T_s in LDS):
//   A  wave 0 finds the entering column cf (first negative f-row entry) and the first local row
//      lb with a negative "-b" entry by ballots, then builds the record: in phase 1 (lb exists,
//      simplex.py:72-76) the first positive entry of row lb (:81-85) by ballots; in phase 2 the
//      ratio test on column cf over the local rows (:105-141) -- first candidate and class masks
//      by ballots, the class-0 maximum of an order-preserving key (ties to the larger row) by a
//      DPP (key, row) reduction;
//   B  wave 0 stores its candidate row(s) (row B: the lb row or the best ratio row; row A: the
//      first candidate when its ratio is NaN, :117-121) and its record, all as 8-B {payload, tag}
//      sc1 granules (a double as two granules of 32-bit halves; the record as four): every
//      granule is its own flag, so nothing is drained before the record (MI355X_MICROARCH.md,
//      "R2's granule needs no ordering at all");
//   C  lanes 0..G-1 poll one record each (sc1 loads) until its tags match, and fold it into LDS
//      atomics (min first-negative-b row, min first candidate, max class-0 key, min class-1/2
//      rows); every workgroup reaches the same decision (the arg-min is order-independent);
//   D  the winning row is staged into LDS with sc1 loads, each granule's tag checked (a bounded
//      re-poll if one is still in flight);
//   E  the Jordan step (:149-177) on the LDS rows in place, flattened over (rows x columns) so
//      all 16 waves share any shape, with the same per-element expression as k_update (pc
//      column snapshotted first); ballots over the new f-row and "-b" column give the next
//      step's cf and lb with one LDS atomicMin per wave.
// Tags are (epoch << 20) | (s + 1): unique per launch and step while the caller rotates `epoch`
// over 1..4095 and zeroes the exchange buffer when it wraps.  Records and rows are double-
// buffered by s & 1: a workgroup writing slot s & 1 at step s has passed step s-1's poll, which
// every workgroup reached only after its step s-2 reads.  Every spin is bounded in time: on a
// timeout the workgroup latches ctl->dec[0][0] and leaves, so the grid always drains.
constexpr int kResBlock = 1024;
constexpr int kResWaves = kResBlock / kWave;
constexpr int kResPollers = 256;                 // records polled by threads 0..G-1 (G <= 256)
constexpr int kResRecWords = 4;                  // 32-B record: 4 granules
constexpr int64_t kResSpinTicks = 200000000;     // 2 s of s_memrealtime (100 MHz)
// The bound every spin uses (smx_tune_resident_timeout; tests shorten it to force the timeout
// and exercise the host's recovery, device.py)
__device__ int64_t g_res_spin_ticks = kResSpinTicks;
constexpr int kResTimeout = 1;                   // ctl->dec[0][0]: a hand-off timed out
constexpr int kResMaxRows = 65534;               // 16-bit row fields in the record
constexpr int kResTraceSteps = 64;               // diagnostic trace: steps recorded
constexpr int kResTracePh = 8;                   // stamps per step and workgroup

__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t dbits(double x) { return __double_as_longlong(x); }
__device__ __forceinline__ double bitsd(uint64_t x) { return __longlong_as_double((long long)x); }
__device__ __forceinline__ int64_t rt_now() { return (int64_t)__builtin_amdgcn_s_memrealtime(); }
// order-preserving key of a ratio v < 0 (class 0: the larger v wins): ~bits grows with v
__device__ __forceinline__ unsigned long long key0(double v) { return ~dbits(v); }
// Division by the pivot element without the per-element half of the hardware sequence.
// hipcc lowers x / e to v_div_scale(e) ; v_rcp ; v_div_scale(x) ; 2 Newton steps on the
// reciprocal ; q = x'*y ; r = fma(-e', q, x') ; v_div_fmas(r, y, q) ; v_div_fixup -- eleven
// dependent ops chained through VCC, so no two divisions of a wave overlap.  When both biased
// exponents lie in [kFdLo, kFdHi] (|x|, |e| in [2^-127, 2^129): quotient far from overflow,
// underflow and denormals, x != 0) neither v_div_scale rescales (x' = x, e' = e, VCC = 0),
// v_div_fmas is a plain fma and v_div_fixup returns its input, so the sequence IS
//     y = refine(rcp(e)) (once per pivot) ; q = x*y ; r = fma(-e, q, x) ; fma(r, y, q)
// -- the same instructions on the same operands, bit-identical by construction, and three
// independent ops per element.  Outside the window the element takes the real division.
// smx_fastdiv_check (tests/test_gpu_resident.py) compares both on millions of operand pairs.
constexpr uint32_t kFdLo = 896, kFdHi = 1152;
struct FastDiv {
    double e, y;
    bool ok;   // e itself inside the window
};
__device__ __forceinline__ bool fd_in(double x) {
    const uint32_t bexp = ((uint32_t)(dbits(x) >> 52)) & 0x7ffu;
    return bexp - kFdLo <= kFdHi - kFdLo;
}
__device__ __forceinline__ FastDiv fd_prep(double e) {
    FastDiv f;
    f.e = e;
    f.ok = fd_in(e);
    const double y0 = __builtin_amdgcn_rcp(e);
    const double t0 = fma(-e, y0, 1.0);
    const double y1 = fma(y0, t0, y0);
    const double t1 = fma(-e, y1, 1.0);
    f.y = fma(y1, t1, y1);
    return f;
}
__device__ __forceinline__ double fd_div(double x, const FastDiv& f) {
    if (f.ok && fd_in(x)) {
        const double q = x * f.y;
        const double r = fma(-f.e, q, x);
        return fma(r, f.y, q);
    }
    return x / f.e;
}

// Self-check of fd_div against the compiler's division (smx_fastdiv_check): out[0] operand
// pairs inside the window, out[1] pairs whose results differ in any bit.
__global__ __launch_bounds__(256) void k_fastdiv_check(const double* __restrict__ num,
                                                       const double* __restrict__ den,
                                                       int64_t count,
                                                       unsigned long long* __restrict__ out) {
    unsigned long long in = 0, bad = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double x = num[i], e = den[i];
        const FastDiv f = fd_prep(e);
        in += (f.ok && fd_in(x)) ? 1 : 0;
        bad += (dbits(fd_div(x, f)) != dbits(x / e)) ? 1 : 0;
    }
    atomicAdd(&out[0], in);
    atomicAdd(&out[1], bad);
}


// One polling wave's reduction of its 64 records (record indices; -1 none; k0 = 0: no class 0,
// no class-0 key is 0 since that would be a NaN).
struct ResWave {
    int nb, fi, c1, i0;
    unsigned long long k0;
};

// What a workgroup learns from the G records of step s.
struct ResDecision {
    int status, r, c, owner, rowsel;   // rowsel: 0 row A, 1 row B of the owner's slot
    int gnb;                           // global first-negative-b row (ctl->negb)
    int cf;                            // first negative f-row column (ctl->negf)
};

// OVL (round 4, the default): the bulk of step s's Jordan step overlaps step s+1's hand-off.
// After staging pivot row s, only the f-row and the "-b" column are updated (E1); the records
// of step s+1 read every other value they need -- the entering column, the phase-1 row -- as
// T_{s+1} = upd_s(T_s) on the fly, the candidate rows are published as T_s values plus their
// pivot-column entry (xpc), and the rest of the table (E2) is updated by the twelve non-polling
// waves WHILE the four polling waves wait for the other workgroups' records.  The receiver of a
// row applies the same upd_s to it when staging it.  Same operations on the same operands in
// the same order: the same bits.
template <bool OVL>
__global__ __launch_bounds__(kResBlock) void k_resident(
    double* __restrict__ buf0, double* __restrict__ buf1, int64_t ld, int n, int m, int flen,
    int fscan, int parity, int k, int rpw, smx_ctl* __restrict__ ctl, int32_t* __restrict__ log,
    double* __restrict__ xhist, int64_t log_cap, uint64_t* __restrict__ xrec,
    uint64_t* __restrict__ xrow, int64_t ldx, uint32_t epoch, uint64_t* __restrict__ trace,
    int trace_from, uint64_t* __restrict__ xpc) {
    extern __shared__ double s_T[];   // (rpw + 1) rows of ldl, then s_prow[C], then s_pc[rpw + 1]
    __shared__ uint32_t s_rec[kResPollers][kResRecWords];
    __shared__ ResWave s_wred[kResPollers / kWave];
    __shared__ int s_err;
    __shared__ int s_cfu;
    __shared__ int s_rab[2];   // OVL: local candidate rows A / B of this step (-1: none)
    constexpr int NT = kResBlock;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar)
    const int g = blockIdx.x;
    const int G = gridDim.x;
    const int C = m + 1;
    const int64_t ldg = 2 * ldx;              // granules per exchanged row (two per double)
    const int ldl = C | 1;                    // odd LDS stride: column reads spread over banks
    double* s_prow = s_T + (int64_t)(rpw + 1) * ldl;
    double* s_pc = s_prow + C;
    const int row0 = g * rpw;
    const int nl = max(0, min(rpw, n - row0));   // constraint rows owned (0 for trailing groups)
    const int fl = rpw;                          // local index of the f-row replica
    const int nelem = (rpw + 1) * C;             // flattened elements of the LDS image
    const int nch = (C + kWave - 1) / kWave;     // 64-column chunks per row
    const int nunits = (rpw + 1) * nch;          // (row, chunk) units of the update
    const int uq = kResWaves / nch, ur = kResWaves - (kResWaves / nch) * nch;
    auto step_unit = [&](int& l, int& h) {       // advance a unit by kResWaves (scalar)
        l += uq;
        h += ur;
        if (h >= nch) {
            h -= nch;
            ++l;
        }
    };
    auto stamp = [&](int s, int ph) {
        if (trace != nullptr && tid == 0 && s >= trace_from && s < trace_from + kResTraceSteps)
            trace[((int64_t)(s - trace_from) * G + g) * kResTracePh + ph] = (uint64_t)rt_now();
    };

    if (ctl->term) return;
    const int64_t npiv0 = ctl->npiv[parity];
    int xp0 = ctl->xpos[parity][0], xp1 = ctl->xpos[parity][1];

    // flattened elements of this thread: e = tid + q * NT over (rpw + 1) rows x C columns, walked
    // as (local row, column) pairs advanced by (dli, dj) per step (no per-element division)
    const int li_0 = tid / C, j_0 = tid - (tid / C) * C;
    const int dli = NT / C, dj = NT - (NT / C) * C;
    auto advance = [&](int& li, int& j) {
        li += dli;
        j += dj;
        if (j >= C) {
            j -= C;
            ++li;
        }
    };
    auto valid_row = [&](int li) { return li < nl || li == fl; };   // li <= rpw checked by e
    // load T_0
    if (tid == 0) s_err = 0;
    {
        const double* Tin = parity ? buf1 : buf0;
        int li = li_0, j = j_0;
        for (int e = tid; e < nelem; e += NT, advance(li, j))
            if (valid_row(li)) s_T[li * ldl + j] = Tin[(int64_t)(li == fl ? n : row0 + li) * ld + j];
    }
    __syncthreads();

    int s = 0;
    ResDecision d;
    int last_r = SMX_NONE, last_c = SMX_NONE;
    double last_e = 0.0;
    // OVL: step s-1's pivot while its bulk update is still pending (lag): s_prow / s_pc hold its
    // pivot row and column, every value outside the f-row and the "-b" column is T_{s-1}
    bool lag = false;
    int rp_local = -1, cp = SMX_NONE, rp = SMX_NONE;
    double ep = 1.0;
    FastDiv fdp{1.0, 1.0, true};
    auto updp = [&](bool isr, bool isc, double x, double pr, double pc) -> double {
        const double t = x * ep - pr * pc;
        const double num = isr ? (isc ? 1.0 : -x) : (isc ? x : t);
        return fd_div(num, fdp);
    };
    // T_s[l][j] of an own row (OVL): the LDS value, or upd_{s-1} of it outside the "-b" column
    auto curv = [&](int l, int j) -> double {
        const double x = s_T[l * ldl + j];
        if (!OVL || !lag || j == m) return x;
        return updp(l == rp_local, j == cp, x, s_prow[j], s_pc[l]);
    };
    for (;; ++s) {
        const uint32_t want = (epoch << 20) | (uint32_t)(s + 1);
        const uint64_t tag = (uint64_t)want << 32;
        const int slot = s & 1;
        int cf = SMX_NONE, lb = SMX_NONE;   // meaningful in wave 0 (the decision reads them)
        // ---- A + B: wave 0 builds, backs and publishes this workgroup's record ------------------
        if (wid == 0) {
            stamp(s, 0);
            // entering column: first negative f-row entry j < fscan (simplex.py:94-98), and the
            // first local row whose "-b" entry is negative (:72-76), by ballots
            for (int jb = 0; jb < fscan; jb += kWave) {
                const int j = jb + lane;
                const uint64_t mk = __ballot(j < fscan && s_T[fl * ldl + j] < 0.0);
                if (mk) {
                    cf = jb + __ffsll((long long)mk) - 1;
                    break;
                }
            }
            for (int ib = 0; ib < nl; ib += kWave) {
                const int i = ib + lane;
                const uint64_t mk = __ballot(i < nl && s_T[i * ldl + m] < 0.0);
                if (mk) {
                    lb = row0 + ib + __ffsll((long long)mk) - 1;
                    break;
                }
            }
            int p1 = SMX_NONE, fidx = SMX_NONE, bcls = 3, bidx = SMX_NONE;
            bool fnan = false;
            double bv = 0.0;
            if (lb != SMX_NONE) {   // phase 1: first positive entry of row lb (simplex.py:81-85)
                const int il = lb - row0;
                for (int jb = 0; jb < m; jb += kWave) {
                    const int j = jb + lane;
                    const uint64_t mk = __ballot(j < m && curv(il, j) > 0.0);
                    if (mk) {
                        p1 = jb + __ffsll((long long)mk) - 1;
                        break;
                    }
                }
            } else if (cf != SMX_NONE) {   // phase 2: ratio test on column cf (:105-141)
                unsigned long long lkey = 0;   // this lane's best class-0 key and its row
                int lrow = -1;
                int c1 = SMX_NONE, c2 = SMX_NONE;
                for (int ib = 0; ib < nl; ib += kWave) {
                    const int i = ib + lane;
                    const double a = (i < nl) ? curv(i, cf) : 0.0;
                    const bool cand = (i < nl) && a != 0.0;
                    const double v = cand ? s_T[i * ldl + m] / a : 0.0;
                    const uint64_t mf = __ballot(cand);
                    if (fidx == SMX_NONE && mf) {
                        const int l = __ffsll((long long)mf) - 1;
                        fidx = row0 + ib + l;
                        fnan = __shfl(isnan(v) ? 1 : 0, l, kWave) != 0;
                    }
                    const bool nn = cand && !isnan(v);
                    if (nn && v < 0.0 && key0(v) >= lkey) {   // rows ascend: ties -> larger row
                        lkey = key0(v);
                        lrow = row0 + i;
                    }
                    const uint64_t m1 = __ballot(nn && v == 0.0), m2 = __ballot(nn && v > 0.0);
                    if (c1 == SMX_NONE && m1) c1 = row0 + ib + __ffsll((long long)m1) - 1;
                    if (c2 == SMX_NONE && m2) c2 = row0 + ib + __ffsll((long long)m2) - 1;
                }
                if (__ballot(lkey != 0)) {   // class 0: the largest v, ties to the larger row
                    // (key, row) maximum by DPP; v from its key (key0 is a bijection on v < 0)
                    const KeyRow kr = wave_max_keyrow_dpp(KeyRow{lkey, lrow});
                    bidx = kr.row;
                    bv = bitsd(~kr.key);
                    bcls = 0;
                } else if (c1 != SMX_NONE) {
                    bcls = 1;
                    bidx = c1;
                } else if (c2 != SMX_NONE) {
                    bcls = 2;
                    bidx = c2;
                }
            }
            stamp(s, 1);
            if (lane == 0) s_cfu = cf;   // read by every thread after the pre-poll barrier
            if (s < k) {
                const int rb = (lb != SMX_NONE) ? lb : (bcls < 2 ? bidx : -1);
                const int ra = (lb == SMX_NONE && fidx != SMX_NONE && fnan) ? fidx : -1;
                uint64_t* dst = xrow + ((int64_t)slot * G + g) * 2 * ldg;
                // the candidate rows as tagged granules: each double as two {32-bit half, tag}
                // sc1 stores, so the record below needs no drain of these stores before it (the
                // reader checks every granule's tag; the drain cost ~1 us per pivot at 1024^2).
                // Four LDS reads in flight, then eight sc1 stores
                auto put = [&](uint64_t* d, int il) {
                    for (int jb = 0; jb < C; jb += 4 * kWave) {
                        uint64_t v[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int j = jb + u * kWave + lane;
                            v[u] = j < C ? dbits(s_T[il * ldl + j]) : 0;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int j = jb + u * kWave + lane;
                            if (j < C) {
                                st_sc1(d + 2 * j, tag | (uint32_t)v[u]);
                                st_sc1(d + 2 * j + 1, tag | (uint32_t)(v[u] >> 32));
                            }
                        }
                    }
                };
                if constexpr (OVL) {
                    // published by the non-polling waves during the poll (below), each chunk by
                    // the wave whose E2 unit it is, read before that wave updates it
                    if (lane == 0) {
                        s_rab[0] = ra >= 0 ? ra - row0 : -1;
                        s_rab[1] = rb >= 0 ? rb - row0 : -1;
                    }
                } else {
                    if (rb >= 0) put(dst + ldg, rb - row0);
                    if (ra >= 0) put(dst, ra - row0);
                }
                if (OVL && lag && lane < 2) {   // the rows' step s-1 pivot-column entries
                    const int rr = lane ? rb : ra;   // lane 0 row A, lane 1 row B
                    if (rr >= 0) {
                        const uint64_t v = dbits(s_pc[rr - row0]);
                        uint64_t* pd = xpc + (((int64_t)slot * G + g) * 2 + lane) * 2;
                        st_sc1(pd, tag | (uint32_t)v);
                        st_sc1(pd + 1, tag | (uint32_t)(v >> 32));
                    }
                }
            }
            if (lane == 0) {
                uint64_t* rec = xrec + ((int64_t)slot * G + g) * kResRecWords;
                const uint32_t w0 = (lb == SMX_NONE ? 0xffffu : (uint32_t)lb) |
                                    ((p1 == SMX_NONE ? 0x1fffu : (uint32_t)p1) << 16) |
                                    ((fnan ? 1u : 0u) << 29) | ((uint32_t)bcls << 30);
                const uint32_t w1 = (fidx == SMX_NONE ? 0xffffu : (uint32_t)fidx) |
                                    ((bcls < 3 ? (uint32_t)bidx : 0xffffu) << 16);
                const uint64_t vb = dbits(bv);
                st_sc1(rec + 0, tag | w0);
                st_sc1(rec + 1, tag | w1);
                st_sc1(rec + 2, tag | (uint32_t)vb);
                st_sc1(rec + 3, tag | (uint32_t)(vb >> 32));
            }
            stamp(s, 2);
        }

        // ---- C: lanes 0..G-1 poll one record each; ballots reduce them per wave ---------------
        // Workgroup t owns rows [t*rpw, (t+1)*rpw), so "smallest row" = lowest record index with
        // a value, and among equal class-0 keys "larger row" = highest record index.
        __syncthreads();   // pollers start once this workgroup's record is out (less traffic)
        if (tid < G) {
            const uint64_t* rec = xrec + ((int64_t)slot * G + tid) * kResRecWords;
            const int64_t t0 = rt_now();
            uint64_t w[kResRecWords];
            for (;;) {
#pragma unroll
                for (int q = 0; q < kResRecWords; ++q) w[q] = ld_sc1(rec + q);
                bool ok = true;
#pragma unroll
                for (int q = 0; q < kResRecWords; ++q) ok = ok && (uint32_t)(w[q] >> 32) == want;
                if (ok) break;
                if (rt_now() - t0 > g_res_spin_ticks) {
                    s_err = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int q = 0; q < kResRecWords; ++q) s_rec[tid][q] = (uint32_t)w[q];
        }
        if (OVL && wid >= kResPollers / kWave) {
            // the twelve non-polling waves, (row, 64-column) units: the candidate rows' T_s
            // values out as tagged granules (step s < k), then E2 of step s-1 -- every column
            // but "-b" (E1 did it) -- each unit read before its own wave rewrites it
            constexpr int NW = kResWaves - kResPollers / kWave;
            const int pa = s < k ? s_rab[0] : -1, pb = s < k ? s_rab[1] : -1;
            uint64_t* dst = xrow + ((int64_t)slot * G + g) * 2 * ldg;
            for (int u = wid - kResPollers / kWave; u < nl * nch; u += NW) {   // wave-uniform
                const int l = u / nch, j = (u - l * nch) * kWave + lane;
                if (j >= C) continue;
                const double x = s_T[l * ldl + j];
                if (l == pa || l == pb) {   // (row A is a NaN-ratio candidate, B another row)
                    const uint64_t v = dbits(x);
                    uint64_t* d = dst + (l == pb ? ldg : 0) + 2 * j;
                    st_sc1(d, tag | (uint32_t)v);
                    st_sc1(d + 1, tag | (uint32_t)(v >> 32));
                }
                if (lag && j != m)
                    s_T[l * ldl + j] = updp(l == rp_local, j == cp, x, s_prow[j], s_pc[l]);
            }
        }
        if (wid < kResPollers / kWave) {   // waves holding records (tid < G)
            const bool mine = tid < G;
            const uint32_t w0 = mine ? s_rec[tid][0] : 0xffffffffu;
            const uint32_t w1 = mine ? s_rec[tid][1] : 0xffffffffu;
            const uint32_t cls = w0 >> 30;
            const uint64_t mnb = __ballot(mine && (w0 & 0xffffu) != 0xffffu);
            const uint64_t mfi = __ballot(mine && (w1 & 0xffffu) != 0xffffu);
            const uint64_t mc1 = __ballot(mine && cls == 1);
            const uint64_t mc0 = __ballot(mine && cls == 0);
            unsigned long long kx = 0;
            if (mc0) {
                if (mine && cls == 0)
                    kx = key0(bitsd((uint64_t)s_rec[tid][2] | ((uint64_t)s_rec[tid][3] << 32)));
                const unsigned long long mykey = kx;
#pragma unroll
                for (int mask = 32; mask >= 1; mask >>= 1) kx = max(kx, __shfl_xor(kx, mask, kWave));
                const uint64_t mt = __ballot(mine && cls == 0 && mykey == kx);
                if (lane == 0) s_wred[wid].i0 = wid * kWave + 63 - __clzll((long long)mt);
            }
            if (lane == 0) {
                s_wred[wid].nb = mnb ? wid * kWave + __ffsll((long long)mnb) - 1 : -1;
                s_wred[wid].fi = mfi ? wid * kWave + __ffsll((long long)mfi) - 1 : -1;
                s_wred[wid].c1 = mc1 ? wid * kWave + __ffsll((long long)mc1) - 1 : -1;
                s_wred[wid].k0 = kx;
            }
        }
        __syncthreads();
        if (s_err) break;
        {
            // every thread derives the same decision from the <= 4 wave summaries (no second
            // barrier): lowest wave wins the "smallest row" fields; class 0: the largest key,
            // ties to the higher wave (larger rows)
            int onb = -1, ofi = -1, oc1 = -1, oi0 = -1;
            unsigned long long k0 = 0;
            for (int w = 0; w < (G + kWave - 1) / kWave; ++w) {
                const ResWave sw = s_wred[w];
                if (onb < 0) onb = sw.nb;
                if (ofi < 0) ofi = sw.fi;
                if (oc1 < 0) oc1 = sw.c1;
                if (sw.k0 != 0 && sw.k0 >= k0) {
                    k0 = sw.k0;
                    oi0 = sw.i0;
                }
            }
            const int cfu = __builtin_amdgcn_readfirstlane(s_cfu);
            ResDecision e{SMX_NOT_CONVERGE, SMX_NONE, cfu, -1, 1, SMX_NONE, cfu};
            if (onb >= 0) {                                // phase 1 (simplex.py:72-91)
                const uint32_t w0 = s_rec[onb][0];
                const uint32_t p1 = (w0 >> 16) & 0x1fffu;
                e.gnb = e.r = (int)(w0 & 0xffffu);
                e.owner = onb;
                e.c = (p1 == 0x1fffu) ? SMX_NONE : (int)p1;
                e.status = (p1 == 0x1fffu) ? SMX_INCORRECT : SMX_PIVOT;
            } else if (cfu == SMX_NONE) {                  // optimum (:101-103)
                e.status = (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;
            } else if (ofi < 0) {                          // no candidate (:138-139)
                e.status = SMX_NOT_CONVERGE;
            } else if ((s_rec[ofi][0] >> 29) & 1u) {       // a NaN first candidate sticks (:117-121)
                e.status = SMX_PIVOT;
                e.r = (int)(s_rec[ofi][1] & 0xffffu);
                e.owner = ofi;
                e.rowsel = 0;
            } else if (oi0 >= 0 || oc1 >= 0) {             // best: class 0, else class 1
                const int o = oi0 >= 0 ? oi0 : oc1;
                e.status = SMX_PIVOT;
                e.r = (int)(s_rec[o][1] >> 16);
                e.owner = o;
            } else {                                       // min_val > 0 (:138-139)
                e.status = SMX_NOT_CONVERGE;
            }
            d = e;
        }
        stamp(s, 3);
        if (s == k || d.status != SMX_PIVOT) break;

        // ---- D: stage the pivot row, snapshot column c, bookkeeping ----------------------------
        const int r = d.r, c = d.c;
        const uint64_t* src = xrow + (((int64_t)slot * G + d.owner) * 2 + d.rowsel) * ldg;
        // OVL: the owner published T_{s-1} values (its "-b" entry already T_s) and the row's
        // step s-1 pivot-column entry; upd_{s-1} is applied while staging, in place (each lane
        // reads s_prow[j] = row s-1's value and writes row s's)
        double pcr = 0.0;
        const bool isr = d.r == rp;
        if (OVL && lag) {
            const uint64_t* ps = xpc + (((int64_t)slot * G + d.owner) * 2 + d.rowsel) * 2;
            uint64_t lo = ld_sc1(ps), hi = ld_sc1(ps + 1);
            if ((uint32_t)(lo >> 32) != want || (uint32_t)(hi >> 32) != want) {
                const int64_t t0 = rt_now();
                for (;;) {   // bounded like every spin
                    __builtin_amdgcn_s_sleep(1);
                    lo = ld_sc1(ps);
                    hi = ld_sc1(ps + 1);
                    if ((uint32_t)(lo >> 32) == want && (uint32_t)(hi >> 32) == want) break;
                    if (rt_now() - t0 > g_res_spin_ticks || *(volatile int*)&s_err) {
                        s_err = 1;
                        break;
                    }
                }
            }
            pcr = bitsd((lo & 0xffffffffull) | (hi << 32));
        }
        for (int j = tid; j < C; j += NT) {
            uint64_t lo = ld_sc1(src + 2 * j), hi = ld_sc1(src + 2 * j + 1);
            if ((uint32_t)(lo >> 32) != want || (uint32_t)(hi >> 32) != want) {
                const int64_t t0 = rt_now();
                for (;;) {   // a granule still in flight (bounded like every spin)
                    __builtin_amdgcn_s_sleep(1);
                    lo = ld_sc1(src + 2 * j);
                    hi = ld_sc1(src + 2 * j + 1);
                    if ((uint32_t)(lo >> 32) == want && (uint32_t)(hi >> 32) == want) break;
                    if (rt_now() - t0 > g_res_spin_ticks || *(volatile int*)&s_err) {
                        s_err = 1;
                        break;
                    }
                }
            }
            const double pv = bitsd((lo & 0xffffffffull) | (hi << 32));
            s_prow[j] = (OVL && lag && j != m) ? updp(isr, j == cp, pv, s_prow[j], pcr) : pv;
        }
        for (int i = tid; i <= rpw; i += NT)
            if (i < nl || i == fl) s_pc[i] = s_T[i * ldl + c];
        const int64_t kk = npiv0 + s;
        if (tid == 0) {
            if (g == 0 && log_cap > 0) {
                log[2 * (kk % log_cap)] = r;
                log[2 * (kk % log_cap) + 1] = c;
            }
        }
        xp0 = move_label(xp0, r, c);   // label swap (simplex.py:152)
        xp1 = move_label(xp1, r, c);
        __syncthreads();
        if (s_err) break;
        stamp(s, 4);
        const double e = s_prow[c];
        last_r = r;
        last_c = c;
        last_e = e;

        // ---- E: the Jordan step on the LDS rows + the next step's cf / lb ---------------------
        const int r_local = (r >= row0 && r < row0 + nl) ? r - row0 : -1;
        const FastDiv fd = fd_prep(e);
        // units of (one row, 64 columns), dealt to the 16 waves round-robin; the row, chunk and
        // pivot-row test are wave-uniform (scalar), two units in flight per iteration.  When the
        // chunk count divides the wave count each wave keeps ONE chunk for all its rows, so its
        // pivot-row slice and the j == c lane stay in registers (the common shapes, C <= 1024).
        auto upd = [&](int l, bool isc, double x, double pr, double pc) -> double {
            const double t = x * e - pr * pc;
            const double num = (l == r_local) ? (isc ? 1.0 : -x)   // steps 1, 3 (:155-163)
                                              : (isc ? x : t);      // steps 2, 4 (:159-175)
            return fd_div(num, fd);
        };
        if constexpr (OVL) {
            // E1: the f-row and the "-b" column now; the rest (E2) during the next poll
            for (int j = tid; j < C; j += NT)
                s_T[fl * ldl + j] = upd(fl, j == c, s_T[fl * ldl + j], s_prow[j], s_pc[fl]);
            for (int l = tid; l < nl; l += NT)
                s_T[l * ldl + m] = upd(l, m == c, s_T[l * ldl + m], s_prow[m], s_pc[l]);
            lag = true;
            rp_local = r_local;
            rp = r;
            cp = c;
            ep = e;
            fdp = fd;
        } else if (ur == 0) {   // kResWaves % nch == 0: wave wid owns chunk wid % nch
            const int j = (wid - (wid / nch) * nch) * kWave + lane;
            const bool jok = j < C, isc = j == c;
            const double pr = jok ? s_prow[j] : 0.0;
            for (int l = wid / nch; l <= rpw; l += 2 * uq) {   // wave-uniform
                const int l1 = l + uq;
                const bool v0 = valid_row(l), v1 = l1 <= rpw && valid_row(l1);
                double x0 = 0.0, c0 = 0.0, x1 = 0.0, c1 = 0.0;
                if (v0) {
                    c0 = s_pc[l];
                    if (jok) x0 = s_T[l * ldl + j];
                }
                if (v1) {
                    c1 = s_pc[l1];
                    if (jok) x1 = s_T[l1 * ldl + j];
                }
                if (v0 && jok) s_T[l * ldl + j] = upd(l, isc, x0, pr, c0);
                if (v1 && jok) s_T[l1 * ldl + j] = upd(l1, isc, x1, pr, c1);
            }
        } else {
            int li = wid / nch, ch = wid - (wid / nch) * nch;   // wave-uniform
            for (int u = wid; u < nunits; u += 2 * kResWaves) {
                int l1 = li, h1 = ch;
                step_unit(l1, h1);
                const bool v0 = valid_row(li);
                const bool v1 = u + kResWaves < nunits && valid_row(l1);
                const int j0 = ch * kWave + lane, j1 = h1 * kWave + lane;
                double x0 = 0.0, p0 = 0.0, c0 = 0.0, x1 = 0.0, p1 = 0.0, c1 = 0.0;
                if (v0) {
                    c0 = s_pc[li];
                    if (j0 < C) {
                        x0 = s_T[li * ldl + j0];
                        p0 = s_prow[j0];
                    }
                }
                if (v1) {
                    c1 = s_pc[l1];
                    if (j1 < C) {
                        x1 = s_T[l1 * ldl + j1];
                        p1 = s_prow[j1];
                    }
                }
                if (v0 && j0 < C) s_T[li * ldl + j0] = upd(li, j0 == c, x0, p0, c0);
                if (v1 && j1 < C) s_T[l1 * ldl + j1] = upd(l1, j1 == c, x1, p1, c1);
                li = l1;
                ch = h1;
                step_unit(li, ch);
            }
        }
        __syncthreads();
        stamp(s, 5);
        if (tid < 2 && xhist != nullptr && log_cap > 0) {   // (x1, x2) after pivot kk
            const int code = tid ? xp1 : xp0;
            if (code >= row0 && code < row0 + nl)
                xhist[2 * (kk % log_cap) + tid] = s_T[(code - row0) * ldl + m];
            else if (code < 0 && g == 0)
                xhist[2 * (kk % log_cap) + tid] = 0.0;
        }
    }

    if (s_err) {   // a hand-off timed out: leave everything else untouched, report it
        if (tid == 0) atomicOr(&ctl->dec[0][0], kResTimeout);
        return;
    }
    // ---- write back T_s into buf[(parity + s) & 1] (s pivots applied) --------------------------
    if (s > 0) {
        double* Tout = ((parity + s) & 1) ? buf1 : buf0;
        int li = li_0, j = j_0;
        for (int e = tid; e < nelem; e += NT, advance(li, j)) {
            if (!valid_row(li) || (li == fl && g != 0)) continue;
            Tout[(int64_t)(li == fl ? n : row0 + li) * ld + j] = s_T[li * ldl + j];
        }
    }
    if (g == 0 && tid == 0) {
        const int pf = (parity + s) & 1;
        ctl->npivots = npiv0 + s;
        ctl->npiv[pf] = npiv0 + s;
        ctl->xpos[pf][0] = xp0;
        ctl->xpos[pf][1] = xp1;
        ctl->negb[pf] = d.gnb;
        ctl->negf[pf] = d.cf;
        if (s < k) {   // terminal outcome of step s (the table stays, like the chain's update)
            ctl->sel_status = d.status;
            ctl->sel_r = d.r;
            ctl->sel_c = d.c;
            ctl->term = 1;
        } else {
            ctl->negb[pf ^ 1] = SMX_NONE;
            ctl->negf[pf ^ 1] = SMX_NONE;
            if (s > 0) {
                ctl->sel_status = SMX_PIVOT;
                ctl->sel_r = last_r;
                ctl->sel_c = last_c;
                ctl->sel_e = last_e;
            }
        }
    }
}

}  // namespace
