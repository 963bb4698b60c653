// smx_block.hpp -- block pivots: P consecutive Jordan steps (recalculate_matrix, simplex.py:143-177)
// applied in ONE HBM sweep of the tableau, their decisions (pick_element, :70-141) planned ahead
// from the block's input table.
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

template <bool B>
struct SmxBool {
    static constexpr bool value = B;
};

// ---------------------------------------------------------------------------------------------
// Why: one pivot reads and writes every element once (16 B), so a chain of single-pivot sweeps is
// pinned at the copy rate of HBM (16384^2: ~815 us per pivot, 95 % of the measured copy ceiling).
// The per-element arithmetic is only two multiplies, a subtract and a division, and
// tools/compute_probe.hip measured ~5 T element-steps/s of it on the chip against ~0.33 T
// elements/s that HBM streams: one sweep can carry several pivots.
//
// Every value of T_{k+l} follows from T_k, the pivot rows and the per-row multipliers of the
// steps before it, by the update's own expression (the look-ahead's nv(), applied l times):
//     chain(x = T_k[i][j], l):  for q < l:
//         num = (i == r_q) ? (j == c_q ? 1.0 : -x) : (j == c_q ? x : x*e_q - pr_q[j]*mul[i][q])
//         x = num / e_q
//     pr_q      = row r_q of T_{k+q}        (the pivot row of step k+q, C doubles)
//     mul[i][q] = T_{k+q}[i][c_q]           (row i's pivot-column entry before step k+q)
// so chain(T_k[i][j], l) IS T_{k+l}[i][j], bit for bit (same operations on the same operands in
// the same order as l single-pivot sweeps).  A chain of blocks on T_k:
//   k_blk_start                 once per chain: the f-row of T_k (`fr`), its first negative entry
//                               and the records of step k (first negative "-b" row and ratio
//                               candidates on that column, the layout of la_partial);
//   k_blk_step<L>, L = 1..P     one launch per pivot (nparts workgroups): every workgroup decides
//                               block step D = L-1 from its records (phase 1: first positive of
//                               the first-negative-b row, simplex.py:72-91; phase 2: ratio arg-min,
//                               :93-141) and derives the pivot row values it needs on the fly;
//                               workgroup b stores slice b of pr_D and of the next f-row; each
//                               scans the new f-row for its first negative entry (early exit);
//                               then mul[i][D] for its rows and the records of step L (chains of
//                               length L); workgroup 0 does the pivot's log / label / history
//                               bookkeeping;
//   k_blk_sweep                 every element T_k -> T_{k+peff} through the peff decided steps,
//                               out of place when peff is odd and in place when it is even, so the
//                               table after d pivots is in buf[(parity + d) & 1] exactly as in the
//                               single-pivot chains.  In place is safe: each element is read and
//                               written by the same lane and nothing reads T_k after the planner.
// k_blk_step<P> builds the records of the NEXT block's first step (chains of length P from this
// block's T_k), so a block is P + 1 launches.  A terminal outcome at step D latches ctl->term;
// the sweep still applies the D pivots decided before it and every later kernel does nothing.
//
constexpr int kBlkMax = 24;          // pivots per block (mul row stride)
constexpr int kBlkSlots = kBlkMax + 2;   // record / cf slots: steps 1..P-1, and two for step 0
// Planner workgroups: four waves, one per select partial.  (Tried: one-wave workgroups, four per
// partial -- the same threads over 256 CUs instead of 64; every workgroup then merges 256 records
// and the decision phase grew from 2.3-2.8 to 3.7-4.3 us per step: planner 15.2 -> 16.0 us per
// pivot at 16384^2, profiles/r03b/planner_trace_P10_onewave.jsonl.  The kBlkPartsPer knob keeps
// that form buildable.)
constexpr int kBlkNT = kUpdBlock;    // planner workgroup
constexpr int kBlkScan = 4 * kBlkNT; // columns per early-exit scan round
constexpr int kBlkPartsPer = kUpdBlock / kBlkNT;
// Planner workgroups: the select partition's count (at least one slice of the pivot row per
// workgroup), raised to one row per thread on tall tables: at 65536 rows 64 workgroups own
// 1,024 rows each and the row pass runs four rows per thread back to back (config 5's planner
// took 27.5 us per pivot against 14.4 at 16384^2, profiles/r03c/config5_degenerate_1gpu.json;
// 24.2 with 256 workgroups, profiles/r04h/config5_degenerate.json).
constexpr int kBlkPartsMax = 4 * kMaxParts * kBlkPartsPer;
__host__ __device__ __forceinline__ int blk_parts_of(int nparts, int rows) {
    const int by_rows = (rows + kBlkNT - 1) / kBlkNT;
    int g = nparts * kBlkPartsPer;
    if (by_rows > g) g = by_rows;
    return g < kBlkPartsMax ? g : kBlkPartsMax;
}

// The block's plan (slot 0; slot 1's header only carries a zero peff); cfs / loc / np0 are the
// chain's state.
struct BlkHdr {
    int32_t peff;                    // pivots of this block decided so far (the sweep's count)
    int32_t pad0;
    int32_t cfs[kBlkSlots];          // first j < fscan with f[j] < 0 of the step in that slot
    int32_t r[kBlkMax], c[kBlkMax];
    int32_t ok[kBlkMax];             // e inside the fast-division window (fd_prep)
    int32_t loc;                     // buffer index (0/1) of the newest table a sweep wrote
    double e[kBlkMax], y[kBlkMax];   // pivot element and its refined reciprocal (fd_prep)
    int64_t np0;                     // ctl->npivots when the chain started
};
constexpr int64_t kBlkHdrBytes = 1024;   // one plan slot's header
static_assert(sizeof(BlkHdr) <= kBlkHdrBytes, "block header");

// record / cf slot of block step l: 1..P-1 their own; step 0 of block number bn (the next block's
// first step, built by k_blk_step<P>) alternates between two slots, so no launch reads the slot
// it writes even at P = 1
__host__ __device__ __forceinline__ int blk_slot(int l, int P, int bn) {
    return l == 0 ? kBlkMax + (bn & 1) : (l == P ? kBlkMax + ((bn + 1) & 1) : l);
}

// Window planner (smx_window.hpp): slots per row of its [2][R][kWin] window of the first columns
constexpr int kWin = 64;

// Scratch layout (byte offsets; smx_block_bytes): header [2] | records [kBlkSlots][kBlkPartsMax] |
// mul [2][R][kBlkMax] | pr [2][kBlkMax][ld] | fr [2][ld] (the register-form planner's f-row by step
// parity) | the register-form planner's column caches | the window planner's window.  Plan slot 1
// of mul / pr is unused since the pipelined planner left (kept: the layout stays put).
struct BlkLayout {
    int64_t parts, mul, pr, fr, bytes, mul_slot, pr_slot, win, xg;
};
// the persistent window planner's granules (smx_wplan.hpp: records [2][256][4], on-demand pivot
// rows [2][2 * 64 + 2 * kBlkMax], every workgroup's candidate row [2][256][2 + 2 * 64 + 2 * kBlkMax])
constexpr int64_t kBlkXgBytes =
    (2 * 256 * 4 + 2 * (2 * kWin + 2 * kBlkMax) + 2 * 256 * (2 + 2 * kWin + 2 * kBlkMax)) * 8;
// the granules a grid of G planner workgroups uses (the candidates stride by G): what
// k_blk_start zeroes
__host__ __device__ __forceinline__ int64_t blk_xg_used(int G) {
    return 2 * 256 * 4 + 2 * (2 * kWin + 2 * kBlkMax) + (int64_t)2 * G * (2 + 2 * kWin + 2 * kBlkMax);
}
inline int64_t blk_align(int64_t x) { return (x + 255) / 256 * 256; }
inline BlkLayout blk_layout(int64_t R, int64_t ld, int nparts) {
    (void)nparts;   // records sized for the widest planner (the window planner: up to 256)
    BlkLayout L;
    L.parts = 2 * kBlkHdrBytes;
    L.mul = blk_align(L.parts + (int64_t)kBlkSlots * kBlkPartsMax * 32);
    // a plan slot's multipliers [R][kBlkMax], then the sweep's per-row flags int32[R] (blk_rflags),
    // then the same multipliers transposed, [kBlkMax][R] (blk_mulT: the planner's row pass)
    L.mul_slot = blk_align(R * kBlkMax * 8 + blk_align(R * 4) + R * kBlkMax * 8);
    L.pr = L.mul + 2 * L.mul_slot;
    L.pr_slot = blk_align((int64_t)kBlkMax * ld * 8);
    L.fr = L.pr + 2 * L.pr_slot;
    // then the register form's column caches (7 R doubles: unused [3][R], [2][R] T_{k+L}[i][cf],
    // [2][R] T_{k+L}[i][m]), then the window [2][R][kWin] (R = rows + 1: the f-row's too)
    L.win = blk_align(L.fr + 2 * ld * 8 + 7 * R * 8);
    L.xg = blk_align(L.win + (int64_t)2 * R * kWin * 8);
    L.bytes = blk_align(L.xg + kBlkXgBytes);
    return L;
}

// The sweep's per-row flags of a plan slot (after its R multiplier rows): 2 for a pivot row of the
// block, else 1 when every one of the row's multipliers is bounded (bnd_term < kBndSpan), 3 when
// every one is bounded or an exact +-0 and at least one is zero, 0 otherwise -- so
// blk_sweep_body_flag can take the unchecked fast path on a bounded chunk without re-checking the
// row's multipliers, or the pivot rows, itself.  Written by the block's last planner step
// (L == P), f-row included.
__host__ __device__ __forceinline__ int32_t* blk_rflags(double* mul, int64_t R) {
    return reinterpret_cast<int32_t*>(mul + R * kBlkMax);
}
__host__ __device__ __forceinline__ const int32_t* blk_rflags(const double* mul, int64_t R) {
    return reinterpret_cast<const int32_t*>(mul + R * kBlkMax);
}

// The multipliers again, transposed ([q][R], R = rows + 1 as above): the planner's row pass reads
// mul[i][0..D) of its rows -- one lane per row -- and with the row-major [R][kBlkMax] layout every
// one of those D loads of a wave touches 64 lines; transposed, each touches 4 (written beside the
// row-major copy, which the sweep and the pivot-row chains read)
__host__ __device__ __forceinline__ double* blk_mulT(double* mul, int64_t R) {
    return mul + R * kBlkMax + (R * 4 + 255) / 256 * 256 / 8;
}
__host__ __device__ __forceinline__ const double* blk_mulT(const double* mul, int64_t R) {
    return mul + R * kBlkMax + (R * 4 + 255) / 256 * 256 / 8;
}

__device__ __forceinline__ int32_t blk_rflag(bool piv, bool bnd, bool zero) {
    return piv ? 2 : (!bnd ? 0 : (zero ? 3 : 1));
}

struct BlkPiv {
    int r[kBlkMax], c[kBlkMax];
    double e[kBlkMax];
    double y[kBlkMax];   // refined reciprocal of e (fd_prep; register copies only, blk_pv_regs)
};

constexpr double kFdMinAbs = 0x1p-127;   // biased exponent 896
constexpr double kFdMaxAbs = 0x1p130;    // biased exponent 1152 is the last inside
// The same window on the high dword with 32-bit integer ops: t = (hi << 1) + kWinBias (mod 2^32)
// drops the sign and is < kWinSpan exactly when the biased exponent lies in [896, 1152] (fd_in);
// NaN, infinities, zeros and denormals fall outside.  A running unsigned max per lane replaces
// the two fp64 min/max per element and pivot (tools/sweep_probe.hip, profiles/r02_sweep_probe*).
constexpr uint32_t kWinBias = 0x90000000u;   // -(896 << 21) mod 2^32
constexpr uint32_t kWinSpan = 0x20200000u;   // (1153 - 896) << 21
__device__ __forceinline__ uint32_t win_term(double n) {
    uint32_t t;
    // one v_lshl_add_u32 (written out: the compiler turns the shift of the high dword into an
    // alignbit + and + add sequence)
    asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(t) : "v"(__double2hiint(n)), "s"(kWinBias));
    return t;
}

// Bounded operands: the sweep's unchecked fast path (blk_sweep_body_flag).  A unit needs no
// per-element window tracking when every pivot element e_q, every pivot-row value p_q[j] of the
// wave's chunk and every multiplier mq_q of the row lies in [2^-100, 2^101) in magnitude (bnd_term
// < kBndSpan; zeros, denormals, infinities and NaN fall outside) and the unit's input elements are
// finite with |x| < 2^101 (zeros and denormals allowed).  Then every numerator of the chain
//     num = RN(RN(x_q * e) - RN(p * mq)),   x_{q+1} = num / e
// is +0 or inside [2^-254, 2^410):
//   * b = RN(p * mq) is normal with |b| in [2^-200, 2^202];
//   * |a| <= |b| / 2 or |a| >= 2 |b|: |num| >= |b| / 2 (no cancellation); otherwise a - b is exact
//     (Sterbenz) and, unless 0, at least one ulp of |b| / 2 >= 2^-254.  num = -0 needs b = +0, so
//     a zero numerator is +0;
//   * |x_{q+1}| <= (|x_q| + |b / e|)(1 + 2^-52) <= 2^101 + 16 * 2^303 < 2^308 over 16 steps, so
//     |a| < 2^409 and |num| < 2^410.
// There the hoisted-reciprocal division (t = num y, r = fma(-e, t, num), fma(r, y, t)) is the
// compiler's own sequence with no scaling step (numerator exponent far above 53, exponent
// difference below 768, quotient normal) and no fixup case (a +0 numerator gives t's sign, which
// is sign(num) xor sign(e)): bit-identical to num / e (tests/test_gpu_resident.py checks the
// sequence on this domain).  Units outside these bounds keep the window-tracked path.
// SMX_BLK_NOFREE=1 in the environment (read once, by the first smx_block_bytes call -- outside any
// stream capture, since the device-symbol write would invalidate one): every unit takes the
// window-tracked path, for A/B timing on one box (tools/block_bench.py)
__device__ int g_blk_nofree = 0;
constexpr uint32_t kBndBias = 0u - (923u << 21);   // 2^-100 (biased exponent 923) -> 0
constexpr uint32_t kBndSpan = 201u << 21;          // up to biased exponent 1123 (2^101 excluded)
constexpr uint32_t kBndXMax = 1124u << 21;         // (hi << 1) below this: |x| < 2^101, finite
__device__ __forceinline__ uint32_t bnd_term(double v) {
    return ((uint32_t)__double2hiint(v) << 1) + kBndBias;
}
// bounded or an exact +-0 (the zero-extended domain, fd_zero)
__device__ __forceinline__ bool bnd_or_zero(double v) {
    return bnd_term(v) < kBndSpan || (dbits(v) << 1) == 0;
}

// Zeros in the bounded domain (the flag-form sweep, blk_sweep_body_flag; config 5's integer
// tables are ~20 % zeros).  Allow pivot-row values, multipliers and input elements to be exact
// +-0 as well (inputs otherwise in [2^-100, 2^101)).  Where b = RN(p * mq) = +-0 the numerator
// is RN(x e) -+ 0: +-0 when x is, else RN(x e) itself with |x| bounded below -- an input is
// >= 2^-100, a chain value after a b != 0 step is >= 2^-254 / 2^101 = 2^-355 (the numerator
// bound above) and a b = 0 step keeps |x| within a rounding -- so every nonzero numerator lies
// in [2^-456, 2^410): no scaling case, and the sequence above is exact for it.  A ZERO numerator
// is the one case it gets wrong: -0 over e > 0 gives +0 (t = -0, r = +0, fma(+0, y, -0) = +0),
// and every sign-fixed rearrangement fails for one sign of e.  v_div_fixup_f64 -- the last step
// of the compiler's own division -- returns q unchanged for a finite nonzero numerator, a normal
// quotient and a normal e, and sign(n) xor sign(e) zero for a zero numerator: one more VALU
// instruction per element-pivot, paid only on rows or chunks that hold zeros.
__device__ __forceinline__ double fd_zero(double n, double e, double y) {
    const double t = n * y;
    const double r = fma(-e, t, n);
    // (Round 5 tried the sign fix as a compare + a 32-bit select of t's high dword instead: the
    // zero-extended path ran no faster and the whole sweep kernel 5 % slower on the steady-state
    // config-5 blocks, profiles/r05d/.)
    return __builtin_amdgcn_div_fixup(fma(r, y, t), e, n);
}

// The zero-extended domain without the fixup (round 6): divide by a = |e| > 0 with ya = |y| (the
// refined reciprocal is sign-symmetric) and return the NEGATED quotient through the negated last
// step, g = fma(-r, ya, -t) = -RN(r ya + t) (round-to-nearest is sign-symmetric: the same bits as
// -fma(r, ya, t) for every nonzero quotient).  For a zero numerator and a > 0 it gives the right
// signed zero, which the plain form gets wrong for one sign of the divisor: n = +0: t = +0,
// r = RN(-0 + +0) = +0, g = RN(-0 + -0) = -0; n = -0: t = -0, r = RN(+0 + -0) = +0,
// g = RN(-0 + +0) = +0.  So g = -(n / |e|) = -sgn(e) (n / e), bit for bit: the caller folds the
// uniform sign -sgn(e) into the next step's product (blk_sweep_body_flag's s_zm) and applies the
// last one once per element and block -- the same 6 fp64 instructions per element-pivot as the
// unchecked fast path, where fd_zero takes 7.  All three negations are source modifiers.
// SMX_ZNEG=0 (a build knob for A/B timing: make variant VFLAGS=-DSMX_ZNEG=0) keeps fd_zero there.
#ifndef SMX_ZNEG
#define SMX_ZNEG 1
#endif
__device__ __forceinline__ double fd_zneg(double n, double a, double ya) {
    const double t = n * ya;
    const double r = fma(-a, t, n);
    return fma(-r, ya, -t);
}

// Self-check of the unchecked sequences on the domains the bounds guarantee (smx_fastdiv_check
// bounded): out[0] = pairs with e in [2^-100, 2^101) and num = +0 or |num| in [2^-254, 2^410),
// out[1] = those whose unchecked quotient differs from num / e in any bit; out[2] / out[3] the
// same for fd_zero on the zero-extended domain (num = +-0 or |num| in [2^-456, 2^410)).
__global__ __launch_bounds__(256) void k_fastdiv_bounded_check(const double* __restrict__ num,
                                                               const double* __restrict__ den,
                                                               int64_t count,
                                                               unsigned long long* __restrict__ out) {
    unsigned long long in = 0, bad = 0, in2 = 0, bad2 = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double x = num[i], e = den[i];
        const uint32_t xe = ((uint32_t)(dbits(x) >> 52)) & 0x7ffu;
        if (bnd_term(e) >= kBndSpan) continue;
        const double ref = x / e;
        const bool z = (dbits(x) << 1) == 0;
        if (dbits(x) == 0 || (xe >= 1023u - 254u && xe < 1023u + 410u)) {
            const FastDiv f = fd_prep(e);
            const double t = x * f.y;
            const double r = fma(-e, t, x);
            const double q = fma(r, f.y, t);
            ++in;
            bad += (dbits(q) != dbits(ref)) ? 1 : 0;
        }
        if (z || (xe >= 1023u - 456u && xe < 1023u + 410u)) {
            const double y = fd_prep(e).y;
            const double q = fd_zero(x, e, y);
            // fd_zneg with the sign folded back: -sgn(e) * g
            const double q2 = (e < 0.0 ? 1.0 : -1.0) * fd_zneg(x, fabs(e), fabs(y));
            ++in2;
            bad2 += (dbits(q) != dbits(ref) || dbits(q2) != dbits(ref)) ? 1 : 0;
        }
    }
    atomicAdd(&out[0], in);
    atomicAdd(&out[1], bad);
    atomicAdd(&out[2], in2);
    atomicAdd(&out[3], bad2);
}


// chain() with the division in its hoisted-reciprocal form (3 dependent fp64 ops instead of the
// ~10 of the IEEE sequence): bit-identical while every numerator stays inside the window, which
// `wt` tracks (win_term; a caller recomputes with blk_chain when a wave vote says otherwise,
// or when a pivot element itself is outside the window).  The planner's chains are latency-
// bound -- one wave per SIMD, steps in sequence -- so this is what shortens them.
// (Q0 > 0: the chain's steps Q0..L-1 only, from x = T_{k+Q0}[i][j])
template <int L, int Q0 = 0>
__device__ __forceinline__ double blk_chain_fd(double x, int i, int j, const BlkPiv& pv,
                                               const double* p, const double* mq, uint32_t& wt) {
#pragma unroll
    for (int q = Q0; q < L; ++q) {
        const double e = pv.e[q];
        // branch-free (the row and column tests differ across lanes): both numerators, then
        // a select -- the pivot row's products are computed and discarded
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

// T_{k+L}[i][j] from x = T_k[i][j]; p[q] = pr_q[j], mq[q] = mul[i][q] (loaded by the caller, all
// before the first use, so a chain costs one memory round trip, not L)
template <int L, int Q0 = 0>
__device__ __forceinline__ double blk_chain(double x, int i, int j, const BlkPiv& pv,
                                            const double* p, const double* mq) {
#pragma unroll
    for (int q = Q0; q < L; ++q) {
        const double e = pv.e[q];
        // branch-free (the row and column tests differ across lanes): both numerators, then
        // a select -- the pivot row's products are computed and discarded
        const double a = x * e;
        const double b = p[q] * mq[q];
        const bool jc = j == pv.c[q];
        const double num = (i == pv.r[q]) ? (jc ? 1.0 : -x) : (jc ? x : (a - b));
        x = num / e;
    }
    return x;
}

// A chain's operands must all be in registers before its first step: left to itself the
// compiler sinks each load next to its use, and a chain of L steps then waits for L memory round
// trips one after the other (the planner's scans and row pass grew by ~0.5 us per chain step,
// tools/trace_planner.hip).  An empty asm that "modifies" a value forces its load to have landed
// there, so all of a chain's loads are issued together and waited for once.
__device__ __forceinline__ void blk_pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void blk_pin(int& x) { asm volatile("" : "+v"(x)); }

template <int L>
__device__ __forceinline__ void blk_load_col(const double* __restrict__ pr, int64_t ld, int j,
                                             double* p) {
#pragma unroll
    for (int q = 0; q < L; ++q) p[q] = pr[(int64_t)q * ld + j];
#pragma unroll
    for (int q = 0; q < L; ++q) blk_pin(p[q]);
}

// The first L pivots of an LDS-broadcast BlkPiv in registers (see blk_pin)
template <int L>
__device__ __forceinline__ BlkPiv blk_pv_regs(const BlkPiv& s, bool* allok = nullptr) {
    BlkPiv v;
#pragma unroll
    for (int q = 0; q < L; ++q) {
        v.r[q] = s.r[q];
        v.c[q] = s.c[q];
        v.e[q] = s.e[q];
    }
#pragma unroll
    for (int q = 0; q < L; ++q) {
        blk_pin(v.r[q]);
        blk_pin(v.c[q]);
        blk_pin(v.e[q]);
    }
    bool ok = true;
#pragma unroll
    for (int q = 0; q < L; ++q) {
        const FastDiv f = fd_prep(v.e[q]);
        v.y[q] = f.y;
        ok = ok && f.ok;
    }
    if (allok) *allok = ok;
    return v;
}

// Row r of T_{k+D} at column j (the pivot row of block step D; mqr = mul[r][0..D))
template <int D>
__device__ __forceinline__ double blk_prv(const double* __restrict__ T, int64_t ld, int r, int j,
                                          const BlkPiv& pv, const double* __restrict__ pr,
                                          const double* mqr) {
    double p[kBlkMax];
    blk_load_col<D>(pr, ld, j, p);
    return blk_chain<D>(T[(int64_t)r * ld + j], r, j, pv, p, mqr);
}

// A lane's double, read by every lane (two v_readlane_b32: the value lands in scalar registers)
__device__ __forceinline__ double blk_readlane(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// The f-row entry after a pivot (row `rows` is never the pivot row): simplex.py:159-160/:166-175
__device__ __forceinline__ double blk_fnew(double x, double pj, int j, int c, double e,
                                           double fc) {
    const double a = x * e;
    const double b = pj * fc;
    return ((j == c) ? x : (a - b)) / e;
}


// Workgroup partial of the records (first negative "-b" row; first ratio candidate and best key)
struct BlkRec {
    int nb;
    First f;
    Cand bc;
};

__device__ __forceinline__ void blk_rec_add(BlkRec& R, int i, double bv, bool has_a, double a) {
    // (branch-free, smx_common.hpp better(); the quotient is formed whether or not it counts)
    R.nb = ((bv < 0.0) & (i < R.nb)) ? i : R.nb;            // simplex.py:73-76
    const bool use = has_a & (a != 0.0);                    // simplex.py:112 (NaN counts)
    const double v = bv / a;                                // simplex.py:115
    R.f = first_sel(use & (i < R.f.idx), First{i, v}, R.f);
    const Cand x = classify(v, i);
    R.bc = cand_sel(((int)use & (int)!isnan(v) & (int)better(x, R.bc)) != 0, x, R.bc);
}

// The workgroup's record (thread 0 holds it afterwards; the others an unspecified value)
__device__ __forceinline__ smx_part blk_rec_reduce(BlkRec R) {
    __shared__ int s_b[kBlkNT / kWave];
    __shared__ First s_f[kBlkNT / kWave];
    __shared__ Cand s_c[kBlkNT / kWave];
    const int tid = threadIdx.x;
    int nb = wave_min_int_dpp(R.nb);
    First f = wave_first_dpp(R.f);
    Cand bc = wave_best_dpp(R.bc);
    const int wid = tid >> 6;
    if ((tid & 63) == 0) {
        s_b[wid] = nb;
        s_f[wid] = f;
        s_c[wid] = bc;
    }
    __syncthreads();
    smx_part pt{};
    if (tid == 0) {
        for (int w = 1; w < kBlkNT / kWave; ++w) {
            nb = min(nb, s_b[w]);
            if (s_f[w].idx < f.idx) f = s_f[w];
            if (better(s_c[w], bc)) bc = s_c[w];
        }
        pt.p1col = nb;
        pt.first = f.idx;
        pt.first_v = f.v;
        pt.best_cls = bc.cls;
        pt.best_i = bc.idx;
        pt.best_v = bc.v;
    }
    return pt;
}

__device__ __forceinline__ void blk_rec_store(BlkRec R, smx_part* out) {
    __shared__ int s_b[kBlkNT / kWave];
    __shared__ First s_f[kBlkNT / kWave];
    __shared__ Cand s_c[kBlkNT / kWave];
    const int tid = threadIdx.x;
    int nb = wave_min_int_dpp(R.nb);
    First f = wave_first_dpp(R.f);
    Cand bc = wave_best_dpp(R.bc);
    const int wid = tid >> 6;
    if ((tid & 63) == 0) {
        s_b[wid] = nb;
        s_f[wid] = f;
        s_c[wid] = bc;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kBlkNT / kWave; ++w) {
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
        *out = pt;
    }
}

// Every lane merges up to kBlkPartsMax / kWave records of a slot (loaded together: one round trip),
// then the wave reduces them (the order of both merges is immaterial: total orders)
__device__ __forceinline__ void blk_merge_records(const smx_part* __restrict__ slot, int G,
                                                  int& nb, First& f, Cand& bb) {
    constexpr int U = kBlkPartsMax / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    smx_part p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int k = lane + u * kWave;
        p[u] = k < G ? slot[k] : smx_part{SMX_NONE, SMX_NONE, 0.0, 3, SMX_NONE, 0.0};
    }
    int n = SMX_NONE;
    First fi{SMX_NONE, 0.0};
    Cand b = cand_none();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        n = min(n, p[u].p1col);
        if (p[u].first < fi.idx) fi = First{p[u].first, p[u].first_v};
        const Cand o{p[u].best_cls, p[u].best_i, p[u].best_v};
        if (better(o, b)) b = o;
    }
    nb = wave_min_int_dpp(n);
    f = wave_first_dpp(fi);
    bb = wave_best_dpp(b);
}

// Chain start, one launch (round 5: k_blk_prime, one 1024-thread workgroup for the f-row, then
// k_blk_first for the records -- 9.8 + 6.7 us and a launch gap at 16384^2): every workgroup finds
// the f-row's first negative entry j < fscan itself (simplex.py:94-98; rounds of 4 kBlkNT
// columns with early exit -- the same minimum in every workgroup), copies its slice of the f-row
// into fr[parity], and builds its record of step 0 on that column (workgroup b of G: local rows
// b*NT + tid + q*G*NT, global row indices row0 + i); workgroup 0 writes the chain state (loc =
// buffer index of T, np0 = the pivot count, even for a stopped chain).
__global__ __launch_bounds__(kBlkNT) void k_blk_start(const double* __restrict__ T, int64_t ld,
                                                      int rows, int m, int fscan, int parity,
                                                      int loc, int row0,
                                                      const smx_ctl* __restrict__ ctl,
                                                      BlkHdr* __restrict__ h,
                                                      BlkHdr* __restrict__ h1,
                                                      double* __restrict__ fr,
                                                      smx_part* __restrict__ parts,
                                                      uint64_t* __restrict__ xg) {
    __shared__ int s_tmp[kBlkNT / kWave];
    const int b = blockIdx.x, G = gridDim.x, tid = threadIdx.x;
    // the persistent window planner's granules: tag 0 never matches (its tags are >= 2)
    if (xg)
        for (int64_t t = b * kBlkNT + tid; t < blk_xg_used(G); t += G * kBlkNT) xg[t] = 0;
    if (b == 0 && tid == 0) {
        h->loc = loc;
        h->np0 = ctl->npivots;
        h1->peff = 0;
    }
    if (ctl->term) return;
    const int C = m + 1;
    const double* f = T + (int64_t)rows * ld;
    double* fo = fr + (int64_t)parity * ld;
    const int S = (C + G - 1) / G;
    for (int j = b * S + tid; j < min(C, (b + 1) * S); j += kBlkNT) fo[j] = f[j];
    int cf = SMX_NONE;
    for (int j0 = 0; j0 < fscan && cf == SMX_NONE; j0 += 4 * kBlkNT) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kBlkNT + tid;
            v[u] = j < fscan ? f[j] : 0.0;
        }
        int mn = SMX_NONE;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kBlkNT + tid;
            if (j < fscan && v[u] < 0.0 && j < mn) mn = j;
        }
        cf = block_min_int_dpp<kBlkNT>(mn, s_tmp);
    }
    if (b == 0 && tid == 0) {
        h->cfs[blk_slot(0, 1, 0)] = cf;
        h->peff = 0;
    }
    BlkRec R{SMX_NONE, First{SMX_NONE, 0.0}, cand_none()};
    for (int i = b * kBlkNT + tid; i < rows; i += G * kBlkNT) {
        const double* row = T + (int64_t)i * ld;
        const double bv = row[m];
        const double a = cf != SMX_NONE ? row[cf] : 0.0;
        blk_rec_add(R, row0 + i, bv, cf != SMX_NONE, a);
    }
    blk_rec_store(R, parts + (int64_t)blk_slot(0, 1, 0) * G + b);
}

__device__ __forceinline__ void blk_load_pivots(const BlkHdr* __restrict__ h, int D, BlkPiv* s_pv) {
    const int t = threadIdx.x;
    if (t < D) {
        s_pv->r[t] = h->r[t];
        s_pv->c[t] = h->c[t];
        s_pv->e[t] = h->e[t];
    }
}

// Row-sharded blocks: this rank's send slot for block step D (layout of k_pack, smx_shard.hpp):
// the header from its local records of step D, row A = its first ratio candidate when that ratio
// is NaN (simplex.py:117-121), row B = its first-negative-b row (phase 1) or its best ratio row,
// both as values of T_{k+D} (chains of length D from the rank's rows of T_k), and hdr[7] = the
// phase-1 column of row B (simplex.py:81-85) when this rank holds a negative "-b" entry.
// Workgroup b writes slice b of the rows; workgroup 0 the header.
template <int D>
__global__ __launch_bounds__(kBlkNT) void k_bsh_pack(
    const double* __restrict__ T, int64_t ld, int rows, int m, int row0, int P, int bn,
    const smx_ctl* __restrict__ ctl, const BlkHdr* __restrict__ h,
    const smx_part* __restrict__ parts, int nparts, const double* __restrict__ mul,
    const double* __restrict__ pr, double* __restrict__ send) {
    constexpr int NT = kBlkNT;
    __shared__ BlkPiv s_pv;
    __shared__ int s_tmp[NT / kWave];
    __shared__ int s_rows[2];
    __shared__ int s_hi[4];
    __shared__ double s_hd[2];
    const int tid = threadIdx.x, b = blockIdx.x, G = gridDim.x;
    if (ctl->term) return;
    blk_load_pivots(h, D, &s_pv);
    if (tid < kWave) {
        int nb;
        First f;
        Cand bb;
        blk_merge_records(parts + (int64_t)blk_slot(D, P, bn) * nparts, nparts, nb, f, bb);
        if (tid == 0) {
            s_rows[0] = (f.idx != SMX_NONE && isnan(f.v)) ? f.idx - row0 : -1;
            s_rows[1] = (nb != SMX_NONE) ? nb - row0 : (bb.cls < 3 ? bb.idx - row0 : -1);
            s_hi[0] = nb;
            s_hi[1] = f.idx;
            s_hi[2] = bb.cls;
            s_hi[3] = bb.idx;
            s_hd[0] = f.v;
            s_hd[1] = bb.v;
        }
    }
    __syncthreads();
    const int C = m + 1;
    const int64_t HDR = SMX_SHARD_HDR;
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        const int rl = s_rows[w];
        if (rl < 0) continue;
        double mqr[kBlkMax];
#pragma unroll
        for (int q = 0; q < D; ++q) mqr[q] = mul[(int64_t)rl * kBlkMax + q];
        const int S = ((C + G - 1) / G + 1) & ~1;
        const int s1 = min(C, (b + 1) * S);
        double* dst = send + HDR + (int64_t)w * ld;
        for (int j = b * S + tid; j < s1; j += NT) dst[j] = blk_prv<D>(T, ld, rl, j, s_pv, pr, mqr);
    }
    if (b != 0) return;
    int p1 = SMX_NONE;
    if (s_hi[0] != SMX_NONE) {
        // phase 1 on the owner's row: first j < m with T_{k+D}[r][j] > 0, early exit by rounds
        const int rl = s_rows[1];
        double mqr[kBlkMax];
#pragma unroll
        for (int q = 0; q < D; ++q) mqr[q] = mul[(int64_t)rl * kBlkMax + q];
        for (int j0 = 0; j0 < m && p1 == SMX_NONE; j0 += kBlkScan) {
            int mine = SMX_NONE;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = j0 + k * NT + tid;
                if (j < m && blk_prv<D>(T, ld, rl, j, s_pv, pr, mqr) > 0.0 && j < mine) mine = j;
            }
            p1 = block_min_int_dpp<NT>(mine, s_tmp);
        }
    }
    if (tid == 0) {
        send[0] = (double)s_hi[0];
        send[1] = (double)s_hi[1];
        send[2] = s_hd[0];
        send[3] = (double)s_hi[2];
        send[4] = (double)s_hi[3];
        send[5] = s_hd[1];
        send[6] = (double)h->cfs[blk_slot(D, P, bn)];
        send[7] = (double)p1;
    }
}

// Light exchange of the row-sharded protocol: only the headers are all-gathered (SMX_SHARD_HDR
// doubles per rank, `hdrs` = [nranks][SMX_SHARD_HDR]); every rank reaches the same decision from
// them, the owner of the winning row copies it (row A or B of its send slot) into `row` and the
// others fill it with the bit pattern 0x8000000000000000, so ONE all-reduce (max over int64)
// leaves the owner's row, bit for bit (-0.0 included: it IS that pattern), on every rank.
__global__ __launch_bounds__(kUpdBlock) void k_bsh_pick(const double* __restrict__ hdrs,
                                                        int nranks, int64_t ld, int m, int flen,
                                                        int rank, const double* __restrict__ send,
                                                        double* __restrict__ row) {
    __shared__ int s_own;
    __shared__ int64_t s_within;
    if (threadIdx.x == 0) {
        const ShardDecision d = merge_headers_s(hdrs, nranks, ld, m, flen, SMX_SHARD_HDR);
        const bool mine = d.status == SMX_PIVOT && d.owner == rank;
        s_own = mine ? 1 : 0;
        s_within = mine ? d.off - (int64_t)d.owner * SMX_SHARD_HDR : 0;
    }
    __syncthreads();
    const bool own = s_own != 0;
    const double* src = send + s_within;
    unsigned long long* out = reinterpret_cast<unsigned long long*>(row);
    for (int64_t j = (int64_t)blockIdx.x * kUpdBlock + threadIdx.x; j < ld;
         j += (int64_t)gridDim.x * kUpdBlock)
        out[j] = own ? (unsigned long long)__double_as_longlong(src[j]) : 0x8000000000000000ull;
}

#ifdef SMX_BLK_TRACE
// Diagnostic build only (tools/trace_planner.hip): per-workgroup s_memrealtime stamps (100 MHz,
// chip-wide) of every planner step, [block step L][workgroup][phase]: 0 entry, 1 decision known,
// 2 pivot element known, 3 pivot-row / f-row slice written, 4 next entering column found,
// 5 row pass operands staged, 6 row pass done, 7 records stored (the persistent window planner:
// 6 the LAST wave's row pass done, 8 after the records' workgroup barrier).
constexpr int kBlkTraceParts = 64;
constexpr int kBlkTracePh = 10;
__device__ unsigned long long g_blk_trace[kBlkMax + 1][kBlkTraceParts][kBlkTracePh];
#define SMX_BLK_STAMP_AT(ph)                                                           \
    do {                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < kBlkTraceParts)                           \
            g_blk_trace[L][blockIdx.x][ph] = __builtin_amdgcn_s_memrealtime();         \
    } while (0)
// waves whose chains left the fast-division window (they recompute with the IEEE division):
// [L][0] phase-2 pivot-row chains, [L][1] row pass
__device__ unsigned g_blk_fallback[kBlkMax + 1][2];
#define SMX_BLK_FALLBACK(k)                                                            \
    do {                                                                               \
        if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(&g_blk_fallback[L][k], 1u);    \
    } while (0)
// the latest of the workgroup's waves
#define SMX_BLK_STAMP_WMAX(ph)                                                         \
    do {                                                                               \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < kBlkTraceParts)                    \
            atomicMax(&g_blk_trace[L][blockIdx.x][ph],                                 \
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());           \
    } while (0)
#ifdef SMX_BLK_TRACE_P2
// phase-2 anatomy instead: 2 operands landed, 3 fast chains done, 4 after the exact fallback
#define SMX_BLK_STAMP(ph) \
    do {                  \
        if ((ph) < 2 || (ph) > 4) SMX_BLK_STAMP_AT(ph); \
    } while (0)
#define SMX_BLK_STAMP_P2(ph) SMX_BLK_STAMP_AT(ph)
#else
#define SMX_BLK_STAMP(ph) SMX_BLK_STAMP_AT(ph)
#define SMX_BLK_STAMP_P2(ph) \
    do {                     \
    } while (0)
#endif
#else
#define SMX_BLK_FALLBACK(k) \
    do {                    \
    } while (0)
#define SMX_BLK_STAMP_P2(ph) \
    do {                     \
    } while (0)
#define SMX_BLK_STAMP(ph) \
    do {                  \
    } while (0)
#define SMX_BLK_STAMP_WMAX(ph) \
    do {                       \
    } while (0)
#endif

// One pivot of the block: decide block step D = L-1 and build the records of step L.
// Round 4, tried and not kept (tools/trace_planner.hip, 16384^2, per-step mean over 2-3 blocks,
// profiles/r04h/ and r04i/): the decision-independent operands (pivot-row slices at the phase-2
// columns, the f-row, the row pass's multipliers and cached columns) issued at step entry --
// decision phase 2.67 -> 3.6 us, post-decision phase 0.4 us shorter, step 13.4 -> 14.1 us at
// P = 10 (also with the merging wave's record loads issued first); the first 32 columns of each
// row staged in LDS by LDS-DMA for the row pass's column read -- row pass 2.53 -> 2.51 us;
// the row pass's column load issued before the step's first stores -- 0.1 us.
// SH = false: the decision from the records of step D and the pivot-row values derived on the
// fly; SH = true (row-sharded): from the P gathered send slots in `recv` (merge_headers), the
// pivot row taken from the winning slot.  Pivot rows are LOCAL indices in the header (-1 when
// another rank owns the row); the log and the labels use global ones.
template <int L, bool SH>
__device__ __forceinline__ bool blk_step_body(
    const double* __restrict__ T, int64_t ld, int rows, int m, int flen, int fscan, int row0,
    int P, int parity, int bn, smx_ctl* __restrict__ ctl, BlkHdr* __restrict__ h,
    smx_part* __restrict__ parts, double* __restrict__ mul, double* __restrict__ pr,
    double* __restrict__ fr, const double* __restrict__ recv, int nranks,
    int32_t* __restrict__ log, double* __restrict__ xhist, int64_t log_cap,
    const double* __restrict__ xrow, int64_t xslot) {
    BlkHdr* __restrict__ hs = h;   // the chain state (cfs) lives in the block's header
    constexpr int D = L - 1;
    constexpr int NT = kBlkNT;
    constexpr int SCANU = 4;   // scan rounds: all four columns of a thread issued at once
    __shared__ BlkPiv s_pv;
    __shared__ double s_col[3][kBlkMax];      // pr_q at columns c, m, cf
    __shared__ int s_tmp[NT / kWave];
    __shared__ Decision s_d;
    __shared__ int s_nb, s_c;
    __shared__ int64_t s_off;
    __shared__ double s_e, s_fc, s_pm, s_pa;
    const int tid = threadIdx.x;
    const int b = blockIdx.x, G = gridDim.x;
    SMX_BLK_STAMP(0);
    // The stop flag is loaded together with the decision's operands and tested after them (one
    // memory round trip instead of two): on a stopped chain those loads read stale scratch and
    // their results are discarded.
    const int stopped = ctl->term;
    const int sp = (parity + D) & 1;   // step parity of block step D
    const int C = m + 1;
    blk_load_pivots(h, D, &s_pv);
    if (SH) {
        if (tid == 0) {
            // full exchange: recv = the gathered send slots; light (xslot = SMX_SHARD_HDR): recv
            // = the gathered headers and xrow = the pivot row (k_bsh_pick + max all-reduce)
            const int64_t slot = xslot > 0 ? xslot : SMX_SHARD_HDR + 2 * ld;
            const ShardDecision sd = merge_headers_s(recv, nranks, ld, m, flen, slot);
            int gnb = SMX_NONE;
            for (int p = 0; p < nranks; ++p) gnb = min(gnb, (int)recv[p * slot]);
            s_d = Decision{sd.status, sd.r, sd.c};
            s_nb = gnb;
            s_c = (int)recv[6];
            s_off = sd.off;
        }
    } else if (tid < kWave) {
        // the decision of step D from its records (every workgroup, identically)
        const int c = hs->cfs[blk_slot(D, P, bn)];
        int nb;
        First f;
        Cand bb;
        blk_merge_records(parts + (int64_t)blk_slot(D, P, bn) * G, G, nb, f, bb);
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
            s_nb = nb;
            s_d = d;
            s_c = c;                   // cf of step D (the terminal state's negf)
        }
    }
    __syncthreads();
    SMX_BLK_STAMP(1);
    if (stopped) {
        // Everything decoded above (s_d, s_nb, s_c, s_off from the records or the gathered
        // headers) is stale on a stopped chain: nothing derived from it may be dereferenced
        // before this return (test_gpu_block_sharded: a terminal block followed by more blocks).
        if (D == 0 && b == 0 && tid == 0) h->peff = 0;   // a later block of a stopped chain
        return true;
    }
    const int nb = s_nb;
    Decision d = s_d;
    auto terminal = [&](const Decision& dd) {
        if (b == 0 && tid == 0) {
            ctl->sel_status = dd.status;
            ctl->sel_r = dd.r;
            ctl->sel_c = dd.c;
            ctl->negb[sp] = nb;        // the state of T_{k+D}, where the chain stops
            ctl->negf[sp] = s_c;
            ctl->term = 1;
            h->peff = D;
        }
    };
    if (d.status != SMX_PIVOT) {
        terminal(d);
        return true;
    }
    const int r = d.r;                                   // global pivot row
    const int r_local = (r >= row0 && r < row0 + rows) ? r - row0 : -1;
    const double* prow = SH ? (xrow ? xrow : recv + s_off) : nullptr;   // T_{k+D}[r][*] (sharded)
    double mqr[kBlkMax];
    if (!SH) {
#pragma unroll
        for (int q = 0; q < D; ++q) mqr[q] = mul[(int64_t)r_local * kBlkMax + q];
#pragma unroll
        for (int q = 0; q < D; ++q) blk_pin(mqr[q]);
    }
    // this block's first D pivots (s_pv is complete up to D since the decision)
    bool okD = true;
    const BlkPiv pvD = blk_pv_regs<D>(s_pv, &okD);
    auto prv = [&](int j) -> double {
        if (SH) return prow[j];
        double x = T[(int64_t)r_local * ld + j];
        double p[kBlkMax];
        blk_load_col<D>(pr, ld, j, p);
        blk_pin(x);
        uint32_t wt = 0;
        const double v = blk_chain_fd<D>(x, r_local, j, pvD, p, mqr, wt);
        if (okD && __all(wt < kWinSpan)) return v;
        return blk_chain<D>(x, r_local, j, pvD, p, mqr);
    };
    const double* fo = fr + (int64_t)sp * ld;          // f-row of T_{k+D}
    double* fn = fr + (int64_t)(sp ^ 1) * ld;          // f-row of T_{k+L}
    double* prD = pr + (int64_t)D * ld;
    int c, cf;
    double e, fc;
    // Phase 2 of the register form (the benchmark's every step): row r's operands for the pivot
    // element, the "-b" column, this thread's slice column and its first-round scan column
    // are loaded in ONE round trip, and the thread whose scan column is the next entering column
    // hands its pivot-row value and operands to the row pass through LDS -- three dependent round
    // trips fewer than the phases below (pivot element, then slice, then scan, then that column).
    // Three chains per thread: the two uniform columns are split over the lanes (even lanes c, odd
    // lanes m; every lane takes e = T_{k+D}[r][c] from lane 0 and T_{k+D}[r][m] from lane 1), and
    // the first scan round covers the first NT = 256 columns (the first negative f-row entry of
    // the benchmark's LPs lies within the first ~60 columns; the earlier first round of 1024
    // columns cost 7 chains and 7 (D + 2) loads per thread on every step: tools/trace_planner.hip,
    // profiles/r03b/).  Same chains on the same operands: the same values.
    if (!SH && nb == SMX_NONE) {
        c = d.c;
        const double* Tr = T + (int64_t)r_local * ld;
        const int S = ((C + G - 1) / G + 1) & ~1;
        const int s0 = b * S, s1 = min(C, s0 + S);
        constexpr int NSC = NT >= 128 ? 1 : 128 / NT;   // first-round scan columns per thread
        constexpr int NJ = 2 + NSC;   // c or m (by lane parity), slice, scan columns
        int jj[NJ];
        jj[0] = (tid & 1) ? m : c;
        jj[1] = s0 + tid;
#pragma unroll
        for (int k = 0; k < NSC; ++k) jj[2 + k] = tid + k * NT;
        double x[NJ], pq[NJ][kBlkMax], fv[NJ];
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
            const int jc = min(jj[u], C - 1);
            x[u] = Tr[jc];
            fv[u] = fo[jc];
#pragma unroll
            for (int q = 0; q < D; ++q) pq[u][q] = pr[(int64_t)q * ld + jc];
        }
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
            blk_pin(x[u]);
            blk_pin(fv[u]);
#pragma unroll
            for (int q = 0; q < D; ++q) blk_pin(pq[u][q]);
        }
        SMX_BLK_STAMP_P2(2);
        double v[NJ];
        uint32_t wt = 0;
#pragma unroll
        for (int u = 0; u < NJ; ++u) v[u] = blk_chain_fd<D>(x[u], r_local, jj[u], pvD, pq[u], mqr, wt);
#ifdef SMX_BLK_TRACE_P2
        blk_pin(v[0]);
#endif
        SMX_BLK_STAMP_P2(3);
        if (!okD || !__all(wt < kWinSpan)) {
            SMX_BLK_FALLBACK(0);
#pragma unroll
            for (int u = 0; u < NJ; ++u) v[u] = blk_chain<D>(x[u], r_local, jj[u], pvD, pq[u], mqr);
        }
        SMX_BLK_STAMP_P2(4);
        e = blk_readlane(v[0], 0);
        fc = blk_readlane(fv[0], 0);
        SMX_BLK_STAMP(2);
        // slice b of the pivot row and of the next f-row (columns beyond the first NT: as below)
        if (jj[1] < s1) {
            prD[jj[1]] = v[1];
            fn[jj[1]] = blk_fnew(fv[1], v[1], jj[1], c, e, fc);
        }
        for (int j = s0 + tid + NT; j < s1; j += NT) {
            const double vv = prv(j);
            prD[j] = vv;
            fn[j] = blk_fnew(fo[j], vv, j, c, e, fc);
        }
        SMX_BLK_STAMP(3);
        // the next entering column: first j < fscan with f_{k+L}[j] < 0 (simplex.py:94-98)
        int mine = SMX_NONE;
#pragma unroll
        for (int k = NJ - 1; k >= 2; --k)
            if (jj[k] < fscan && blk_fnew(fv[k], v[k], jj[k], c, e, fc) < 0.0) mine = jj[k];
        cf = block_min_int_dpp<NT>(mine, s_tmp);
        if (cf != SMX_NONE) {
            // the owner of column cf: its pivot-row value and operands for the row pass
            if (tid == cf % NT) {
#pragma unroll
                for (int k = 2; k < NJ; ++k)
                    if (k - 2 == cf / NT) {
                        s_pa = v[k];
#pragma unroll
                        for (int q = 0; q < D; ++q) s_col[2][q] = pq[k][q];
                    }
            }
        } else {
            for (int j0 = NSC * NT; j0 < fscan && cf == SMX_NONE; j0 += kBlkScan) {
                int mn = SMX_NONE;
#pragma unroll SCANU
                for (int k = 0; k < 4; ++k) {
                    const int j = j0 + k * NT + tid;
                    if (j < fscan && blk_fnew(fo[j], prv(j), j, c, e, fc) < 0.0 && j < mn) mn = j;
                }
                cf = block_min_int_dpp<NT>(mn, s_tmp);
            }
            if (tid == 0) {
                s_pa = cf != SMX_NONE ? prv(cf) : 0.0;
                if (cf != SMX_NONE)
                    for (int q = 0; q < D; ++q) s_col[2][q] = pr[(int64_t)q * ld + cf];
            }
        }
        if (tid < 2) {   // lane 0 holds column c's operands, lane 1 column m's
            if (tid == 1) s_pm = v[0];
#pragma unroll
            for (int q = 0; q < D; ++q) s_col[tid][q] = pq[0][q];
        }
        SMX_BLK_STAMP(4);
    } else {
    if (!SH && nb != SMX_NONE) {
        // phase 1: first j < m with T_{k+D}[r][j] > 0 (simplex.py:81-85), early exit by rounds
        // (sharded: the owner of the row computed it in k_bsh_pack; merge_headers returned it)
        int p1 = SMX_NONE;
        for (int j0 = 0; j0 < m && p1 == SMX_NONE; j0 += kBlkScan) {
            int mine = SMX_NONE;
#pragma unroll SCANU
            for (int k = 0; k < 4; ++k) {
                const int j = j0 + k * NT + tid;
                if (j < m && prv(j) > 0.0 && j < mine) mine = j;
            }
            p1 = block_min_int_dpp<NT>(mine, s_tmp);
        }
        if (p1 == SMX_NONE) {
            d.c = SMX_NONE;
            d.status = SMX_INCORRECT;   // simplex.py:88-89
            terminal(d);
            return true;
        }
        d.c = p1;
    }
    c = d.c;
    if (tid == 0) {
        s_e = prv(c);
        s_fc = fo[c];
        s_pm = prv(m);
    }
    __syncthreads();
    SMX_BLK_STAMP(2);
    e = s_e;
    fc = s_fc;
    // slice b of the pivot row and of the next f-row
    {
        const int S = ((C + G - 1) / G + 1) & ~1;
        const int s1 = min(C, (b + 1) * S);
        for (int j = b * S + tid; j < s1; j += NT) {
            const double v = prv(j);
            prD[j] = v;
            fn[j] = blk_fnew(fo[j], v, j, c, e, fc);
        }
    }
    SMX_BLK_STAMP(3);
    // the next entering column: first j < fscan with f_{k+L}[j] < 0 (simplex.py:94-98)
    cf = SMX_NONE;
    for (int j0 = 0; j0 < fscan && cf == SMX_NONE; j0 += kBlkScan) {
        int mine = SMX_NONE;
#pragma unroll SCANU
        for (int k = 0; k < 4; ++k) {
            const int j = j0 + k * NT + tid;
            if (j < fscan && blk_fnew(fo[j], prv(j), j, c, e, fc) < 0.0 && j < mine) mine = j;
        }
        cf = block_min_int_dpp<NT>(mine, s_tmp);
    }
    SMX_BLK_STAMP(4);
    if (tid == 0) s_pa = cf != SMX_NONE ? prv(cf) : 0.0;
    }   // the general path
    // the labels after this pivot (simplex.py:152), identically in every workgroup
    const int hx0 = move_label(ctl->xpos[sp][0], r, c);
    const int hx1 = move_label(ctl->xpos[sp][1], r, c);
    const int64_t kpiv = ctl->npiv[sp];
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
        h->r[D] = r_local;
        h->c[D] = c;
        h->e[D] = e;
        h->y[D] = fd.y;
        h->ok[D] = fd.ok ? 1 : 0;
        h->peff = D + 1;
        hs->cfs[blk_slot(L, P, bn)] = cf;
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
    // step L's pivots in LDS-broadcast form: s_pv[D] = this pivot; the pivot rows at the columns
    // the row pass reads (uniform)
    {
        __syncthreads();   // s_pa / s_pm / s_col of the phase-2 path are written before this
        if (tid == 0) {
            s_pv.r[D] = r_local;
            s_pv.c[D] = c;
            s_pv.e[D] = e;
            s_col[1][D] = s_pm;
            s_col[2][D] = s_pa;
        }
        if (tid < D && !(!SH && nb == SMX_NONE)) {   // (the phase-2 path wrote them already)
            s_col[0][tid] = pr[(int64_t)tid * ld + c];
            s_col[1][tid] = pr[(int64_t)tid * ld + m];
            if (cf != SMX_NONE) s_col[2][tid] = pr[(int64_t)tid * ld + cf];
        }
    }
    __syncthreads();
    SMX_BLK_STAMP(5);
    const int64_t hslot = 2 * (kpiv % (log_cap > 0 ? log_cap : 1));
    // x-history of this pivot: the labels' rows as local indices (their "-b" entries of T_{k+L})
    const int hl0 = hx0 >= row0 && hx0 < row0 + rows ? hx0 - row0 : -1;
    const int hl1 = hx1 >= row0 && hx1 < row0 + rows ? hx1 - row0 : -1;
    // Column cache: a column read over all rows is one 8-byte load per row, a DRAM page apart
    // each, and such reads are most of a step's time (round 4's k_blk_first, two of them per
    // row, took ~8 us at 16384 rows).  Within a block the base table is fixed, so its "-b" column is read
    // once (step 0) and the column the next step's records are built on -- the next entering
    // column in phase 2 -- is kept from the step that read it: one strided column per step
    // instead of three.
    // the row pass's shared operands in registers: the L pivots and the pivot rows at c, m, cf
    BlkPiv pvL;
    bool okL = true;
    double colv[3][kBlkMax];
    pvL = blk_pv_regs<L>(s_pv, &okL);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int q = 0; q < L; ++q) colv[k][q] = s_col[k][q];
#pragma unroll
        for (int q = 0; q < L; ++q) blk_pin(colv[k][q]);
    }
    // Chain-result cache (the register form): step L keeps T_{k+L}[i][m] and T_{k+L}[i][cf] --
    // the values its records were built on -- in cb / ca by step parity, so step L+1 takes its
    // multipliers T_{k+L}[i][c] (c = this cf in phase 2) as they are and its "-b" values with ONE
    // more step, instead of re-deriving both by chains of length L from T_k; only the new
    // column's chain remains (L+1 chain steps per row instead of 3L-1).  Same operations on the
    // same operands in the same order as the full chains, so the same bits.  (The layout's first
    // 3 R doubles after the f-rows are unused since the pipelined planner left.)
    double* cca = fr + 2 * ld + 3 * (int64_t)rows;
    double* ccb = cca + 2 * (int64_t)rows;
    const bool reuse_c = D > 0 && c == s_c;   // phase 2: c is the column of step D's records
    double* mT = blk_mulT(mul, rows + 1);
    BlkRec R{SMX_NONE, First{SMX_NONE, 0.0}, cand_none()};
    for (int i = b * NT + tid; i < rows; i += G * NT) {
        const double* row = T + (int64_t)i * ld;
        double* mr = mul + (int64_t)i * kBlkMax;
        const double xc = reuse_c ? cca[(int64_t)(D & 1) * rows + i] : row[c];
        const double xb = D > 0 ? ccb[(int64_t)(D & 1) * rows + i] : row[m];
        const double xa = cf != SMX_NONE ? row[cf] : 0.0;
        double bv, a;
        {
            double mq[kBlkMax];
            double x3[3] = {xc, xb, xa};
#pragma unroll
            for (int q = 0; q < D; ++q) mq[q] = mT[(int64_t)q * (rows + 1) + i];
#pragma unroll
            for (int q = 0; q < D; ++q) blk_pin(mq[q]);
#pragma unroll
            for (int k = 0; k < 3; ++k) blk_pin(x3[k]);
            // x3[0]: T_{k+D}[i][c] itself when cached (reuse_c), else T_k[i][c]; x3[1]:
            // T_{k+D}[i][m] (cached) from step 1 on, T_k[i][m] at step 0
            constexpr int QB = D > 0 ? D : 0;
            uint32_t wt = 0;
            mq[D] = reuse_c ? x3[0] : blk_chain_fd<D>(x3[0], i, c, pvL, colv[0], mq, wt);
            bv = blk_chain_fd<L, QB>(x3[1], i, m, pvL, colv[1], mq, wt);
            a = cf != SMX_NONE ? blk_chain_fd<L>(x3[2], i, cf, pvL, colv[2], mq, wt) : 0.0;
            if (!okL || !__all(wt < kWinSpan)) {   // some numerator outside the window
                SMX_BLK_FALLBACK(1);
                if (!reuse_c) mq[D] = blk_chain<D>(x3[0], i, c, pvL, colv[0], mq);
                bv = blk_chain<L, QB>(x3[1], i, m, pvL, colv[1], mq);
                a = cf != SMX_NONE ? blk_chain<L>(x3[2], i, cf, pvL, colv[2], mq) : 0.0;
            }
            mr[D] = mq[D];
            mT[(int64_t)D * (rows + 1) + i] = mq[D];
            ccb[(int64_t)(L & 1) * rows + i] = bv;
            if (cf != SMX_NONE) cca[(int64_t)(L & 1) * rows + i] = a;
            if (L == P) {   // the sweep's per-row flag (blk_rflags)
                bool bnd = true, zero = false, piv = false;
#pragma unroll
                for (int q = 0; q < L; ++q) {
                    bnd = bnd && bnd_or_zero(mq[q]);
                    zero = zero || (dbits(mq[q]) << 1) == 0;
                    piv = piv || i == pvL.r[q];
                }
                blk_rflags(mul, rows + 1)[i] = blk_rflag(piv, bnd, zero);
            }
        }
        if (xhist && log_cap > 0) {
            if (i == hl0) xhist[hslot] = bv;
            if (i == hl1) xhist[hslot + 1] = bv;
        }
        blk_rec_add(R, row0 + i, bv, cf != SMX_NONE, a);
    }
    SMX_BLK_STAMP(6);
    blk_rec_store(R, parts + (int64_t)blk_slot(L, P, bn) * G + b);
    SMX_BLK_STAMP(7);
    return false;
}

#define SMX_BLK_STEP_PARAMS                                                                         \
    const double* __restrict__ T, int64_t ld, int rows, int m, int flen, int fscan, int row0,      \
        int P, int parity, int bn, smx_ctl* __restrict__ ctl, BlkHdr* __restrict__ h,              \
        smx_part* __restrict__ parts, double* __restrict__ mul, double* __restrict__ pr,           \
        double* __restrict__ fr, const double* __restrict__ recv, int nranks,                      \
        int32_t* __restrict__ log, double* __restrict__ xhist, int64_t log_cap,                    \
        const double* __restrict__ xrow, int64_t xslot
#define SMX_BLK_STEP_ARGS                                                                           \
    T, ld, rows, m, flen, fscan, row0, P, parity, bn, ctl, h, parts, mul, pr, fr, recv, nranks,     \
        log, xhist, log_cap, xrow, xslot

// The register-form planner launch (row-sharded chains; unsharded with smx_tune_block_planner(1))
template <int L, bool SH>
__global__ __launch_bounds__(kBlkNT) void k_blk_step(SMX_BLK_STEP_PARAMS) {
    blk_step_body<L, SH>(SMX_BLK_STEP_ARGS);
}

#undef SMX_BLK_STEP_PARAMS
#undef SMX_BLK_STEP_ARGS

// The sweep: T_k -> T_{k+P} for every element (P = peff pivots of this block).
// Every element runs the P steps of chain() (above); the division takes the hoisted-reciprocal
// form where the operands allow it (the domains below) and the IEEE division otherwise.

// The exact path of one unit (two adjacent columns of one row): every rule of simplex.py:155-175
// with the hardware division, the pivots' rows and columns read from the header as it goes (the
// rare path: no registers held for them across the sweep).  prs(q) returns the chunk's pivot-row
// values of pivot q at this lane's two columns.
template <int P, class PRS>
__device__ __forceinline__ dbl2 blk_exact_h(dbl2 v, int row, int j, const BlkHdr* __restrict__ h,
                                            const double* eq, PRS prs, const double* pc) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const int rq = h->r[q], cq = h->c[q];
        const dbl2 p = prs(q);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int jj = j + hh;
            double num;
            if (row == rq) {
                num = (jj == cq) ? 1.0 : -v[hh];
            } else {
                const double a = v[hh] * eq[q];
                const double b = p[hh] * pc[q];
                num = (jj == cq) ? v[hh] : (a - b);
            }
            v[hh] = num / eq[q];
        }
    }
    return v;
}

// The flag-form sweep: one row per step of a wave, the planner's per-row flags (blk_rflags) instead
// of per-row checks.  The unchecked fast path needs a bounded chunk (e and the chunk's pivot-row
// values in [2^-100, 2^101), checked once per sweep), a flagged row (no pivot row, every
// multiplier bounded: the planner checked them when it computed them) and bounded inputs (one vote
// per row).  Re-checking the row's P multipliers in the sweep cost ~30 scalar and ~12 vector
// instructions per row beside the 120 fp64 ones, and the row's branch waited on them:
// tools/sweep_lab.hip, 16384^2, P = 10: 894 -> 753 us per sweep (profiles/r03/sweep_lab.jsonl).
// The fast path is straight-line: a per-pivot (uniform, never taken) branch to select a pivot
// column's numerator cost another ~20 % (lab V7 vs V6), so pivot columns are NOT special here.  On
// a flagged row the pivot column's lane computes RN(x e) - RN(e x) = +0 at its step (its element
// IS mul[i][q] there) and carries harmless finite values after it; blk_fixcols (k_blk_sweep_rest)
// then rewrites every pivot column from the planner's multipliers.  Rows or chunks outside the fast
// domain take the window-tracked path (a pivot column's zero numerator fails its vote), then the
// exact path, which applies every rule itself.
//
// Two layouts (FORM):
//  4  wave-chunk: every wave keeps one 128-column chunk (w % nchunks) for the whole pass, its
//     pivot-row slices in registers (2P doubles per lane) and e / y in scalar registers -- the
//     fastest up to ~12 pivots (profiles/r03/, tools/sweep_lab2.hip V1);
//  5  workgroup-chunk: the four waves of a workgroup share one chunk (blockIdx % nchunks) and its
//     pivot-row slices live in LDS (P KiB per workgroup), (e, y) pairs in LDS as well: ~60-70
//     VGPRs at any P, so 16-24 pivots per sweep keep 7-8 waves per SIMD instead of spilling
//     scalars (tools/sweep_lab2.hip V3 / V6, profiles/r04b/lab2.jsonl: P = 20 1.33 ms vs 1.43 ms
//     for the register layout at 16384^2).
// Diagnostic build only (-DSMX_PATH_COUNT, Makefile target `diag` -> libsmx_diag.so): how many
// (row, 128-column chunk) units of the flag-form sweep take each path, summed over every launch
// until smx_diag_path_counts reads (and optionally clears) them.  Per wave in registers, one add
// per counter and wave at the end (lane k adds counter k).  The product build has none of it.
enum : int {
    kPcFast = 0,        // chunk_free, row flag 1, bounded inputs: the unchecked fast path
    kPcZero,            // the zero-extended domain (fd_zero)
    kPcWindow,          // the window-tracked path, vote passed
    kPcWindowFail,      // the window-tracked path, vote failed -> exact
    kPcExact,           // straight to the exact path (a pivot row, or a pivot not ok)
    kPcChunkNotFree,    // units in chunks that are not chunk_free (e / pivot-row values)
    kPcChunkNotZok,     // units in chunks that are not even chunk_zok
    kPcRowFlag0,        // units of rows with flag 0 (a multiplier unbounded, not zero)
    kPcRowFlag3,        // units of rows with flag 3 (bounded or zero, at least one zero)
    kPcXFail,           // chunk_free and flag 1, but an input element out of bounds
    kPcChunkE,          // units in chunks whose pivots fail (e outside the window / bounds)
    kPcChunkP,          // units in chunks with a pivot-row value neither bounded nor zero
    kPcClkCycles,       // per wave: s_memtime ticks (shader clock) over the wave's sweep body
    kPcClkTicks,        // per wave: s_memrealtime ticks (100 MHz) over the same span
    kPcCount
};
#ifdef SMX_PATH_COUNT
__device__ unsigned long long g_path_cnt[kPcCount];
#define SMX_PC_DECL                                                                             \
    uint64_t pc_cnt[kPcCount] = {};                                                             \
    const uint64_t pc_t0 = __builtin_amdgcn_s_memtime();                                        \
    const uint64_t pc_r0 = __builtin_amdgcn_s_memrealtime();
#define SMX_PC(k) (++pc_cnt[(k)])
#define SMX_PC_FLUSH                                                                            \
    do {                                                                                        \
        pc_cnt[kPcClkCycles] = __builtin_amdgcn_s_memtime() - pc_t0;                            \
        pc_cnt[kPcClkTicks] = __builtin_amdgcn_s_memrealtime() - pc_r0;                         \
        const int l_ = threadIdx.x & (kWave - 1);                                               \
        uint64_t v_ = 0;                                                                        \
        _Pragma("unroll") for (int k_ = 0; k_ < kPcCount; ++k_) if (l_ == k_) v_ = pc_cnt[k_];  \
        if (l_ < kPcCount && v_) atomicAdd(&g_path_cnt[l_], (unsigned long long)v_);            \
    } while (0)
#else
#define SMX_PC_DECL
#define SMX_PC(k) ((void)0)
#define SMX_PC_FLUSH ((void)0)
#endif

// FORM 6 (round 6): the LDS layout in work items.  A workgroup of FORM 5 keeps one chunk for all
// its rows, so where a few chunks run a slower path (config 5's block 0: 5 of 257 chunks on the
// window-tracked path) their workgroups finish last and the sweep waits for them (1.33x block 2's
// cycles at 1.05x its instructions).  FORM 6 cuts every workgroup's rows into K
// contiguous segments (K = g_sweep_items) and takes segment k at chunk (c0 + k * stride) mod
// nchunks, stride ~ nchunks / K: for every k the map c0 -> chunk is a shift, so each (chunk,
// segment) is still swept by exactly the workgroups that would have swept it, and a slow chunk's
// rows spread over ~K times as many workgroups.  The pivot-row slices are restaged per item.
__device__ int g_sweep_items = 16;

template <int P, int FORM>
__device__ __forceinline__ void blk_sweep_body_flag(const double* Tin, double* Tout, int64_t ld,
                                                    int R, int C, const BlkHdr* __restrict__ h,
                                                    const double* __restrict__ pr,
                                                    const double* __restrict__ mul) {
    constexpr bool LDS = FORM >= 5;
    constexpr bool ITEMS = FORM == 6;
    __shared__ dbl2 s_pr[LDS ? P : 1][kWave];
    __shared__ dbl2 s_ey[LDS ? P : 1];
    // the zero-extended path's scalars (fd_zneg): the chain carries g_q = -sgn(e_q) x_{q+1}, so
    // step q's product x_q e_q is g_{q-1} M_q with M_q = -sgn(e_{q-1}) e_q (M_0 = e_0, exact sign
    // flips), the divisor |M_q| = |e_q| (a source modifier), the reciprocal |y_q|; the element
    // after the block is s_zf g_{P-1}, s_zf = -sgn(e_{P-1})
    // (the LDS layout only: in the register layout, whose e / y sit in scalar registers, the
    // per-pivot LDS reads cost more than the fixup saved -- config 5 at 12 pivots per sweep, block
    // 0 unchanged and the fast-path blocks 13 % slower, profiles/r06aa/)
    __shared__ dbl2 s_zm[LDS ? P : 1];
    __shared__ double s_zf;
    const int32_t* __restrict__ rfl = blk_rflags(mul, R);
    const int lane = threadIdx.x & (kWave - 1);
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the pivots' rows and columns are NOT held here: the row flags say which rows are pivot
    // rows, and only the exact path (blk_exact_h) needs the indices, which it reads from h --
    // 2P fewer scalar registers (and spills) in the loop
    double eq[LDS ? 1 : P], yq[LDS ? 1 : P];
    bool allok = true;
#pragma unroll
    for (int q = 0; q < P; ++q) allok = allok && h->ok[q] != 0;
    constexpr int kChunk = 2 * kWave;
    const int nchunks = (C + kChunk - 1) / kChunk;
    int ch, base, qs;
    int c0 = 0, K = 1, stride = 1, seg = R;
    if constexpr (LDS) {
        ch = (int)blockIdx.x % nchunks;
        base = ((int)blockIdx.x / nchunks) * kUpdWaves + wib;
        qs = ((int)gridDim.x / nchunks) * kUpdWaves;
        if constexpr (ITEMS) {
            c0 = ch;
            K = max(1, min(g_sweep_items, nchunks));
            stride = max(1, nchunks / K);
            seg = ((R + K - 1) / K + qs - 1) / qs * qs;   // a multiple of qs: the same interleave
        }
    } else {
        const int NW = (int)gridDim.x * kUpdWaves;
        const int w = (int)blockIdx.x * kUpdWaves + wib;
        ch = w % nchunks;
        base = w / nchunks;
        qs = NW / nchunks;
    }
    int j = ch * kChunk + 2 * lane;
    dbl2 prs[LDS ? 1 : P];
    auto stage = [&]() {
        for (int t = threadIdx.x; t < P * kWave; t += kUpdBlock) {
            const int q = t / kWave, jl = ch * kChunk + 2 * (t % kWave);
            s_pr[q][t % kWave] = jl < C ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + jl)
                                        : dbl2{0.0, 0.0};
        }
    };
    if constexpr (LDS) {
        stage();
        if (threadIdx.x < P) {
            const int q = threadIdx.x;
            const double e = h->e[q];
            s_ey[q] = dbl2{e, h->y[q]};
            const double M = q == 0 ? e : (h->e[q - 1] < 0.0 ? e : -e);
            s_zm[q] = dbl2{M, fabs(h->y[q])};
            if (q == P - 1) s_zf = e < 0.0 ? 1.0 : -1.0;
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int q = 0; q < P; ++q) {
            eq[q] = h->e[q];
            yq[q] = h->y[q];
            prs[q] = (j < C) ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j)
                             : dbl2{0.0, 0.0};
        }
    }
    auto PR = [&](int q) -> dbl2 {
        if constexpr (LDS) return s_pr[q][lane];
        else return prs[q];
    };
    auto EY = [&](int q) -> dbl2 {
        if constexpr (LDS) return s_ey[q];
        else return dbl2{eq[q], yq[q]};
    };
    const bool kNoFree = g_blk_nofree != 0;
    SMX_PC_DECL
    bool chunk_zok, chunk_free;
    auto chunk_flags = [&]() {
        uint32_t et = 0, pt = 0;
        bool zok = true;   // every pivot-row value bounded or an exact +-0
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const dbl2 p = PR(q);
            et = max(et, bnd_term(EY(q)[0]));
            if (j < C) {
                pt = max(pt, bnd_term(p[0]));
                zok = zok && bnd_or_zero(p[0]);
            }
            if (j + 1 < C) {
                pt = max(pt, bnd_term(p[1]));
                zok = zok && bnd_or_zero(p[1]);
            }
        }
        // chunk_free: bounded, no zeros (fast path); chunk_zok: bounded or zero (zero-safe path)
        chunk_zok = !kNoFree && allok && et < kBndSpan && __all(zok);
        chunk_free = chunk_zok && __all(pt < kBndSpan);
    };
    chunk_flags();
    double eqa[P];   // the exact path's pivot elements (loaded there, rare)
    // Every vector load of the loop is this inline asm: a load the compiler can see (the slow
    // path's reload) made it put s_waitcnt vmcnt(0) at the head of the fast path, waiting for
    // the next row's prefetch before computing this row (sweep 990 us at P = 10, 16384^2, against
    // 750 us for the lab's loop, tools/sweep_lab.hip).
    int jc = min(j, (C - 1) & ~1);
    auto ldc = [&](int row) {
        dbl2 v;
        const double* p = Tin + (int64_t)min(row, R - 1) * ld + jc;
        asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
        return v;
    };
    auto rowf = [&](dbl2 x0, int i0) {
        const double* m0 = mul + (int64_t)i0 * kBlkMax;
        double pc0[P];
#pragma unroll
        for (int q = 0; q < P; ++q) pc0[q] = m0[q];
        int rf = rfl[i0];
        // the row's flag and multipliers in ONE scalar round trip: left alone, the compiler
        // waits for the flag, branches, and only then issues the multipliers' loads
#pragma unroll
        for (int q = 0; q < P; ++q) asm volatile("" : "+s"(pc0[q]));
        asm volatile("" : "+s"(rf));
        dbl2 v0 = x0;
        bool ok = false;
        const uint32_t xt = max((uint32_t)__double2hiint(x0[0]) << 1,
                                (uint32_t)__double2hiint(x0[1]) << 1);
#ifdef SMX_PATH_COUNT
        if (!chunk_free) SMX_PC(kPcChunkNotFree);
        if (!chunk_zok) SMX_PC(kPcChunkNotZok);
        if (!(allok && et < kBndSpan)) SMX_PC(kPcChunkE);
        if (!__all(zok)) SMX_PC(kPcChunkP);
        if (rf == 0) SMX_PC(kPcRowFlag0);
        if (rf == 3) SMX_PC(kPcRowFlag3);
        if (chunk_free && rf == 1 && !__all(xt < kBndXMax)) SMX_PC(kPcXFail);
#endif
        if (chunk_free && rf == 1 && __all(xt < kBndXMax)) {
            SMX_PC(kPcFast);
            if constexpr (!LDS) {
                // the 2P products p * mq first (they do not depend on the chain) and held there:
                // issued back to back, the chains after them run without waiting on any
                // (tools/sweep_lab.hip V1: this order, 750-770 us at P = 10, 16384^2; interleaved
                // with the chains as the compiler otherwise places them, ~850 us)
                dbl2 bq[P];
#pragma unroll
                for (int q = 0; q < P; ++q)
                    bq[q] = dbl2{prs[q][0] * pc0[q], prs[q][1] * pc0[q]};
#pragma unroll
                for (int q = 0; q < P; ++q) asm volatile("" : "+v"(bq[q]));
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    const double e = eq[q], y = yq[q];
                    double n[2];
                    n[0] = v0[0] * e - bq[q][0];
                    n[1] = v0[1] * e - bq[q][1];
                    double rr[2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const double tq = n[k] * y;
                        const double r = fma(-e, tq, n[k]);
                        rr[k] = fma(r, y, tq);
                    }
                    v0 = dbl2{rr[0], rr[1]};
                }
            } else {
                // products inline: the slices and (e, y) come from LDS per pivot, few registers
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    const dbl2 p = s_pr[q][lane];
                    const dbl2 ey = s_ey[q];
                    const double e = ey[0], y = ey[1];
                    double n[2];
                    n[0] = v0[0] * e - p[0] * pc0[q];
                    n[1] = v0[1] * e - p[1] * pc0[q];
                    double rr[2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const double tq = n[k] * y;
                        const double r = fma(-e, tq, n[k]);
                        rr[k] = fma(r, y, tq);
                    }
                    v0 = dbl2{rr[0], rr[1]};
                }
            }
            ok = true;
        } else if (chunk_zok && (rf & 1) && __all(bnd_or_zero(x0[0]) && bnd_or_zero(x0[1]))) {
            // the zero-extended domain (rf 1 or 3, a chunk or row with exact zeros): the same
            // arithmetic, the division made zero-safe -- the register layout with fd_zero's
            // v_div_fixup (one more instruction per element-pivot), the LDS layout with the
            // sign-folded negated division (fd_zneg, s_zm: the fast path's instruction count;
            // DESIGN 20.4)
            asm volatile("" ::: "memory");   // keeps this path out of the fast path's code
            SMX_PC(kPcZero);
            if constexpr (!LDS) {
                // the 2P products first, as on the fast path (they do not depend on the chain)
                dbl2 bq[P];
#pragma unroll
                for (int q = 0; q < P; ++q)
                    bq[q] = dbl2{prs[q][0] * pc0[q], prs[q][1] * pc0[q]};
#pragma unroll
                for (int q = 0; q < P; ++q) asm volatile("" : "+v"(bq[q]));
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    const double e = eq[q], y = yq[q];
                    const double n0 = v0[0] * e - bq[q][0];
                    const double n1 = v0[1] * e - bq[q][1];
                    v0 = dbl2{fd_zero(n0, e, y), fd_zero(n1, e, y)};
                }
            } else {
#pragma unroll
                for (int q = 0; q < P && !SMX_ZNEG; ++q) {
                    const dbl2 p = PR(q);
                    const dbl2 ey = EY(q);
                    const double e = ey[0], y = ey[1];
                    double n[2];
                    n[0] = v0[0] * e - p[0] * pc0[q];
                    n[1] = v0[1] * e - p[1] * pc0[q];
                    v0 = dbl2{fd_zero(n[0], e, y), fd_zero(n[1], e, y)};
                }
#pragma unroll
                for (int q = 0; q < P && SMX_ZNEG; ++q) {
                    const dbl2 p = PR(q);
                    const dbl2 my = s_zm[q];
                    const double M = my[0], ya = my[1];
                    double n[2];
                    n[0] = v0[0] * M - p[0] * pc0[q];
                    n[1] = v0[1] * M - p[1] * pc0[q];
                    v0 = dbl2{fd_zneg(n[0], fabs(M), ya), fd_zneg(n[1], fabs(M), ya)};
                }
            }
            if (LDS && SMX_ZNEG) v0 = dbl2{v0[0] * s_zf, v0[1] * s_zf};
            ok = true;
        } else if (allok && rf != 2) {   // not a pivot row (rf == 2): the window-tracked path
            // numerators checked once per row by a vote.  Exact zeros are inside the domain too
            // (round 6): fd_zero's v_div_fixup gives a zero numerator its sign, every other
            // numerator must lie in the exponent window (a finite nonzero one in it, a normal
            // quotient: div_fixup returns the hoisted sequence's quotient unchanged).  A pivot
            // column's lane computes RN(x e) - RN(e x) = +0 at its step like on the fast path and
            // is rewritten by blk_fixcols.  (Counting zeros as outside sent every unit of a chunk
            // with a pivot-row value outside the bounds to the exact path on config 5's integer
            // tables -- a few chunks' waves 5-10x slower than the rest, block 0 at 2x block 2's
            // time with ~1.2x its instructions: profiles/r06i/7_paths.log, 8_pmcpaths/.)
            uint32_t wt = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const dbl2 p = PR(q);
                const dbl2 ey = EY(q);
                const double e = ey[0], y = ey[1];
                double n[2];
                n[0] = v0[0] * e - p[0] * pc0[q];
                n[1] = v0[1] * e - p[1] * pc0[q];
                double rr[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const uint32_t tk = win_term(n[k]);
                    wt = max(wt, (dbits(n[k]) << 1) == 0 ? 0u : tk);
                    rr[k] = fd_zero(n[k], e, y);
                }
                v0 = dbl2{rr[0], rr[1]};
            }
            ok = __all(wt < kWinSpan);
            SMX_PC(ok ? kPcWindow : kPcWindowFail);
        } else {
            SMX_PC(kPcExact);
        }
        if (!ok) {
            // reloaded (not written yet, even in place) so x0 need not stay live beside the
            // fast arithmetic; the wait covers the next row's prefetch too (rare path)
            x0 = ldc(i0);
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(x0) :: "memory");
#pragma unroll
            for (int q = 0; q < P; ++q) eqa[q] = h->e[q];
            v0 = blk_exact_h<P>(x0, i0, j, h, eqa, PR, pc0);
        }
        if (j < C)
            __builtin_nontemporal_store(v0, reinterpret_cast<dbl2*>(Tout + (int64_t)i0 * ld + j));
    };
    if constexpr (!ITEMS) {
        if (base >= R) return;
    }
    for (int it = 0; it < K; ++it) {
        int lo = 0, hi = R;
        if constexpr (ITEMS) {
            lo = it * seg;
            hi = min(R, lo + seg);
            if (it > 0) {
                // the next item's chunk: every wave is done with the previous slices first
                ch = (c0 + it * stride) % nchunks;
                j = ch * kChunk + 2 * lane;
                jc = min(j, (C - 1) & ~1);
                __syncthreads();
                stage();
                __syncthreads();
                chunk_flags();
            }
            if (lo + base >= hi) continue;   // (every wave still meets the barriers above)
        }
        // prefetch depth 1 over single rows: before a register set is used, the ops issued after
        // its load are the previous row's store and the other set's load (vmcnt(2); vmcnt(1)
        // first)
        const int r0 = lo + base;
        dbl2 a = ldc(r0), b = ldc(r0 + qs);
        asm volatile("s_waitcnt vmcnt(1)" : "+v"(a) :: "memory");
        for (int i0 = r0; i0 < hi; i0 += 2 * qs) {
            rowf(a, i0);
            if (i0 + qs >= hi) break;
            a = ldc(i0 + 2 * qs);
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(b) :: "memory");
            rowf(b, i0 + qs);
            if (i0 + 2 * qs >= hi) break;
            b = ldc(i0 + 3 * qs);
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(a) :: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    SMX_PC_FLUSH;   // every exit of the loop lands here (diagnostic build only)
}

// After a flag-form sweep: every element of every pivot column, rewritten from the planner's
// multipliers.  For column c whose LAST pivot in the block is q, the element's value before step q
// is T_{k+q}[i][c] = mul[i][q] (bit for bit, the planner's own chain), so its steps q..P-1 follow
// from mul alone: step q's numerator is the element itself, or 1.0 on the pivot row
// (simplex.py:155-160); later steps apply the full rules with the exact division.  Writes `out`,
// the buffer the sweep wrote.  One (row, pivot) pair per thread, grid-stride.
__device__ __forceinline__ void blk_fixcols(double* out, int64_t ld, int R, int P,
                                            const BlkHdr* __restrict__ h,
                                            const double* __restrict__ mul,
                                            const double* __restrict__ pr) {
    // pairs ordered pivot-major (t = q R + i): a wave's lanes share q, so the pivot rows' values
    // at column c are one address per load; every operand of the chain is loaded before its
    // first step (the loop that loaded them step by step took 9-13 us per block at 16384^2 --
    // a memory round trip per step).  Row i's multipliers come from the transposed copy (the
    // planner's row pass writes it for every row but the f-row, R - 1): a wave's 64 rows are
    // then 8 lines per multiplier instead of 64.
    const double* mT = blk_mulT(mul, R);
    const int64_t pairs = (int64_t)R * P;
    for (int64_t t = (int64_t)blockIdx.x * kUpdBlock + threadIdx.x; t < pairs;
         t += (int64_t)gridDim.x * kUpdBlock) {
        const int q = (int)(t / R), i = (int)(t % R);
        const int c = h->c[q];
        bool last = true;
        for (int q2 = q + 1; q2 < P; ++q2) last = last && h->c[q2] != c;
        if (!last) continue;
        const double* mr = mul + (int64_t)i * kBlkMax;
        const bool frow = i == R - 1;
        double mq[kBlkMax], pc[kBlkMax], eq[kBlkMax];
        int rq[kBlkMax];
#pragma unroll
        for (int q2 = 0; q2 < kBlkMax; ++q2) {
            const bool act = q2 >= q && q2 < P;
            mq[q2] = act ? (frow ? mr[q2] : mT[(int64_t)q2 * R + i]) : 0.0;
            pc[q2] = (act && q2 > q) ? pr[(int64_t)q2 * ld + c] : 0.0;
            eq[q2] = act ? h->e[q2] : 1.0;
            rq[q2] = act ? h->r[q2] : -1;
        }
        double x = 0.0;
#pragma unroll
        for (int q2 = 0; q2 < kBlkMax; ++q2) {
            if (q2 < q || q2 >= P) continue;
            double num;
            if (q2 == q)
                num = (i == rq[q2]) ? 1.0 : mq[q2];
            else if (i == rq[q2])
                num = -x;   // c is not pivot q2's column (q is its last pivot)
            else
                num = x * eq[q2] - pc[q2] * mq[q2];
            x = num / eq[q2];
        }
        out[(int64_t)i * ld + c] = x;
    }
}

// Output: in place when ipx >= 0 and ipx + (pivots applied) is even, else into b_other; the
// chain state's loc records which buffer (in_idx = index of b_in) now holds the newest table.
__device__ __forceinline__ double* blk_out(double* b_in, double* b_other, int ipx, int in_idx,
                                           int applied, BlkHdr* __restrict__ hs) {
    const bool inplace = ipx >= 0 && ((ipx + applied) & 1) == 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) hs->loc = inplace ? in_idx : in_idx ^ 1;
    return inplace ? b_in : b_other;
}

// The sweep of a block that applied all P of its pivots (h->peff == P; otherwise it does nothing
// and k_blk_sweep_rest handles the block): one body per kernel, so the register allocation is
// that body's alone.  FORM 4 / 5: blk_sweep_body_flag's layouts.  Output per blk_out.
template <int P, int FORM>
__global__ __launch_bounds__(kUpdBlock) void k_blk_sweep(double* b_in, double* b_other, int64_t ld,
                                                         int R, int C,
                                                         const BlkHdr* __restrict__ h,
                                                         const double* __restrict__ mul,
                                                         const double* __restrict__ pr,
                                                         BlkHdr* __restrict__ hs, int ipx,
                                                         int in_idx) {
    if (h->peff != P) return;
    double* out = blk_out(b_in, b_other, ipx, in_idx, P, hs);
    blk_sweep_body_flag<P, FORM>(b_in, out, ld, R, C, h, pr, mul);
}

// End of a block chain: the state of the final table into ctl slot `parity` (first negative
// "-b" row from the records, first negative f-row entry from the chain state); one full wave.
__device__ __forceinline__ void blk_publish_wave(const BlkHdr* __restrict__ h,
                                                 const smx_part* __restrict__ parts, int nparts,
                                                 int slot, int parity, smx_ctl* __restrict__ ctl) {
    if (ctl->term) return;
    const smx_part* sp = parts + (int64_t)slot * nparts;
    int nb = SMX_NONE;
    for (int k = threadIdx.x; k < nparts; k += kWave) nb = min(nb, sp[k].p1col);
    nb = wave_min_int_dpp(nb);
    if (threadIdx.x == 0) {
        ctl->negb[parity] = nb;
        ctl->negf[parity] = h->cfs[slot];
        ctl->negb[parity ^ 1] = SMX_NONE;
        ctl->negf[parity ^ 1] = SMX_NONE;
    }
}

// After k_blk_sweep<P> (one launch, whichever case holds):
// * fix = 1 and the block applied all P pivots (flag form): blk_fixcols, the pivot columns;
// * a block that stopped early (a terminal outcome after 0 < peff < P pivots; once per LP):
//   every element through the peff pivots with the exact division, a rolled loop reading each
//   pivot's operands as it goes -- one small kernel for every count instead of a body per count;
// * otherwise nothing.
// * pctl != nullptr (the chain's last block): workgroup 0's first wave also publishes the chain's
//   final state (k_blk_publish's work, one launch and its gap fewer per chain).
__global__ __launch_bounds__(kUpdBlock) void k_blk_sweep_rest(double* b_in, double* b_other,
                                                              int64_t ld, int R, int C, int P,
                                                              const BlkHdr* __restrict__ h,
                                                              const double* __restrict__ mul,
                                                              const double* __restrict__ pr,
                                                              BlkHdr* __restrict__ hs, int ipx,
                                                              int in_idx, int fix, int ipx_full,
                                                              const smx_part* __restrict__ pparts,
                                                              int pnparts, int pslot, int pparity,
                                                              smx_ctl* __restrict__ pctl) {
    if (pctl != nullptr && blockIdx.x == 0 && threadIdx.x < kWave)
        blk_publish_wave(hs, pparts, pnparts, pslot, pparity, pctl);
    const int peff = h->peff;
    if (peff == P && fix) {
        double* out = (ipx_full >= 0 && ((ipx_full + P) & 1) == 0) ? b_in : b_other;
        blk_fixcols(out, ld, R, P, h, mul, pr);
        return;
    }
    if (peff <= 0 || peff >= P) return;
    double* out = blk_out(b_in, b_other, ipx, in_idx, peff, hs);
    const int64_t half = (C + 1) / 2;   // dbl2 units per row (ld is even)
    const int64_t units = (int64_t)R * half;
    for (int64_t u = (int64_t)blockIdx.x * kUpdBlock + threadIdx.x; u < units;
         u += (int64_t)gridDim.x * kUpdBlock) {
        const int i = (int)(u / half);
        const int j = (int)(u % half) * 2;
        double v[2] = {b_in[(int64_t)i * ld + j], j + 1 < C ? b_in[(int64_t)i * ld + j + 1] : 0.0};
        for (int q = 0; q < peff; ++q) {
            const int rq = h->r[q], cq = h->c[q];
            const double eq = h->e[q], mq = mul[(int64_t)i * kBlkMax + q];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int jj = j + hh;
                double num;
                if (i == rq) {
                    num = (jj == cq) ? 1.0 : -v[hh];
                } else {
                    const double a = v[hh] * eq;
                    const double b = pr[(int64_t)q * ld + (jj < C ? jj : j)] * mq;
                    num = (jj == cq) ? v[hh] : (a - b);
                }
                v[hh] = num / eq;
            }
        }
        out[(int64_t)i * ld + j] = v[0];
        if (j + 1 < C) out[(int64_t)i * ld + j + 1] = v[1];
    }
}

// End of a block chain: the state of the final table into ctl slot `parity` (first negative
// "-b" row from the next step's records, entering column from its cf slot), like k_publish.
__global__ __launch_bounds__(kWave) void k_blk_publish(const BlkHdr* __restrict__ h,
                                                       const smx_part* __restrict__ parts,
                                                       int nparts, int slot, int parity,
                                                       smx_ctl* __restrict__ ctl) {
    blk_publish_wave(h, parts, nparts, slot, parity, ctl);
}

}  // namespace
