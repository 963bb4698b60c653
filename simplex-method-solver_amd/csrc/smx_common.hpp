// smx_common.hpp -- constants, ratio-test order, wave reductions, the decision from partials and from gathered shard headers
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

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

// (Branch-free: the reductions below run these per lane, and "if (better(o, a)) a = o" on a
// struct compiled to exec-masked branch regions -- ~770 instructions and ~1.8 us for a wave's
// three reductions and a merge in the persistent planner, profiles/r06o/.  Same order.)
__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
    const bool c0 = (a.v > b.v) | ((a.v == b.v) & (a.idx > b.idx));
    const bool cx = a.idx < b.idx;
    return (a.cls < b.cls) | ((a.cls == b.cls) & (a.cls == 0 ? c0 : cx));
}
__device__ __forceinline__ Cand cand_sel(bool t, const Cand& a, const Cand& b) {
    return Cand{t ? a.cls : b.cls, t ? a.idx : b.idx, t ? a.v : b.v};
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

__device__ __forceinline__ First first_sel(bool t, const First& a, const First& b) {
    return First{t ? a.idx : b.idx, t ? a.v : b.v};
}

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
        a = cand_sel(better(o, a), o, a);
    }
    return a;
}

__device__ __forceinline__ First wave_first(First a) {
#pragma unroll
    for (int mask = 32; mask >= 1; mask >>= 1) {
        First o = shfl_xor_first(a, mask);
        a = first_sel(o.idx < a.idx, o, a);
    }
    return a;
}

// The same three reductions through DPP instead of LDS-crossbar shuffles (the planner's per-step
// decision and record merge, smx_block.hpp): lane pairs within quads (quad_perm), then the
// half-row and row mirrors (lane i <-> 7 - i, 15 - i) leave every lane of a 16-lane row holding
// its row's result; the four rows' results are then read from lanes 0 / 16 / 32 / 48 into scalar
// registers and combined.  Each "take" is a strict total order (ties only between identical
// values), so any pairing gives the butterfly's result bit for bit.  The whole wave must be active.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
    return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    return __hiloint2double(dpp_i<CTRL>(__double2hiint(x)), dpp_i<CTRL>(__double2loint(x)));
}
__device__ __forceinline__ double readlane_d(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}
constexpr int kDppXor1 = 0xB1;     // quad_perm [1, 0, 3, 2]
constexpr int kDppXor2 = 0x4E;     // quad_perm [2, 3, 0, 1]
constexpr int kDppHalfMirror = 0x141;
constexpr int kDppMirror = 0x140;

__device__ __forceinline__ int wave_min_int_dpp(int x) {
    x = min(x, dpp_i<kDppXor1>(x));
    x = min(x, dpp_i<kDppXor2>(x));
    x = min(x, dpp_i<kDppHalfMirror>(x));
    x = min(x, dpp_i<kDppMirror>(x));
    const int a = min(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16));
    const int b = min(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48));
    return min(a, b);
}

template <int CTRL>
__device__ __forceinline__ Cand dpp_cand(const Cand& a) {
    return Cand{dpp_i<CTRL>(a.cls), dpp_i<CTRL>(a.idx), dpp_d<CTRL>(a.v)};
}
__device__ __forceinline__ Cand readlane_cand(const Cand& a, int l) {
    return Cand{__builtin_amdgcn_readlane(a.cls, l), __builtin_amdgcn_readlane(a.idx, l),
                readlane_d(a.v, l)};
}
__device__ __forceinline__ Cand wave_best_dpp(Cand a) {
    Cand o = dpp_cand<kDppXor1>(a);
    a = cand_sel(better(o, a), o, a);
    o = dpp_cand<kDppXor2>(a);
    a = cand_sel(better(o, a), o, a);
    o = dpp_cand<kDppHalfMirror>(a);
    a = cand_sel(better(o, a), o, a);
    o = dpp_cand<kDppMirror>(a);
    a = cand_sel(better(o, a), o, a);
    Cand r = readlane_cand(a, 0);
#pragma unroll
    for (int l = 16; l < kWave; l += 16) {
        o = readlane_cand(a, l);
        r = cand_sel(better(o, r), o, r);
    }
    return r;
}

template <int CTRL>
__device__ __forceinline__ First dpp_first(const First& a) {
    return First{dpp_i<CTRL>(a.idx), dpp_d<CTRL>(a.v)};
}
__device__ __forceinline__ First wave_first_dpp(First a) {
    First o = dpp_first<kDppXor1>(a);
    a = first_sel(o.idx < a.idx, o, a);
    o = dpp_first<kDppXor2>(a);
    a = first_sel(o.idx < a.idx, o, a);
    o = dpp_first<kDppHalfMirror>(a);
    a = first_sel(o.idx < a.idx, o, a);
    o = dpp_first<kDppMirror>(a);
    a = first_sel(o.idx < a.idx, o, a);
    First r{__builtin_amdgcn_readlane(a.idx, 0), readlane_d(a.v, 0)};
#pragma unroll
    for (int l = 16; l < kWave; l += 16) {
        o = First{__builtin_amdgcn_readlane(a.idx, l), readlane_d(a.v, l)};
        r = first_sel(o.idx < r.idx, o, r);
    }
    return r;
}

// Lexicographic (key, row) maximum over the wave by DPP (the resident loop's class-0 ratio:
// the largest key, ties to the larger row); every lane gets the result.  Whole wave active.
struct KeyRow {
    unsigned long long key;
    int row;
};
template <int CTRL>
__device__ __forceinline__ KeyRow dpp_keyrow(const KeyRow& a) {
    const unsigned lo = (unsigned)dpp_i<CTRL>((int)(unsigned)a.key);
    const unsigned hi = (unsigned)dpp_i<CTRL>((int)(unsigned)(a.key >> 32));
    return KeyRow{((unsigned long long)hi << 32) | lo, dpp_i<CTRL>(a.row)};
}
__device__ __forceinline__ bool keyrow_gt(const KeyRow& a, const KeyRow& b) {
    return a.key > b.key || (a.key == b.key && a.row > b.row);
}
__device__ __forceinline__ KeyRow readlane_keyrow(const KeyRow& a, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)a.key, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(a.key >> 32), l);
    return KeyRow{((unsigned long long)hi << 32) | lo, __builtin_amdgcn_readlane(a.row, l)};
}
__device__ __forceinline__ KeyRow wave_max_keyrow_dpp(KeyRow a) {
    KeyRow o = dpp_keyrow<kDppXor1>(a);
    if (keyrow_gt(o, a)) a = o;
    o = dpp_keyrow<kDppXor2>(a);
    if (keyrow_gt(o, a)) a = o;
    o = dpp_keyrow<kDppHalfMirror>(a);
    if (keyrow_gt(o, a)) a = o;
    o = dpp_keyrow<kDppMirror>(a);
    if (keyrow_gt(o, a)) a = o;
    KeyRow r = readlane_keyrow(a, 0);
#pragma unroll
    for (int l = 16; l < kWave; l += 16) {
        o = readlane_keyrow(a, l);
        if (keyrow_gt(o, r)) r = o;
    }
    return r;
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

// `slot`: stride of the gathered headers (the full send slot, SMX_SHARD_HDR + 2 * ld, or just
// SMX_SHARD_HDR when only the headers were gathered; `off` then still names the row in the
// owner's own send slot as owner * slot + (SMX_SHARD_HDR or SMX_SHARD_HDR + ld))
__device__ ShardDecision merge_headers_s(const double* __restrict__ recv, int nranks, int64_t ld,
                                         int m, int flen, int64_t slot) {
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

__device__ ShardDecision merge_headers(const double* __restrict__ recv, int nranks, int64_t ld,
                                       int m, int flen) {
    return merge_headers_s(recv, nranks, ld, m, flen, SMX_SHARD_HDR + 2 * ld);
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

}  // namespace
