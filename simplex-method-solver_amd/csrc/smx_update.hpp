// smx_update.hpp -- k_update: the Jordan step (recalculate_matrix, simplex.py:143-177) in all its modes
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
#pragma once
#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------------------------------------
// k_update: the modified Jordan step (simplex.py:149-177), out of place.
//
// Streaming shape (measured on MI355X with tools/hbm_probe.hip: a grid-wide sweep in address
// order, where every resident wave works inside one narrow moving window of the tableau, streams
// faster than per-wave private regions).  A unit is one row x one chunk of 64 lanes x 2 doubles
// (1 KiB); unit u = row * nchunks + chunk; wave w takes units w, w + NW, w + 2 NW, ... in
// batches of U (U 16-B loads in flight per lane before any arithmetic).  When NW is a multiple
// of nchunks a wave always sees the same chunk, so its pivot-row slice stays in registers.
// T[i][c] is a wave-uniform scalar load per unit.  Per element:
//     num = (i == r) ? (j == c ? 1.0 : -x)          steps 1 and 3
//                    : (j == c ? x   : x*e - pr*pc) steps 2 and 4
//     out = num / e
// which is exactly the value the reference leaves in new_table[i][j] after steps 1-4.
//
// Modes: kSingle (decision from k_select's partials), kShard (decision merged from the gathered
// shard headers, nparts = rank count), kForced (given r, c), kFused / kShardFused (as kSingle /
// kShard, plus look-ahead workgroups [0, nparts) writing the next step's records; in these modes
// forced_r = 1 when the look-ahead workgroups also sweep, and kShardFused's rank count is
// forced_c).
enum UpdMode { kSingle = 0, kShard = 1, kForced = 2, kFused = 3, kShardFused = 4 };

#ifdef SMX_TRACE
// Diagnostic build only (tools/trace_fused.hip): per-workgroup s_memrealtime stamps (100 MHz,
// chip-wide) of the last two update launches, [launch parity][block][phase]:
// 0 entry, 1 decision known, 2 look-ahead records written, 3 sweep done.
constexpr int kTraceBlocks = 4096;
__device__ unsigned long long g_trace[2][kTraceBlocks][4];
#define SMX_STAMP(ph)                                                                  \
    do {                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < kTraceBlocks)                             \
            g_trace[parity & 1][blockIdx.x][ph] = __builtin_amdgcn_s_memrealtime();    \
    } while (0)
#else
#define SMX_STAMP(ph) \
    do {              \
    } while (0)
#endif

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NTL>
__device__ __forceinline__ dbl2 ld2(const double* p) {
    if (NTL) return __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(p));
    return *reinterpret_cast<const dbl2*>(p);
}

// One batch = U units of this wave: their rows, chunks and the 16-B tableau slices.
template <int U>
struct Batch {
    int i[U], ch[U];
    dbl2 x[U];
    double pc[U];
};

// DIAG (timing only, never selectable in normal use): multiply by 1/e instead of dividing.
template <int MODE, int U, bool NTS, bool NTL, bool PIPE, bool DIAG = false>
__global__ __launch_bounds__(kUpdBlock) void k_update(
    const double* __restrict__ Tin, double* __restrict__ Tout, int64_t ld, int rows_local,
    int n, int m, int flen, int fscan, int row0, int parity, smx_ctl* __restrict__ ctl,
    const smx_part* __restrict__ parts, int nparts, int32_t* __restrict__ log,
    double* __restrict__ xhist, int64_t log_cap, const double* __restrict__ recv, int forced_r,
    int forced_c, double* __restrict__ send) {
    __shared__ int s_dec[3];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    if (MODE != kForced && ctl->term) return;
    SMX_STAMP(0);
    const int R = rows_local + 1;  // + the f-row (local row rows_local)
    const int C = m + 1;
    constexpr int kChunk = kWave * 2;                  // doubles per unit
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int64_t units = (int64_t)nchunks * R;
    // kFused: workgroups [0, nparts) compute the look-ahead records; they join the sweep only
    // when forced_r (= "look-ahead sweeps") is set: tableaux beyond the Infinity Cache, whose
    // stream needs every resident wave's loads in flight (launch_update_mode)
    constexpr bool LA = MODE == kFused || MODE == kShardFused;
    const bool la_sweep = LA && forced_r != 0;
    const int lab = (LA && !la_sweep) ? nparts : 0;
    const bool la = LA && (int)blockIdx.x < nparts;
    const bool sweeps = !la || la_sweep;
    const int NW = ((int)gridDim.x - lab) * kUpdWaves;
    const int w = sweeps ? ((int)blockIdx.x - lab) * kUpdWaves +
                               __builtin_amdgcn_readfirstlane(tid >> 6)
                         : 0;
    // unit u = i * nchunks + ch; advancing u by NW advances (i, ch) by (qs, rs)
    const int qs = NW / nchunks, rs = NW % nchunks;
    int i_cur = w / nchunks, ch_cur = w % nchunks;

    // address part of a batch: independent of the pivot, so the first batch's loads are in
    // flight while the selection decision below is still being reduced
    auto fetch = [&](Batch<U>& b) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            b.i[k] = i_cur;
            b.ch[k] = ch_cur;
            ch_cur += rs;
            i_cur += qs;
            if (ch_cur >= nchunks) {
                ch_cur -= nchunks;
                ++i_cur;
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            b.x[k] = dbl2{0.0, 0.0};
            const int j = b.ch[k] * kChunk + 2 * lane;
            if (b.i[k] < R && j < C) b.x[k] = ld2<NTL>(Tin + (int64_t)b.i[k] * ld + j);
        }
    };
    smx_part rec{SMX_NONE, SMX_NONE, 0.0, 3, SMX_NONE, 0.0};
    int negf0 = SMX_NONE;
    if (MODE == kFused && tid < kWave) {   // the decision's loads first (in-order vmcnt)
        if (tid < nparts) rec = parts[(size_t)parity * nparts + tid];
        negf0 = ctl->negf[parity];
    }
    Batch<U> cur;
    if (sweeps) fetch(cur);

    int r, c;
    const double* prow;
    if (MODE == kForced) {
        r = forced_r;
        c = forced_c;
        prow = Tin + (int64_t)r * ld;
    } else if (MODE == kSingle || MODE == kFused) {
        Decision dd;
        int negb_f = SMX_NONE;
        if (MODE == kFused)   // whole block (phase-1 row scan); parts = this step's slot
            dd = decide_fused<kUpdBlock>(rec, negf0, n, m, flen, Tin, ld, &negb_f);
        if (tid < kWave) {
            Decision d;
            if (MODE == kFused)
                d = dd;
            else
                d = decide_from_parts(ctl, parts, nparts, parity, n, m, flen);
            if (tid == 0) {
                s_dec[0] = d.status;
                s_dec[1] = d.r;
                s_dec[2] = d.c;
                if (blockIdx.x == 0) {
                    if (MODE == kFused) ctl->negb[parity] = negb_f;   // host-visible state
                    ctl->sel_status = d.status;
                    ctl->sel_r = d.r;
                    ctl->sel_c = d.c;
                    if (d.status == SMX_PIVOT) {
                        ctl->sel_e = Tin[(int64_t)d.r * ld + d.c];
                        const int64_t k = ctl->npiv[parity];
                        if (log_cap > 0) {
                            log[2 * (k % log_cap)] = d.r;
                            log[2 * (k % log_cap) + 1] = d.c;
                        }
                        ctl->npivots = k + 1;
                        ctl->npiv[parity ^ 1] = k + 1;
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int code = move_label(ctl->xpos[parity][q], d.r, d.c);
                            ctl->xpos[parity ^ 1][q] = code;
                            if (xhist && log_cap > 0 && code < 0)   // non-basic: value 0
                                xhist[2 * (k % log_cap) + q] = 0.0;
                        }
                    } else {
                        ctl->term = 1;
                    }
                }
            }
        }
        __syncthreads();
        if (s_dec[0] != SMX_PIVOT) return;
        r = __builtin_amdgcn_readfirstlane(s_dec[1]);
        c = __builtin_amdgcn_readfirstlane(s_dec[2]);
        prow = Tin + (int64_t)r * ld;
    } else {  // kShard(Fused): every block merges the P gathered headers itself
        __shared__ int64_t s_off;
        if (tid == 0) {
            const int nranks = (MODE == kShardFused) ? forced_c : nparts;
            const ShardDecision d = merge_headers(recv, nranks, ld, m, flen);
            s_dec[0] = d.status;
            s_dec[1] = d.r;
            s_dec[2] = d.c;
            s_off = d.off;
            if (blockIdx.x == 0) publish_shard_decision(d, recv, ctl, log, log_cap, true);
        }
        __syncthreads();
        if (s_dec[0] != SMX_PIVOT) return;
        r = __builtin_amdgcn_readfirstlane(s_dec[1]);
        c = __builtin_amdgcn_readfirstlane(s_dec[2]);
        prow = recv + s_off;
    }
    const double e = prow[c];
    SMX_STAMP(1);
    // history: rows whose new "-b" entry is x1 / x2 of the new tableau (find_optimum)
    int hx0 = -1, hx1 = -1;
    int64_t hslot = 0;
    if ((MODE == kSingle || MODE == kFused) && xhist != nullptr && log_cap > 0) {
        hx0 = move_label(ctl->xpos[parity][0], r, c);
        hx1 = move_label(ctl->xpos[parity][1], r, c);
        hslot = 2 * (ctl->npiv[parity] % log_cap);
    }
    // local index of the pivot row, -1 when another rank owns it (never the f-row replica,
    // whose local index rows_local may equal r - row0 for a row of the next rank)
    const int r_local = (r >= row0 && r < row0 + rows_local) ? r - row0 : -1;
    if (LA && la) {
        // this workgroup's share of step k+1's select inputs (one kernel per pivot)
        la_partial<kUpdBlock, true>(Tin, ld, rows_local, m, fscan, row0, r_local, c, e, prow,
                                    const_cast<smx_part*>(parts) + (size_t)(parity ^ 1) * nparts,
                                    blockIdx.x, nparts, ctl, parity ^ 1);
        if (MODE == kShardFused && send != nullptr) {
            // The last look-ahead workgroup to finish packs step k+1's header and candidate
            // rows into the send slot (values of T_{k+1} via nv), so a sharded pivot is this
            // kernel + the all-gather.  nparts counter atomics, not one per workgroup.
            __shared__ int s_last;
            __syncthreads();
            if (tid == 0) {
                __threadfence();   // release this workgroup's record (and negf from group 0)
                s_last = atomicAdd(&ctl->nla, 1) == nparts - 1;
            }
            __syncthreads();
            if (s_last) {
                __threadfence();   // acquire the other workgroups' records
                pack_ahead(Tin, ld, rows_local, m, row0, r_local, c, e, prow, ctl,
                           parts + (size_t)(parity ^ 1) * nparts, nparts, parity ^ 1, send, 0, 1);
                if (tid == 0) ctl->nla = 0;
            }
        }
        SMX_STAMP(2);
        if (!la_sweep) return;
    }
    int ch_pr = -1;
    dbl2 pr = dbl2{0.0, 0.0};
    const int negslot = parity ^ 1;
    int lb = SMX_NONE;   // fused next-step scan: first row with new b < 0 (this lane)
    int lf = SMX_NONE;   // fused next-step scan: first f-row column with new f < 0 (this lane)

    for (int64_t u = w; u < units; u += (int64_t)U * NW) {
#pragma unroll
        for (int k = 0; k < U; ++k)
            cur.pc[k] = (cur.i[k] < R) ? Tin[(int64_t)cur.i[k] * ld + c] : 0.0;
        Batch<U> nxt;
        if (PIPE && u + (int64_t)U * NW < units) fetch(nxt);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int i = cur.i[k];
            if (i >= R) continue;
            const int j = cur.ch[k] * kChunk + 2 * lane;
            if (cur.ch[k] != ch_pr) {
                ch_pr = cur.ch[k];
                pr = (j < C) ? *reinterpret_cast<const dbl2*>(prow + j) : dbl2{0.0, 0.0};
            }
            dbl2 o;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int jj = j + h;
                const double xv = cur.x[k][h];
                double num;
                if (i == r_local) {
                    num = (jj == c) ? 1.0 : -xv;
                } else {
                    const double a = xv * e;
                    const double b = pr[h] * cur.pc[k];
                    num = (jj == c) ? xv : (a - b);
                }
                if (DIAG)
                    o[h] = num * (1.0 / e);
                else
                    o[h] = num / e;
                if (MODE != kForced && jj < C) {
                    if ((MODE == kSingle || MODE == kFused) && jj == m) {
                        if (i == hx0) xhist[hslot] = o[h];
                        if (i == hx1) xhist[hslot + 1] = o[h];
                    }
                    if (LA) {
                        // next-step scans come from the look-ahead records
                    } else if (i < rows_local) {
                        if (jj == m && o[h] < 0.0) lb = min(lb, row0 + i);
                    } else if (jj < fscan && o[h] < 0.0) {
                        lf = min(lf, jj);
                    }
                }
            }
            if (j < C) {
                double* dst = Tout + (int64_t)i * ld + j;
                if (NTS)
                    __builtin_nontemporal_store(o, reinterpret_cast<dbl2*>(dst));
                else
                    *reinterpret_cast<dbl2*>(dst) = o;
            }
        }
        if (PIPE) {
            cur = nxt;
        } else if (u + (int64_t)U * NW < units) {
            fetch(cur);
        }
    }
    SMX_STAMP(3);
    if (MODE == kSingle || MODE == kShard) {
        lb = wave_min_int(lb);
        lf = wave_min_int(lf);
        if (lane == 0) {
            if (lb != SMX_NONE) atomicMin(&ctl->negb[negslot], lb);
            if (lf != SMX_NONE) atomicMin(&ctl->negf[negslot], lf);
        }
    }
}

}  // namespace
