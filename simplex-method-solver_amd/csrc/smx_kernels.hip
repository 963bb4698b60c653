// smx_kernels.hip -- CDNA4 (gfx950) kernels of the simplex pivot engine + the C ABI of smx.h.
//
// Hot path of jqnfxa/Simplex-Method-Solver src/simplex.py, re-designed for MI355X.  One
// translation unit; the device code is split by role into the headers included below:
//   smx_common.hpp    ratio-test order, wave reductions, decisions from partials / shard headers
//   smx_select.hpp    k_reset, k_select, k_finalize (pick_element, simplex.py:70-141)
//   smx_lookahead.hpp the fused chain's look-ahead (next step's selection inputs from T_k)
//   smx_update.hpp    k_update: recalculate_matrix (simplex.py:143-177), every mode
//   smx_shard.hpp     row-sharded exchange kernels
//   smx_batch.hpp     k_copy (copy-ceiling probe), k_batch (one small LP per wavefront)
//   smx_resident.hpp  k_resident: the whole pivot loop in one persistent launch, tableau in LDS
//   smx_block.hpp     k_blk_*: P pivots per HBM sweep, decisions planned from the sweep's input
// and this file holds the host side: grid sizing, variants, chains, graphs, RCCL, the C ABI.
//
// Arithmetic parity: every element is (t*e - pr*pc)/e with each op rounded on its own, exactly
// as CPython evaluates simplex.py:173-175.  This file is compiled with -ffp-contract=off and
// additionally pins `#pragma clang fp contract(off)`; fp64 division is the IEEE-correct
// div_scale/rcp/fma/div_fmas/div_fixup sequence (never a reciprocal multiply).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <mutex>
#include <thread>
#include <vector>
#include <type_traits>
#include <utility>
#include <string.h>

#include <rccl/rccl.h>

#include "smx.h"

#pragma clang fp contract(off)

static_assert(sizeof(smx_ctl) == 128, "smx_ctl layout");
static_assert(offsetof(smx_ctl, term) == 16 && offsetof(smx_ctl, npivots) == 40 &&
                  offsetof(smx_ctl, shard_off) == 56 && offsetof(smx_ctl, xpos) == 64 &&
                  offsetof(smx_ctl, npiv) == 80 && offsetof(smx_ctl, dec) == 96,
              "smx_ctl offsets (mirrored in simplex_mi355x/_lib.py)");
static_assert(sizeof(smx_part) == 32, "smx_part layout");


// Device code, in dependency order (each part reopens the anonymous namespace).
#include "smx_common.hpp"
#include "smx_select.hpp"
#include "smx_lookahead.hpp"
#include "smx_update.hpp"
#include "smx_shard.hpp"
#include "smx_batch.hpp"
#include "smx_resident.hpp"
#include "smx_block.hpp"
#include "smx_window.hpp"
#include "smx_wplan.hpp"
#include "smx_host.hpp"
#include "smx_intfirst.hpp"

namespace {

// ---------------------------------------------------------------------------------------------
inline int nparts_for(int rows, int m) {
    // SMX_NPARTS_MAX (experiments): a lower cap on the select / planner workgroup count
    static const int cap_env = [] {
        const char* e = getenv("SMX_NPARTS_MAX");
        return e ? atoi(e) : 0;
    }();
    const int work = rows > m ? rows : m;
    int p = (work + kSelBlock - 1) / kSelBlock;
    if (p < 1) p = 1;
    if (p > kMaxParts) p = kMaxParts;
    if (cap_env > 0 && p > cap_env) p = cap_env;
    return p;
}

inline int fscan_of(const smx_shape& s) { return s.flen < s.m ? s.flen : s.m; }

inline bool shape_ok(const smx_shape* s) {
    if (!s) return false;
    if (s->m < 0 || s->rows < 0 || s->n < s->rows || s->ld < s->m + 1) return false;
    if ((s->ld & 1) != 0) return false;                   // 16-B aligned double2 rows
    if (((s->m + 1) & 1) && s->ld < s->m + 2) return false;  // odd C: vector tail in padding
    if ((s->m + 1) > 2 && (s->ld & 3) != 0) return false;    // VEC = 4 variants: 32-B lanes
    if (s->nparts < 1 || s->nparts > kMaxParts) return false;
    return true;
}

inline hipStream_t S(void* p) { return reinterpret_cast<hipStream_t>(p); }

int launch_select(const double* T, const smx_shape& s, int parity, smx_ctl* ctl, smx_part* parts,
                  hipStream_t st) {
    hipLaunchKernelGGL(k_select, dim3(s.nparts), dim3(kSelBlock), 0, st, T, s.ld, s.rows, s.m,
                       s.row0, parity, ctl, parts);
    return (int)hipGetLastError();
}

template <bool FUSED>
int launch_pack(const double* T, const smx_shape& s, int parity, const smx_ctl* ctl,
                const smx_part* parts, double* send, hipStream_t st) {
    int blocks = (int)((s.m + 2 + kUpdBlock - 1) / kUpdBlock);
    if (blocks > 64) blocks = 64;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_pack<FUSED>, dim3(blocks), dim3(kUpdBlock), 0, st, T, s.ld, s.rows, s.m,
                       s.row0, parity, ctl, parts, s.nparts, send);
    return (int)hipGetLastError();
}

// Fused chain helpers: prime the look-ahead records of step `parity` from T; publish at the end.
int launch_prime(const double* T, const smx_shape& s, int parity, smx_ctl* ctl, smx_part* parts,
                 hipStream_t st) {
    const int fscan = s.flen < s.m ? s.flen : s.m;
    hipLaunchKernelGGL(k_la_prime, dim3(s.nparts), dim3(kUpdBlock), 0, st, T, s.ld, s.rows, s.m,
                       fscan, s.row0, parity, ctl, parts + (size_t)parity * s.nparts);
    return (int)hipGetLastError();
}

int launch_publish(const smx_shape& s, int parity, smx_ctl* ctl, const smx_part* parts,
                   hipStream_t st) {
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(kWave), 0, st, parts + (size_t)parity * s.nparts,
                       s.nparts, parity, ctl);
    return (int)hipGetLastError();
}

// ---- update-kernel variants (rows per unit TR, doubles per lane VEC, non-temporal stores) -----
struct UpdVariant {
    int u, nts, ntl, pipe;
};
constexpr UpdVariant kVariants[] = {{2, 1, 0, 0}, {2, 1, 1, 0}, {2, 1, 0, 1}, {2, 1, 1, 1},
                                    {1, 1, 0, 1}, {1, 1, 1, 1}, {4, 1, 0, 0}, {4, 1, 0, 1},
                                    {2, 0, 0, 0}, {1, 1, 0, 0},
                                    // diagnostics (reciprocal multiply: timing only)
                                    {2, 1, 1, 0}, {1, 1, 1, 1}};
constexpr int kFirstDiagVariant = 10;
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
// Defaults from tools/tune_update.py on MI355X at 16384^2 (profiles/r01_tune_sweep*.jsonl).
// Variant -1 = automatic: U=2 with non-temporal stores and loads (1) for tableaux that stream
// from HBM; plain loads (0) when one buffer is at most kCacheTable bytes, where the ping-pong
// pair stays in the 256 MB Infinity Cache and a non-temporal load only adds latency
// (profiles/r01_sweep_small.jsonl: 1024^2 11.1 vs 13.1 us per fused pivot; from 2048^2 on the
// non-temporal variant is as fast or faster).
int g_variant = -1;       // smx_tune_set overrides
constexpr int kLargeVariant = 1, kSmallVariant = 0;
constexpr int64_t kCacheTable = 16ll << 20;
constexpr int64_t kLaSweepTable = 256ll << 20;
// Sharded fused update: its last look-ahead workgroup can pack the next step itself (pivot =
// update + all-gather).  Off by default: measured at world size 1 (tools/fold_ab.py,
// profiles/r01_fold_ab.jsonl) it adds ~40 us per pivot at the 4- and 8-GPU per-rank shapes
// (4097 / 2049 x 16384: that workgroup's share of the sweep starts late and per-wave throughput
// is latency-bound) and gains nothing at 16384^2; the separate k_pack<true> wins everywhere.
int64_t g_fold_min_bytes = INT64_MAX;   // smx_tune_fold
inline bool folds_pack(const smx_shape& s) {
    return (int64_t)(s.rows + 1) * s.ld * 8 >= g_fold_min_bytes;
}
int g_blocks_per_cu = 0;  // 0: kDefaultBpc, capped by the occupancy API (see blocks_per_cu)
constexpr int kDefaultBpc = 5;

using UpdFn = void (*)(const double*, double*, int64_t, int, int, int, int, int, int, int,
                       smx_ctl*, const smx_part*, int, int32_t*, double*, int64_t, const double*,
                       int, int, double*);

template <int MODE>
UpdFn upd_fn(int v) {
    switch (v) {
        case 0: return k_update<MODE, 2, true, false, false>;
        case 1: return k_update<MODE, 2, true, true, false>;
        case 2: return k_update<MODE, 2, true, false, true>;
        case 3: return k_update<MODE, 2, true, true, true>;
        case 4: return k_update<MODE, 1, true, false, true>;
        case 5: return k_update<MODE, 1, true, true, true>;
        case 6: return k_update<MODE, 4, true, false, false>;
        case 7: return k_update<MODE, 4, true, false, true>;
        case 8: return k_update<MODE, 2, false, false, false>;
        case 9: return k_update<MODE, 1, true, false, false>;
        case 10: return k_update<MODE, 2, true, true, false, true>;
        default: return k_update<MODE, 1, true, true, true, true>;
    }
}

int variant_for(const smx_shape& s) {
    if (g_variant >= 0) return g_variant;
    return (int64_t)(s.rows + 1) * s.ld * 8 <= kCacheTable ? kSmallVariant : kLargeVariant;
}

// Resident blocks per CU for a kernel, cached.  The grid is exactly CUs x this, so every block
// is resident at once and the balanced unit ranges finish together (no second residency round).
// The host-side caches below are shared by smx_mshard_run's per-device threads: one mutex.
std::mutex g_cache_mu;
// smx_mshard_run (RCCL exchange): the first failing rank's own error code and index, kept for
// smx_mshard_last_error (the call itself returns SMX_ERR_COMMS_ABORTED after aborting every
// communicator); guarded by g_cache_mu
int g_mshard_err = 0, g_mshard_err_rank = -1;

// Resident 256-thread blocks per CU of `fn` by the occupancy API (registers and LDS), one block
// of margin below its answer, cached; at most `cap`.
int resident_bpc(const void* fn, int cap);

int blocks_per_cu(const void* fn) {
    if (g_blocks_per_cu > 0) return g_blocks_per_cu;
    return resident_bpc(fn, kDefaultBpc);
}

int resident_bpc(const void* fn, int cap) {
    struct Entry {
        const void* fn;
        int dev;
        int bpc;
    };
    static Entry cache[128];
    static int ncache = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(g_cache_mu);
    for (int i = 0; i < ncache; ++i)
        if (cache[i].fn == fn && cache[i].dev == dev) return cache[i].bpc < cap ? cache[i].bpc : cap;
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, fn, kUpdBlock, 0) != hipSuccess ||
        bpc < 1)
        bpc = 4;
    // ROCm 7.2 over-reports by one block/CU for 256-thread kernels above 80 SGPRs
    // (MI355X_MICROARCH.md, residency): keep one block of margin below the API's answer.
    if (bpc > 1) bpc -= 1;
    if (ncache < 128) cache[ncache++] = Entry{fn, dev, bpc};
    return bpc < cap ? bpc : cap;
}

// CUs of the current device
int num_cus() {
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    std::lock_guard<std::mutex> lock(g_cache_mu);
    if (!cus[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v < 1)
            v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}

// Grid = resident blocks, trimmed so the wave count is a multiple of the chunks per row (then
// every wave keeps one pivot-row slice for the whole sweep).
int update_grid(const smx_shape& s, const void* fn, int reserved, int bpc = 0) {
    const int64_t R = s.rows + 1;
    const int64_t nchunks = (s.m + 1 + 2 * kWave - 1) / (2 * kWave);
    const int64_t units = nchunks * R;
    if (bpc <= 0 || g_blocks_per_cu > 0) bpc = blocks_per_cu(fn);
    int64_t blocks = (int64_t)num_cus() * bpc - reserved;
    if (blocks < 1) blocks = 1;
    // waves = a multiple of lcm(nchunks, waves per block) when that keeps >= 3/4 of them
    int64_t g = nchunks, h = kUpdWaves;
    while (h) {
        const int64_t t = g % h;
        g = h;
        h = t;
    }
    const int64_t lcm = nchunks / g * kUpdWaves;
    const int64_t waves = blocks * kUpdWaves;
    if (waves >= lcm && (waves - waves % lcm) * 4 >= waves * 3) blocks = (waves - waves % lcm) / kUpdWaves;
    const int64_t need = (units + kUpdWaves - 1) / kUpdWaves;
    if (blocks > need) blocks = need;
    if (blocks < 1) blocks = 1;
    return (int)blocks + reserved;
}

template <int MODE>
int launch_update_mode(const double* Tin, double* Tout, const smx_shape& s, int parity,
                       smx_ctl* ctl, const smx_part* parts, int32_t* log, double* xhist,
                       int64_t log_cap, const double* recv, int fr, int fc, hipStream_t st,
                       int reserve = 0, double* send = nullptr) {
    const int v = variant_for(s);
    UpdFn fn = upd_fn<MODE>(v);
    // kFused: the first nparts workgroups compute the look-ahead records; within the Infinity
    // Cache they are reserved (their extra round trips would be the critical path), beyond it
    // they sweep too (profiles/r01_sweep_small.jsonl)
    constexpr bool LA = MODE == kFused || MODE == kShardFused;
    const bool la_sweep = LA && (int64_t)(s.rows + 1) * s.ld * 8 > kLaSweepTable;
    // reserve: resident slots left free for kernels of another stream (overlapped shard chain)
    int grid = update_grid(s, (const void*)fn, (LA && !la_sweep ? s.nparts : 0) + reserve) -
               reserve;
    if (grid < s.nparts) grid = s.nparts;
    if (grid < 1) grid = 1;
    if (LA) fr = la_sweep ? 1 : 0;   // kShardFused: fc = rank count (caller)
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kUpdBlock), 0, st, Tin,
                       Tout, s.ld, s.rows, s.n, s.m, s.flen, fscan_of(s), s.row0, parity, ctl,
                       parts, s.nparts, log, xhist, log_cap, recv, fr, fc, send);
    return (int)hipGetLastError();
}

int launch_update(const double* Tin, double* Tout, const smx_shape& s, int parity, smx_ctl* ctl,
                  const smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
                  hipStream_t st) {
    return launch_update_mode<kSingle>(Tin, Tout, s, parity, ctl, parts, log, xhist, log_cap,
                                       nullptr, 0, 0, st);
}

// Chains (smx_tune_fused): 0 select + update; 1 one fused kernel per pivot (default); 2 as 1, and
// the sharded chain overlaps the next step's look-ahead + all-gather with the sweep on a second
// stream -- correct, but slower on this stack: the two cross-stream waits per step cost more than
// the all-gather they hide (profiles/r01_shard_overlap_trace.txt).
int g_fused = 1;

int launch_chain(double* buf0, double* buf1, const smx_shape& s, int parity, int k, smx_ctl* ctl,
                 smx_part* parts, int32_t* log, double* xhist, int64_t log_cap, hipStream_t st) {
    if (g_fused && k > 0) {
        // prime the records of the first step, one fused kernel per pivot, publish the next
        int err = launch_prime(parity ? buf1 : buf0, s, parity, ctl, parts, st);
        if (err) return err;
        for (int step = 0; step < k; ++step) {
            const int p = (parity + step) & 1;
            err = launch_update_mode<kFused>(p ? buf1 : buf0, p ? buf0 : buf1, s, p, ctl, parts,
                                             log, xhist, log_cap, nullptr, 0, 0, st);
            if (err) return err;
        }
        return launch_publish(s, (parity + k) & 1, ctl, parts, st);
    }
    for (int step = 0; step < k; ++step) {
        const int p = (parity + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        int err = launch_select(tin, s, p, ctl, parts, st);
        if (err) return err;
        err = launch_update(tin, tout, s, p, ctl, parts, log, xhist, log_cap, st);
        if (err) return err;
    }
    return 0;
}

// ---- on-chip resident pivot loop (smx_resident.hpp) ------------------------------------------
// -1: never; 0: automatic (one workgroup per CU, at most one per row); > 0: that many workgroups
int g_resident = 0;
uint64_t* g_resident_trace = nullptr;    // diagnostic stamps (smx_resident_trace)
int g_resident_trace_from = 0;
constexpr int64_t kResLdsMax = 160 * 1024 - 5 * 1024;   // dynamic LDS (static part ~4.2 KiB)
constexpr int64_t kResLdsMin = 82 * 1024;               // > half a CU's LDS: one group per CU

struct ResPlan {
    int G, rpw, ept;
    int64_t lds, rec_bytes, row_off, pc_off, bytes;
};
// The overlapped loop (k_resident<true>: the bulk update hidden under the next hand-off's poll)
// or the round-3 loop (smx_tune_resident_overlap): 2 automatic -- overlapped from 768 columns
// (tools/resident_bench.py, profiles/r04k/: 1024^2 8.8-9.0 vs 9.6-9.7 us per pivot over seeds
// 0..4, 1536^2 10.4 vs 13.4; 512^2 7.5 vs 7.3, where the update it hides is short); 1 / 0 forced.
int g_resident_ovl = 2;
constexpr int kResOvlMinCols = 768;

bool resident_plan(const smx_shape& s, ResPlan* p) {
    if (g_resident < 0) return false;
    if (s.row0 != 0 || s.rows != s.n || s.n < 1 || s.m < 1 || s.n > kResMaxRows) return false;
    if (s.m + 1 > 4096) return false;   // 13-bit phase-1 column in the record
    const int C = s.m + 1;
    // automatic: about four rows per workgroup (tools/resident_bench.py: 256^2 64 groups, 512^2
    // 128, 1024^2 256), six where the overlapped loop runs (its update hides under the poll, so
    // fewer records to poll pay: 1024^2 8.72 / 8.73 / 8.26 / 8.55 us per pivot at 4 / 8 / 6 / 5
    // rows per workgroup, profiles/r05d/), more when the rows do not fit in LDS, at most one
    // workgroup per CU
    const int64_t ldl = C | 1;
    auto lds_of = [&](int r) { return ((int64_t)(r + 1) * ldl + C + (r + 1)) * 8; };
    const int gmax = g_resident > 0 ? g_resident : (num_cus() < kResPollers ? num_cus() : kResPollers);
    const bool ovl = g_resident_ovl == 1 || (g_resident_ovl == 2 && C >= kResOvlMinCols);
    const int per = ovl ? 6 : 4;
    int G = g_resident > 0 ? g_resident : (s.n + per - 1) / per;
    if (G > gmax) G = gmax;
    if (G > s.n) G = s.n;
    int rpw = (s.n + G - 1) / G;
    while (lds_of(rpw) > kResLdsMax && g_resident <= 0 && rpw > 1 && (s.n + rpw - 2) / (rpw - 1) <= gmax)
        --rpw;
    G = (s.n + rpw - 1) / rpw;              // no workgroup without rows
    const int64_t lds = lds_of(rpw);
    if (lds > kResLdsMax || G > kResPollers) return false;
    p->G = G;
    p->rpw = rpw;
    p->ept = (int)(((int64_t)(rpw + 1) * C + kResBlock - 1) / kResBlock);
    p->lds = lds < kResLdsMin ? kResLdsMin : lds;
    p->rec_bytes = (int64_t)2 * G * kResRecWords * 8;
    p->row_off = (p->rec_bytes + 255) / 256 * 256;
    p->pc_off = p->row_off + (int64_t)2 * G * 2 * (2 * s.ld) * 8;  // rows as tagged granules
    p->bytes = p->pc_off + (int64_t)2 * G * 2 * 2 * 8;              // their pivot-column entries
    return true;
}

int launch_resident_kernel(double* buf0, double* buf1, const smx_shape& s, const ResPlan& p,
                           int parity, int k, smx_ctl* ctl, char* xch, uint32_t epoch,
                           int32_t* log, double* xhist, int64_t log_cap, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        for (const void* f : {(const void*)k_resident<true>, (const void*)k_resident<false>}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)kResLdsMax);
            if (e != hipSuccess) return (int)e;
        }
        attr = true;
    }
    const bool ovl = g_resident_ovl == 1 || (g_resident_ovl == 2 && s.m + 1 >= kResOvlMinCols);
    hipLaunchKernelGGL(ovl ? k_resident<true> : k_resident<false>, dim3(p.G),
                       dim3(kResBlock), (size_t)p.lds, st, buf0, buf1,
                       s.ld, s.n, s.m, s.flen, fscan_of(s), parity, k, p.rpw, ctl, log, xhist,
                       log_cap, reinterpret_cast<uint64_t*>(xch),
                       reinterpret_cast<uint64_t*>(xch + p.row_off), s.ld, epoch,
                       g_resident_trace, g_resident_trace_from,
                       reinterpret_cast<uint64_t*>(xch + p.pc_off));
    return (int)hipGetLastError();
}

// k_resident's workgroups wait for each other, so two of its launches must never share the
// device: with each solver on its own stream, two concurrent chains could split the CUs between
// them and every hand-off would wait for workgroups that cannot be scheduled (until the 2 s
// timeout).  Every resident launch therefore waits for the previous one on the same device,
// whatever stream it came from (an event chain per device; other kernels always finish, so they
// only delay a resident launch).
int resident_serialize(hipStream_t st, bool after) {
    static std::mutex mu;
    static hipEvent_t last[64] = {};
    int dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess) (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lock(mu);
    if (!last[dev]) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        hipError_t e = hipSetDevice(dev);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&last[dev], hipEventDisableTiming);
        (void)hipSetDevice(cur);
        if (e != hipSuccess) return (int)e;
        if (!after) return 0;   // no resident launch yet on this device
    }
    return (int)(after ? hipEventRecord(last[dev], st) : hipStreamWaitEvent(st, last[dev], 0));
}

int launch_resident(double* buf0, double* buf1, const smx_shape& s, int parity, int k,
                    smx_ctl* ctl, void* xch, int64_t xch_bytes, uint32_t epoch, int32_t* log,
                    double* xhist, int64_t log_cap, hipStream_t st) {
    ResPlan p;
    if (!resident_plan(s, &p) || xch == nullptr || xch_bytes < p.bytes || epoch < 1 ||
        epoch > 4095 || k >= (1 << 20) - 1)
        return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(&ctl->dec[0][0], 0, sizeof(int32_t), st);   // no latched timeout
    if (e != hipSuccess) return (int)e;
    int err = resident_serialize(st, false);
    if (!err)
        err = launch_resident_kernel(buf0, buf1, s, p, parity, k, ctl, static_cast<char*>(xch),
                                     epoch, log, xhist, log_cap, st);
    if (!err) err = resident_serialize(st, true);
    return err;
}

// ---- block pivots (smx_block.hpp) ------------------------------------------------------------
// smx_tune_block: 0 automatic, 1 never, 2..kBlkMax that many pivots per sweep (at most: a chain
// of k pivots is cut into ceil(k / P) blocks of near-equal size, block_size)
// Automatic policy from tools/block_bench.py (profiles/r01_block_sweep.jsonl,
// profiles/r02g_block_pivots.jsonl): below ~48 MiB the planner's ~15 us per pivot eats the saved
// traffic (2048^2: block 4 = fused within 1 %); 6 pivots per sweep up to 256 MiB (3072^2: 45.8 k
// pivots/s vs 30.1 k fused), 12 beyond (round 2, 16384^2: 125.8 us at 12, 129.5 at 10, 128.0 at
// 14, 139.3 at 8; the sweep is VALU-bound past ~10 pivots).  Round 3, with the cheaper planner
// (profiles/r03b/block_pivots_vs_P.jsonl, k = 96): 8192^2 37.8 / 34.2 / 32.0 / 33.6 / 36.1 us per
// pivot at 8 / 10 / 12 / 14 / 16 (it was 10 up to 1 GiB), 16384^2 109.7 / 101.4 / 98.6 / 104.0 /
// 100.0 / 109.0 at 10 / 12 / 13 / 14 / 15 / 16; 48-256 MiB now 10 (it was 6;
// profiles/r03d/block_pivots_mid_sizes.jsonl: 3072^2 17.0 / 15.7 / 15.8 us per pivot at 6 / 8 /
// 10, 4096^2 20.4 / 18.3 / 18.0).
int g_block = 0;
constexpr int64_t kBlockMinTable = 48ll << 20;
constexpr int64_t kBlockWideTable = 256ll << 20;

// Round 4: tables of 1-4 GiB take up to 20 pivots per sweep (the LDS layout past 12,
// k_blk_sweep<P, 5>): at 16384^2 the per-pivot cost is flat from 12 to 20 (99.4 / 101.5 / 99.1 us
// at 12 / 16 / 20, profiles/r04r/; 100.8 / 98.4 / 97.8 on another box, profiles/r04e/), so the
// larger bound only changes how a chain is cut -- 20 pivots become ONE sweep of 20 instead of two
// of 10 (106.8 us per pivot at 10); at 200 pivots 12 and 20 tie (10,426 / 10,455 pivots/s,
// profiles/r05b/).  Round 5: also beyond 4 GiB -- config 5 (65536 x 32768 degenerate, 17 GB)
// sweeps at 803 / 773 / 743 / 744 us per pivot with 12 / 16 / 20 / 24 pivots per sweep, planner
// 26 / 30 us per pivot at 12 / 20 (profiles/r05b/).  Below 1 GiB (8192^2: 32.0 / 33.6 / 36.1 us
// at 12 / 14 / 16, where the planner's share is larger) it stays at 12.
// Round 6, the persistent window planner (smx_wplan.hpp, ~8 us per pivot wherever it runs):
// kBlkMax = 24 pivots per sweep is the fastest at every size measured (tools/block_bench.py,
// profiles/r06s/, us per pivot at 8 / 12 / 16 / 20 / 24: 3072^2 13.3 / 12.5 / 12.0 / 11.8 / 11.7,
// 4096^2 16.3 / 14.9 / 14.2 / 14.0 / 13.8, 6144^2 24.9 / 20.9 / 19.6 / 20.4 / 19.3; 8192^2 and
// 16384^2 at 16 / 20 / 24 30.5 / 29.4 / 28.7 and 91.7 / 88.7 / 87.0, profiles/r06r/), so
// tables it plans take 24; the others keep the launch-form policy above.
constexpr int64_t kBlockHugeTable = 1ll << 30;
bool wplan_shape(const smx_shape& s);

int block_pivots(const smx_shape& s) {
    if (g_block == 1) return 0;
    if (s.row0 != 0 || s.rows != s.n || s.rows < 1 || s.m < 1) return 0;   // unsharded only
    if (g_block >= 2) return g_block;
    const int64_t bytes = (int64_t)(s.rows + 1) * s.ld * 8;
    if (bytes < kBlockMinTable) return 0;
    if (wplan_shape(s)) return kBlkMax;
    if (bytes >= kBlockHugeTable) return 20;
    return bytes >= kBlockWideTable ? 12 : 10;
}

// Pivots of block b when k pivots are cut into ceil(k / P) blocks of near-equal size (the larger
// ones first): two sweeps of 10 cost less than sweeps of 12 and 8 (1.07 + 1.07 vs 1.28 + 0.96 ms
// at 16384^2), and a short chain never ends in a mostly idle sweep.
int block_size(int k, int P, int b) {
    const int nb = (k + P - 1) / P;
    const int base = k / nb, extra = k % nb;
    return base + (b < extra ? 1 : 0);
}

using BlkSweepFn = void (*)(double*, double*, int64_t, int, int, const BlkHdr*, const double*,
                           const double*, BlkHdr*, int, int);
using BlkStepFn = void (*)(const double*, int64_t, int, int, int, int, int, int, int, int,
                           smx_ctl*, BlkHdr*, smx_part*, double*, double*, double*,
                           const double*, int, int32_t*, double*, int64_t, const double*,
                           int64_t);
using BshPackFn = void (*)(const double*, int64_t, int, int, int, int, int, const smx_ctl*,
                           const BlkHdr*, const smx_part*, int, const double*, const double*,
                           double*);

// Sweep kernels by pivot count (1..kBlkMax) and layout (FORM 4 / 5, blk_sweep_body_flag)
template <int FORM, int... Is>
BlkSweepFn blk_sweep_pick(int P, std::integer_sequence<int, Is...>) {
    static const BlkSweepFn t[] = {k_blk_sweep<Is + 1, FORM>...};
    return t[P - 1];
}
BlkSweepFn blk_sweep_fn(int P, int form) {
    using All = std::make_integer_sequence<int, kBlkMax>;
    return form == 6 ? blk_sweep_pick<6>(P, All{})
                     : form == 5 ? blk_sweep_pick<5>(P, All{}) : blk_sweep_pick<4>(P, All{});
}

template <bool SH, int... Is>
BlkStepFn blk_step_pick(int L, std::integer_sequence<int, Is...>) {
    static const BlkStepFn t[] = {k_blk_step<Is + 1, SH>...};
    return t[L - 1];
}
template <bool SH>
BlkStepFn blk_step_fn_sh(int L) {
    return blk_step_pick<SH>(L, std::make_integer_sequence<int, kBlkMax>{});
}

template <int... Is>
BshPackFn bsh_pack_pick(int D, std::integer_sequence<int, Is...>) {
    static const BshPackFn t[] = {k_bsh_pack<Is>...};
    return t[D];
}
BshPackFn bsh_pack_fn(int D) { return bsh_pack_pick(D, std::make_integer_sequence<int, kBlkMax>{}); }

// Scratch pointers of a block chain (plan slots 0 / 1; h[0] also holds the chain state)
struct BlkPtrs {
    BlkLayout L;
    BlkHdr* h[2];
    smx_part* parts;
    double *mul[2], *pr[2], *fr, *win;
    uint64_t* xg;   // the persistent window planner's granules (k_blk_start zeroes them)
};
// smx_tune_block_planner: 0 (default) the window planner on unsharded chains -- one persistent
// launch per block (k_blk_wplan, smx_wplan.hpp) where its workgroups fit one per CU and its rows
// fit in registers, else one launch per pivot (k_blk_wstep, smx_window.hpp); 2 the window
// planner's launch form always; 1 the register-form chains (k_blk_step<L, false>).  Row-sharded
// chains always run the register form (k_blk_step<L, true>).  g_block_nwin: window slots (2..kWin; tests shrink
// it to drive the window's fallbacks).
int g_block_planner = 0;
int g_block_nwin = kWin;
// (sh: a row-sharded chain -- at world size 1 its shape is the whole table, so the shape alone
// cannot tell)
bool use_window(const smx_shape& s, bool sh) {
    return !sh && g_block_planner != 1 && s.row0 == 0 && s.rows == s.n;
}
bool use_wplan(const smx_shape& s, bool sh) {
    return use_window(s, sh) && g_block_planner == 0 && win_rpw(s.rows) <= kWpMaxRpw &&
           win_groups(s.rows) <= num_cus();
}
bool wplan_shape(const smx_shape& s) { return use_wplan(s, false); }

// Planner workgroups of a chain (every launch of one chain uses the same count, since a step
// merges the records of the step before it by that count)
int blk_G(const smx_shape& s, bool sh) {
    return use_window(s, sh) ? win_groups(s.rows) : blk_parts_of(s.nparts, s.rows);
}

BlkPtrs blk_ptrs(const smx_shape& s, char* blk) {
    BlkPtrs b;
    b.L = blk_layout(s.rows + 1, s.ld, blk_parts_of(s.nparts, s.rows));
    for (int k = 0; k < 2; ++k) {
        b.h[k] = reinterpret_cast<BlkHdr*>(blk + kBlkHdrBytes * k);
        b.mul[k] = reinterpret_cast<double*>(blk + b.L.mul + k * b.L.mul_slot);
        b.pr[k] = reinterpret_cast<double*>(blk + b.L.pr + k * b.L.pr_slot);
    }
    b.parts = reinterpret_cast<smx_part*>(blk + b.L.parts);
    b.fr = reinterpret_cast<double*>(blk + b.L.fr);
    b.win = reinterpret_cast<double*>(blk + b.L.win);
    b.xg = reinterpret_cast<uint64_t*>(blk + b.L.xg);
    return b;
}

// loc: buffer index (0/1) of T
int launch_blk_prime(bool sh, const double* T, const smx_shape& s, int parity, int loc, smx_ctl* ctl,
                     const BlkPtrs& b, hipStream_t st) {
    hipLaunchKernelGGL(k_blk_start, dim3(blk_G(s, sh)), dim3(kBlkNT), 0, st, T, s.ld, s.rows, s.m,
                       fscan_of(s), parity, loc, s.row0, (const smx_ctl*)ctl, b.h[0], b.h[1],
                       b.fr, b.parts, use_wplan(s, sh) ? b.xg : nullptr);
    return (int)hipGetLastError();
}

// One planner launch of block bn (the register-form planner k_blk_step<L, SH>).
int launch_blk_step(bool sh, int L, const double* T, const smx_shape& s, int P, int parity,
                    int bn, smx_ctl* ctl, const BlkPtrs& b, const double* recv, int nranks,
                    int32_t* log, double* xhist, int64_t log_cap, hipStream_t st,
                    const double* xrow = nullptr, int64_t xslot = 0) {
    BlkStepFn fn = sh ? blk_step_fn_sh<true>(L) : blk_step_fn_sh<false>(L);
    hipLaunchKernelGGL(fn, dim3(blk_G(s, sh)), dim3(kBlkNT), 0, st, T, s.ld, s.rows, s.m, s.flen,
                       fscan_of(s), s.row0, P, parity, bn, ctl, b.h[0], b.parts, b.mul[0],
                       b.pr[0], b.fr, recv, nranks, log, xhist, log_cap, xrow, xslot);
    return (int)hipGetLastError();
}

// One window-planner launch (block bn, step L) and, after a block's last step, the pivot rows
// One persistent window-planner launch: block bn's Pb steps (done: pivots of the chain before it)
int launch_blk_wplan(const double* T, const smx_shape& s, int P, int parity, int bn, int done,
                     smx_ctl* ctl, const BlkPtrs& b, int32_t* log, double* xhist,
                     int64_t log_cap, hipStream_t st) {
    hipLaunchKernelGGL(k_blk_wplan, dim3(win_groups(s.rows)), dim3(kWinNT), 0, st, T, s.ld,
                       s.rows, s.m, s.flen, fscan_of(s), P, parity, bn, done, g_block_nwin,
                       win_rpw(s.rows), ctl, b.h[0], b.parts, b.mul[0], b.pr[0], b.xg, log,
                       xhist, log_cap);
    return (int)hipGetLastError();
}

// fromT: the chain's first step (the window is read from the table itself)
int launch_blk_wstep(int L, const double* T, const smx_shape& s, int P, int parity, int bn,
                     smx_ctl* ctl, const BlkPtrs& b, int32_t* log, double* xhist, int64_t log_cap,
                     hipStream_t st, int fromT) {
    hipLaunchKernelGGL(k_blk_wstep, dim3(win_groups(s.rows)), dim3(kWinNT), 0, st, T, s.ld,
                       s.rows, s.m, s.flen, fscan_of(s), P, L, parity, bn, g_block_nwin,
                       win_rpw(s.rows), fromT, ctl, b.h[0], b.parts, b.mul[0], b.win, log, xhist,
                       log_cap);
    return (int)hipGetLastError();
}
int launch_blk_prows(const double* T, const smx_shape& s, int P, const BlkPtrs& b,
                     hipStream_t st) {
    // one column per quad of lanes (16384 columns: 1,024 waves), one row per thread for the flags
    const int64_t work = std::max<int64_t>((int64_t)(s.m + 1) * 4, s.rows + 1);
    const int grid = (int)std::min<int64_t>((work + kProwsNT - 1) / kProwsNT, num_cus() * 8);
    hipLaunchKernelGGL(k_blk_prows, dim3(grid), dim3(kProwsNT), 0, st, T, s.ld, s.rows, s.m, P,
                       (const BlkHdr*)b.h[0], b.mul[0], b.pr[0]);
    return (int)hipGetLastError();
}

// Row-sharded exchange: SMX_XCHG_FULL all-gathers every rank's send slot (header + rows A, B;
// SMX_SHARD_HDR + 2 * ld doubles per rank); SMX_XCHG_LIGHT all-gathers the headers only, then
// k_bsh_pick + ONE max all-reduce of one row (ld doubles) hands the pivot row to every rank.
// Automatic: light from 4 ranks on (each rank receives 64 B per rank plus ~2 rows per pivot
// instead of 2 rows per rank: 2.1 MB -> 0.23 MB at 8 ranks of C = 16384, for a second
// collective's latency), full below.
int g_shard_xchg = -1;
bool xchg_light(int nranks) { return g_shard_xchg < 0 ? nranks >= 4 : g_shard_xchg == 1; }

int launch_bsh_pick(const double* hdrs, const smx_shape& s, int nranks, int rank,
                    const double* send, double* row, hipStream_t st) {
    const int grid = (int)((s.ld + kUpdBlock - 1) / kUpdBlock);
    hipLaunchKernelGGL(k_bsh_pick, dim3(grid < 1 ? 1 : grid), dim3(kUpdBlock), 0, st, hdrs,
                       nranks, s.ld, s.m, s.flen, rank, send, row);
    return (int)hipGetLastError();
}

// The pack's grid: the records are merged by count (blk_parts_of, the step kernels' partition),
// while the grid only slices the candidate rows' columns -- one column per thread (a rank of
// 2,049 rows had ~9 workgroups, so every thread carried ~8 columns' chains of up to P - 1 steps
// one after the other: most of the sharded per-pivot floor)
int launch_bsh_pack(int D, const double* T, const smx_shape& s, int P, int bn,
                    const smx_ctl* ctl, const BlkPtrs& b, double* send, hipStream_t st) {
    const int gc = (int)std::min<int64_t>((s.m + 1 + kBlkNT - 1) / kBlkNT, kBlkPartsMax);
    const int grid = std::max(blk_parts_of(s.nparts, s.rows), gc);
    hipLaunchKernelGGL(bsh_pack_fn(D), dim3(grid), dim3(kBlkNT), 0, st, T, s.ld, s.rows,
                       s.m, s.row0, P, bn, ctl, (const BlkHdr*)b.h[0], (const smx_part*)b.parts,
                       blk_parts_of(s.nparts, s.rows), (const double*)b.mul[0], (const double*)b.pr[0], send);
    return (int)hipGetLastError();
}

int launch_blk_publish(bool sh, const smx_shape& s, int parity, int bn, smx_ctl* ctl, const BlkPtrs& b,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_blk_publish, dim3(1), dim3(kWave), 0, st, (const BlkHdr*)b.h[0],
                       (const smx_part*)b.parts, blk_G(s, sh), blk_slot(0, 1, bn), parity, ctl);
    return (int)hipGetLastError();
}

// Sweep layout (smx_tune_block_form): 0 automatic -- the register layout (4) up to kSweepRegMaxP
// pivots, the LDS layout (5) beyond and wherever the register layout's grid cannot give every
// wave one chunk; 4 / 5 forced (tests, A/B timing).
int g_block_form = 0;
constexpr int kSweepRegMaxP = 12;
constexpr int64_t kSweepItemRows = 2048;   // rows per wave from which FORM 6 is automatic

// Grid of the LDS layout: a multiple of the chunks per row (every workgroup keeps one chunk),
// as many workgroups as are resident at bpc per CU, at least one per chunk.
int sweep_grid_lds(const smx_shape& s, int bpc) {
    const int64_t nchunks = (s.m + 1 + 2 * kWave - 1) / (2 * kWave);
    int64_t per = (int64_t)num_cus() * bpc / nchunks;
    const int64_t rows_per = (s.rows + 1 + kUpdWaves - 1) / kUpdWaves;   // >= 1 row per wave
    if (per > rows_per) per = rows_per;
    if (per < 1) per = 1;
    return (int)(per * nchunks);
}

// ipx / in_idx: see blk_out (ipx 0: in place when the pivots applied are even, the layout of the
// unpipelined chains; -1: never in place); plan slot `slot`.  pub_ctl (the chain's last block):
// the pivot-column pass also publishes the chain's final state (block pub_bn's first records,
// parity pub_parity) -- k_blk_publish's work without its launch.
int launch_block_sweep(bool sh, double* tin, double* tother, const smx_shape& s, int P, char* blk,
                       const BlkLayout& L, hipStream_t st, int slot = 0, int ipx = 0,
                       int in_idx = 0, int ipx_part = 0, smx_ctl* pub_ctl = nullptr,
                       int pub_bn = 0, int pub_parity = 0) {
    const int nchunks = (s.m + 1 + 2 * kWave - 1) / (2 * kWave);
    int form = g_block_form >= 4 && g_block_form <= 6 ? g_block_form
                                                      : (P > kSweepRegMaxP ? 5 : 4);
    int grid = 0;
    if (form == 4) {
        // 5 blocks per CU (all resident at 80 VGPRs), 827-882 vs 855-901 us per 10-pivot sweep
        // at 16384^2 over 7 (profiles/r03/bpc_ab.jsonl); the wave count must be a multiple of the
        // chunks per row (update_grid trims it when it can)
        grid = update_grid(s, (const void*)blk_sweep_fn(P, 4), 0, 5);
        if (((int64_t)grid * kUpdWaves) % nchunks != 0) form = 5;
    }
    if (form == 5 && g_block_form == 0) {
        // tall tables: the work-item layout (FORM 6), where each of a wave's K = 16 items keeps
        // >= 128 rows -- config 5 (65536 rows: 2,341 rows per wave) 7 % faster per sweep, its
        // block 0 12 % (a tail of slow chunks spread over the grid); at 16384^2 (256 rows per
        // wave) it cost 7 %, at 8192^2 35 % (profiles/r06ag/)
        const int64_t per = sweep_grid_lds(s, g_blocks_per_cu > 0 ? g_blocks_per_cu : 8) / nchunks;
        if ((int64_t)(s.rows + 1) >= per * kUpdWaves * kSweepItemRows) form = 6;
    }
    BlkSweepFn fn = blk_sweep_fn(P, form);
    if (form >= 5)   // a grid of 8 workgroups per CU.  At P = 20 only 7 are resident (P KiB of
                     // pivot-row slices in LDS, ~106 SGPRs), but the sweep is fp64-issue-bound
                     // there and the grid sized for 8 is as fast as 7 and faster than the
                     // occupancy API's 6: 16384^2, 200 pivots, mean sweep 1.464 / 1.488 / 1.503 ms
                     // at 8 / 7 / 6 (profiles/r05a/).  smx_tune_set(-2, bpc) overrides it.
        grid = sweep_grid_lds(s, g_blocks_per_cu > 0 ? g_blocks_per_cu : 8);
    BlkHdr* hs = reinterpret_cast<BlkHdr*>(blk);
    const BlkHdr* h = reinterpret_cast<const BlkHdr*>(blk + kBlkHdrBytes * slot);
    const double* mul = reinterpret_cast<const double*>(blk + L.mul + slot * L.mul_slot);
    const double* pr = reinterpret_cast<const double*>(blk + L.pr + slot * L.pr_slot);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kUpdBlock), 0, st, tin, tother, s.ld, s.rows + 1,
                       s.m + 1, h, mul, pr, hs, ipx, in_idx);
    // the flag form's pivot columns, or a block cut short by a terminal outcome (does nothing
    // otherwise)
    // one (row, pivot) pair of the pivot columns per thread where that fits (1,280 workgroups at
    // 16384^2 and 20 pivots: 19.2 -> 17.3 us per block, profiles/r05n/stats20; what remains is the
    // pass's scattered 8-B column stores, one per row and pivot)
    const int64_t fix_wg = ((int64_t)(s.rows + 1) * P + kUpdBlock - 1) / kUpdBlock;
    const int rest_grid = (int)std::max<int64_t>(num_cus() * 2,
                                                 std::min<int64_t>(fix_wg, num_cus() * 8));
    hipLaunchKernelGGL(k_blk_sweep_rest, dim3(rest_grid), dim3(kUpdBlock), 0, st, tin,
                       tother, s.ld, s.rows + 1, s.m + 1, P, h, mul, pr, hs, ipx_part, in_idx, 1,
                       ipx, reinterpret_cast<const smx_part*>(blk + L.parts), blk_G(s, sh),
                       blk_slot(0, 1, pub_bn), pub_parity, pub_ctl);
    return (int)hipGetLastError();
}


// k pivots in blocks of P: prime + first records, then per block P step launches and one sweep;
// publish.  ev (optional): 2 events per block recorded around its sweep.  With comm (row-sharded,
// one rank per GPU): every step launch is preceded by this rank's pack and ONE ncclAllGather of
// the send slots into recv, on the same stream.
int launch_block_chain(double* buf0, double* buf1, const smx_shape& s, int parity, int k, int P,
                       smx_ctl* ctl, char* blk, int32_t* log, double* xhist, int64_t log_cap,
                       hipStream_t st, hipEvent_t* ev = nullptr, double* send = nullptr,
                       double* recv = nullptr, int nranks = 0, ncclComm_t comm = nullptr) {
    const BlkPtrs bp = blk_ptrs(s, blk);
    const bool sh = comm != nullptr;
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    // light exchange: the headers land compact at the start of recv, the pivot row after them
    const bool light = sh && xchg_light(nranks);
    int rank = 0;
    if (light && ncclCommUserRank(comm, &rank) != ncclSuccess) return (int)hipErrorInvalidValue;
    double* xrow = light ? recv + (size_t)nranks * SMX_SHARD_HDR : nullptr;
    int err = launch_blk_prime(sh, parity ? buf1 : buf0, s, parity, parity, ctl, bp, st);
    int p = parity, done = 0, bn = 0;
    while (!err && done < k) {
        // blocks of near-equal size (every rank of a sharded chain cuts k the same way; the
        // step-wise smx_bshard_* drivers may cut it differently -- the results do not depend on
        // the cut)
        const int Pb = block_size(k, P, bn);
        double* tin = p ? buf1 : buf0;
        double* toth = p ? buf0 : buf1;
        const bool wplan = use_wplan(s, sh);
        if (!err && wplan)
            err = launch_blk_wplan(tin, s, Pb, p, bn, done, ctl, bp, log, xhist, log_cap, st);
        for (int l = 1; l <= Pb && !err && !wplan; ++l) {
            if (sh) {
                err = launch_bsh_pack(l - 1, tin, s, Pb, bn, ctl, bp, send, st);
                if (!err && !light) {
                    const ncclResult_t r = ncclAllGather(send, recv, slot, ncclFloat64, comm, st);
                    if (r != ncclSuccess) err = -1000 - (int)r;
                } else if (!err) {
                    ncclResult_t r = ncclAllGather(send, recv, SMX_SHARD_HDR, ncclFloat64, comm, st);
                    if (r == ncclSuccess) {
                        err = launch_bsh_pick(recv, s, nranks, rank, send, xrow, st);
                        if (!err)
                            r = ncclAllReduce(xrow, xrow, (size_t)s.ld, ncclInt64, ncclMax, comm,
                                              st);
                    }
                    if (r != ncclSuccess) err = -1000 - (int)r;
                }
            }
            if (!err && use_window(s, sh))
                err = launch_blk_wstep(l, tin, s, Pb, p, bn, ctl, bp, log, xhist, log_cap, st,
                                       bn == 0 && l == 1);
            else if (!err)   // sharded: each rank writes the x-history of the label rows it owns
                err = launch_blk_step(sh, l, tin, s, Pb, p, bn, ctl, bp, recv, nranks, log,
                                      xhist, log_cap, st, xrow,
                                      light ? (int64_t)SMX_SHARD_HDR : 0);
#ifdef SMX_BLK_TRACE_TWICE
            // diagnostic build (tools/trace_planner.hip): a step is idempotent (it reads slot D /
            // parity sp and writes slot L / parity sp^1), so running it again times it warm
            if (!err && !sh)
                err = launch_blk_step(sh, l, tin, s, Pb, p, bn, ctl, bp, recv, nranks, log,
                                      xhist, log_cap, st, xrow, 0);
#endif
        }
        // (the persistent planner builds the pivot rows itself where its column slices fit)
        if (!err && use_window(s, sh) && !(wplan && wp_inpr(s.m + 1, win_groups(s.rows))))
            err = launch_blk_prows(tin, s, Pb, bp, st);
        if (ev) (void)hipEventRecord(ev[2 * bn], st);
        const bool lastb = done + Pb >= k;   // its pivot-column pass publishes the chain
        if (!err)
            err = launch_block_sweep(sh, tin, toth, s, Pb, blk, bp.L, st, 0, 0, p, 0,
                                     lastb ? ctl : nullptr, bn + 1, (p + Pb) & 1);
        if (ev) (void)hipEventRecord(ev[2 * bn + 1], st);
        p = (p + Pb) & 1;
        done += Pb;
        ++bn;
    }
    if (err) return err;
    return bn == 0 ? launch_blk_publish(sh, s, p, bn, ctl, bp, st) : 0;   // (k = 0: no block)
}

bool block_args_ok(const smx_shape* shape, int k, int P, const void* blk, int64_t blk_bytes) {
    if (!shape_ok(shape) || k < 0 || P < 1 || P > kBlkMax || !blk) return false;
    const smx_shape& s = *shape;
    if (s.row0 != 0 || s.rows != s.n || s.rows < 1 || s.m < 1) return false;
    return blk_bytes >= blk_layout(s.rows + 1, s.ld, blk_parts_of(s.nparts, s.rows)).bytes;
}

// row-sharded blocks: any row block (a rank may own no rows), one f-row replica per rank
bool bshard_args_ok(const smx_shape* shape, int P, const void* blk, int64_t blk_bytes) {
    if (!shape_ok(shape) || P < 1 || P > kBlkMax || !blk) return false;
    const smx_shape& s = *shape;
    if (s.rows < 0 || s.n < 1 || s.m < 1 || s.row0 < 0 || s.row0 + s.rows > s.n) return false;
    return blk_bytes >= blk_layout(s.rows + 1, s.ld, blk_parts_of(s.nparts, s.rows)).bytes;
}

struct Graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

// Timing events of the *_run_timed calls: created once (smx_timer_reserve, or on first need) and
// reused, so no hipEventCreate / hipEventDestroy runs inside a caller's timed region.
// The pool belongs to the device that was current when it was filled; a caller on another device
// gets a fresh pool there.  Any new use of the pool invalidates a pending deferred block readout
// (smx_block_run_timed with NULL outputs -> smx_block_timed_read), which would otherwise read
// events that the new caller re-recorded.
hipEvent_t* g_timer_ev = nullptr;
size_t g_timer_n = 0;
int g_timer_dev = -1;
int g_timed_blocks = 0;   // blocks of the pending deferred smx_block_run_timed (0: none)

int timer_events(size_t n, hipEvent_t** out) {
    g_timed_blocks = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (g_timer_n && dev != g_timer_dev) {
        (void)hipSetDevice(g_timer_dev);
        for (size_t i = 0; i < g_timer_n; ++i) (void)hipEventDestroy(g_timer_ev[i]);
        (void)hipSetDevice(dev);
        g_timer_n = 0;
    }
    g_timer_dev = dev;
    if (n > g_timer_n) {
        hipEvent_t* grown = static_cast<hipEvent_t*>(realloc(g_timer_ev, n * sizeof(hipEvent_t)));
        if (!grown) return 1;
        g_timer_ev = grown;
        for (; g_timer_n < n; ++g_timer_n)
            if (hipEventCreate(&g_timer_ev[g_timer_n]) != hipSuccess) return 1;
    }
    *out = g_timer_ev;
    return 0;
}

}  // namespace

extern "C" {

int smx_timer_reserve(int32_t events) {
    hipEvent_t* ev;
    return events < 0 ? (int)hipErrorInvalidValue
                      : (timer_events((size_t)events, &ev) ? (int)hipErrorOutOfMemory : 0);
}

#ifndef SMX_SRC_HASH
#define SMX_SRC_HASH "unstamped"
#endif
int smx_version(char* buf, int len) {
    // "src=" + the source stamp of csrc/Makefile (SRC_HASH), checked by simplex_mi355x/_lib.py
    const char* v = "smx 0.2 gfx950 fp64 src=" SMX_SRC_HASH;
    if (buf && len > 0) {
        strncpy(buf, v, (size_t)len - 1);
        buf[len - 1] = 0;
    }
    return 8;
}

int smx_nparts_for(int32_t rows, int32_t m) { return nparts_for(rows, m); }

int smx_tune_set(int32_t variant, int32_t blocks_per_cu_override) {
    if (variant >= kNumVariants) return (int)hipErrorInvalidValue;
    if (variant >= kFirstDiagVariant) {   // wrong-bits timing variants: explicit opt-in only
        const char* env = getenv("SMX_ALLOW_DIAG");
        if (!env || env[0] != '1') return (int)hipErrorInvalidValue;
    }
    if (variant >= 0 || variant == -2) g_variant = variant >= 0 ? variant : -1;
    if (blocks_per_cu_override >= 0) g_blocks_per_cu = blocks_per_cu_override;
    return 0;
}

int64_t smx_tune_fold(int64_t min_bytes) {
    const int64_t prev = g_fold_min_bytes;
    if (min_bytes >= 0) g_fold_min_bytes = min_bytes;
    return prev;
}

int smx_tune_fused(int32_t on) {
    const int prev = g_fused;
    if (on >= 0) g_fused = on > 3 ? 3 : on;
    return prev;
}

int smx_tune_get(int32_t* variant, int32_t* blocks_per_cu_override, int32_t* nvariants,
                 int32_t* units_in_flight, int32_t* vec, int32_t* nt) {
    if (variant) *variant = g_variant;
    if (blocks_per_cu_override) *blocks_per_cu_override = g_blocks_per_cu;
    if (nvariants) *nvariants = kNumVariants;
    const int gv = g_variant >= 0 ? g_variant : kLargeVariant;   // auto: report the HBM one
    if (units_in_flight) *units_in_flight = kVariants[gv].u;
    if (vec) *vec = 2;
    if (nt) *nt = kVariants[gv].nts | (kVariants[gv].ntl << 1) | (kVariants[gv].pipe << 2);
    return 0;
}

int smx_reset(const double* T, const smx_shape* shape, int32_t parity, int32_t clear_count,
              smx_ctl* ctl, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_reset, dim3(1), dim3(1024), 0, S(stream), T, shape->ld, shape->rows,
                       shape->m, fscan_of(*shape), shape->row0, parity & 1, clear_count, ctl);
    return (int)hipGetLastError();
}

int smx_select(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
               smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_select(T, *shape, parity & 1, ctl, parts, S(stream));
}

int smx_finalize(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                 const smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kWave), 0, S(stream), parts, shape->nparts,
                       parity & 1, shape->n, shape->m, shape->flen, T, shape->ld, ctl);
    return (int)hipGetLastError();
}

int smx_update(const double* Tin, double* Tout, const smx_shape* shape, int32_t parity,
               smx_ctl* ctl, const smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
               void* stream) {
    if (!shape_ok(shape) || Tin == Tout) return (int)hipErrorInvalidValue;
    return launch_update(Tin, Tout, *shape, parity & 1, ctl, parts, log, xhist, log_cap,
                         S(stream));
}

int smx_set_xpos(smx_ctl* ctl, int32_t parity, int32_t x1code, int32_t x2code, void* stream) {
    hipLaunchKernelGGL(k_set_xpos, dim3(1), dim3(kWave), 0, S(stream), ctl, parity & 1, x1code,
                       x2code);
    return (int)hipGetLastError();
}

int smx_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
            smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
            void* stream) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 0) return (int)hipErrorInvalidValue;
    return launch_chain(buf0, buf1, *shape, parity & 1, k, ctl, parts, log, xhist, log_cap,
                        S(stream));
}

int smx_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
                  void* stream, float* host_update_ms, float* host_total_ms) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 1 || !host_update_ms || !host_total_ms)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    const int p0 = parity & 1;
    hipEvent_t* ev = nullptr;
    int err = 0;
    if (timer_events((size_t)(2 * k + 1), &ev)) return (int)hipErrorOutOfMemory;
    (void)hipEventRecord(ev[2 * k], st);
    if (g_fused) err = launch_prime(p0 ? buf1 : buf0, *shape, p0, ctl, parts, st);
    for (int step = 0; step < k && !err; ++step) {
        const int p = (p0 + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        if (g_fused) {
            (void)hipEventRecord(ev[2 * step], st);
            err = launch_update_mode<kFused>(tin, tout, *shape, p, ctl, parts, log, xhist,
                                             log_cap, nullptr, 0, 0, st);
            (void)hipEventRecord(ev[2 * step + 1], st);
            continue;
        }
        err = launch_select(tin, *shape, p, ctl, parts, st);
        if (err) break;
        (void)hipEventRecord(ev[2 * step], st);
        err = launch_update(tin, tout, *shape, p, ctl, parts, log, xhist, log_cap, st);
        (void)hipEventRecord(ev[2 * step + 1], st);
    }
    if (!err && g_fused) err = launch_publish(*shape, (p0 + k) & 1, ctl, parts, st);
    if (!err) err = (int)hipEventSynchronize(ev[2 * k - 1]);
    if (!err) {
        for (int step = 0; step < k; ++step)
            (void)hipEventElapsedTime(&host_update_ms[step], ev[2 * step], ev[2 * step + 1]);
        (void)hipEventElapsedTime(host_total_ms, ev[2 * k], ev[2 * k - 1]);
    }
    return err;
}

int smx_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                     int32_t k, smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist,
                     int64_t log_cap, void* stream, void** graph_out) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 1 || !graph_out) return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    Graph* g = new Graph();
    hipError_t err = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    if (err != hipSuccess) {
        delete g;
        return (int)err;
    }
    int lerr = launch_chain(buf0, buf1, *shape, parity & 1, k, ctl, parts, log, xhist, log_cap,
                            st);
    err = hipStreamEndCapture(st, &g->graph);
    if (lerr || err != hipSuccess) {
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return lerr ? lerr : (int)err;
    }
    err = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    if (err != hipSuccess) {
        (void)hipGraphDestroy(g->graph);
        delete g;
        return (int)err;
    }
    *graph_out = g;
    return 0;
}

int smx_graph_launch(void* graph, void* stream) {
    if (!graph) return (int)hipErrorInvalidValue;
    return (int)hipGraphLaunch(static_cast<Graph*>(graph)->exec, S(stream));
}

int smx_graph_destroy(void* graph) {
    if (!graph) return 0;
    Graph* g = static_cast<Graph*>(graph);
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    delete g;
    return 0;
}

int smx_update_forced(const double* Tin, double* Tout, const smx_shape* shape, int32_t r,
                      int32_t c, void* stream) {
    if (!shape_ok(shape) || Tin == Tout) return (int)hipErrorInvalidValue;
    if (r < 0 || r >= shape->rows || c < 0 || c > shape->m) return (int)hipErrorInvalidValue;
    return launch_update_mode<kForced>(Tin, Tout, *shape, 0, nullptr, nullptr, nullptr, nullptr,
                                       0, nullptr, r, c, S(stream));
}

int smx_shard_pack(const double* T, const smx_shape* shape, int32_t parity, const smx_ctl* ctl,
                   const smx_part* parts, double* send, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_pack<false>(T, *shape, parity & 1, ctl, parts, send, S(stream));
}

int smx_shard_merge(const double* recv, int32_t nranks, const smx_shape* shape,
                    int32_t parity, smx_ctl* ctl, int32_t* log, int64_t log_cap, void* stream) {
    (void)parity;
    if (!shape_ok(shape) || nranks < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_merge, dim3(1), dim3(kWave), 0, S(stream), recv, nranks, shape->ld,
                       shape->n, shape->m, shape->flen, ctl, log, log_cap);
    return (int)hipGetLastError();
}

int smx_shard_update(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                     const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                     int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || Tin == Tout || nranks < 1) return (int)hipErrorInvalidValue;
    smx_shape sh = *shape;
    sh.nparts = nranks;   // the update kernel's partial count is the rank count in shard mode
    return launch_update_mode<kShard>(Tin, Tout, sh, parity & 1, ctl, nullptr, log, nullptr,
                                      log_cap, recv, 0, 0, S(stream));
}


int smx_batch_solve(const double* tabs, const int32_t* dims, int32_t B, int32_t Rmax,
                    int32_t ldb, int32_t max_pivots, double* out, int32_t* rc, double* xv,
                    double* snaps, int32_t* status, int32_t* npivots, void* stream) {
    if (B < 0 || Rmax < 1 || Rmax > kWave || ldb < 1 || ldb > 64 || max_pivots < 0)
        return (int)hipErrorInvalidValue;
    if (B == 0) return 0;
    const dim3 grid((B + 3) / 4), block(256);
    hipStream_t st = S(stream);
    if (ldb <= 4)
        hipLaunchKernelGGL(k_batch<4>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else if (ldb <= 8)
        hipLaunchKernelGGL(k_batch<8>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else if (ldb <= 16)
        hipLaunchKernelGGL(k_batch<16>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else if (ldb <= 32)
        hipLaunchKernelGGL(k_batch<32>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    else
        hipLaunchKernelGGL(k_batch<64>, grid, block, 0, st, tabs, dims, B, Rmax, ldb, max_pivots,
                           out, rc, xv, snaps, status, npivots);
    return (int)hipGetLastError();
}


// ---- native RCCL shard driver: the all-gather on the solver's own stream --------------------
// (torch.distributed would run it on its own NCCL stream: one cross-stream event wait per pivot,
// ~14 us measured; here the whole pivot -- select, pack, ncclAllGather, update -- is one
// stream-ordered sequence that can also be captured in a hipGraph.)
static int nccl_err(ncclResult_t r) { return r == ncclSuccess ? 0 : -1000 - (int)r; }

int smx_comm_unique_id(void* id_out) {
    if (!id_out) return (int)hipErrorInvalidValue;
    ncclUniqueId id;
    const int err = nccl_err(ncclGetUniqueId(&id));
    if (!err) memcpy(id_out, &id, sizeof(id));
    return err;
}

int smx_comm_init(void** comm_out, int32_t nranks, const void* id, int32_t rank) {
    if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return (int)hipErrorInvalidValue;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const int err = nccl_err(ncclCommInitRank(&comm, nranks, uid, rank));
    if (!err) *comm_out = comm;
    return err;
}

int smx_comm_destroy(void* comm) {
    if (!comm) return 0;
    return nccl_err(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)));
}

int smx_comm_info(void* comm, int32_t* count, int32_t* rank, int32_t* device) {
    if (!comm || !count || !rank || !device) return (int)hipErrorInvalidValue;
    ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
    int v = 0;
    int err = nccl_err(ncclCommCount(c, &v));
    if (err) return err;
    *count = v;
    if ((err = nccl_err(ncclCommUserRank(c, &v)))) return err;
    *rank = v;
    if ((err = nccl_err(ncclCommCuDevice(c, &v)))) return err;
    *device = v;
    return 0;
}

namespace {
// Fused sharded chain, per pivot: k_pack<true> (step k's records -> header + candidate rows)
// -> one ncclAllGather -> k_update<kShardFused> (merge, sweep, step k+1's records; with
// smx_tune_fold also step k+1's pack, then the next k_pack is skipped).  Primed by k_la_prime,
// closed by k_publish.  e_upd: 2k events around the updates.
int shard_chain_fused(double* buf0, double* buf1, const smx_shape& s, int parity, int k,
                      smx_ctl* ctl, smx_part* parts, double* send, double* recv, int nranks,
                      ncclComm_t comm, int32_t* log, int64_t log_cap, hipEvent_t* e_upd,
                      hipStream_t st) {
    double* T0 = parity ? buf1 : buf0;
    const bool fold = folds_pack(s);
    int err = launch_prime(T0, s, parity, ctl, parts, st);
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    for (int step = 0; step < k && !err; ++step) {
        const int p = (parity + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        if (step == 0 || !fold)
            err = launch_pack<true>(tin, s, p, ctl, parts + (size_t)p * s.nparts, send, st);
        if (!err) err = nccl_err(ncclAllGather(send, recv, slot, ncclFloat64, comm, st));
        if (err) break;
        if (e_upd) (void)hipEventRecord(e_upd[2 * step], st);
        err = launch_update_mode<kShardFused>(tin, tout, s, p, ctl, parts, log, nullptr, log_cap,
                                              recv, 0, nranks, st, 0, fold ? send : nullptr);
        if (e_upd) (void)hipEventRecord(e_upd[2 * step + 1], st);
    }
    if (!err) err = launch_publish(s, (parity + k) & 1, ctl, parts, st);
    return err;
}

// The two halves of an overlapped sharded step (also exported for the P-rank simulation tests):
// ahead = step k+1's records (s.nparts of them, slot parity^1) and, if `pack`, its header and
// candidate rows into `send`, from T_k and step k's gathered headers; sweep = the update of step
// k without look-ahead workgroups, leaving `reserve` resident slots free.
int launch_ahead(const double* T, const smx_shape& s, int parity, const double* recv,
                 int nranks, smx_ctl* ctl, smx_part* parts, double* send, bool pack,
                 hipStream_t st) {
    smx_part* pn = parts + (size_t)(parity ^ 1) * s.nparts;
    hipLaunchKernelGGL(k_shard_la, dim3(s.nparts), dim3(kUpdBlock), 0, st, T, s.ld, s.rows, s.m,
                       s.flen, fscan_of(s), s.row0, recv, nranks, ctl, pn, parity ^ 1);
    if (pack)
        hipLaunchKernelGGL(k_pack_ahead, dim3(s.nparts), dim3(kUpdBlock), 0, st, T, s.ld, s.rows,
                           s.m, s.flen, s.row0, recv, nranks, ctl, pn, s.nparts, parity ^ 1,
                           send);
    return (int)hipGetLastError();
}

int launch_sweep(const double* Tin, double* Tout, const smx_shape& s, int parity,
                 const double* recv, int nranks, smx_ctl* ctl, int32_t* log, int64_t log_cap,
                 int reserve, hipStream_t st) {
    smx_shape sy = s;
    sy.nparts = 0;   // no look-ahead workgroups
    return launch_update_mode<kShardFused>(Tin, Tout, sy, parity, ctl, nullptr, log, nullptr,
                                           log_cap, recv, 0, nranks, st, reserve);
}

// The exchange stream and two events of the overlapped chain, created once per device.
struct Overlap {
    hipStream_t s2 = nullptr;
    hipEvent_t ev_sweep = nullptr, ev_gather = nullptr;
    uint64_t* sig[2] = {nullptr, nullptr};   // signal memory: sweeps done, gathers done
    uint64_t seq = 0;                        // next base of the (monotonic) counters
};

int overlap_for_device(Overlap** out) {
    static Overlap cache[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return (int)hipErrorInvalidDevice;
    Overlap& o = cache[dev];
    if (!o.s2) {
        hipError_t e = hipStreamCreateWithFlags(&o.s2, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&o.ev_sweep, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&o.ev_gather, hipEventDisableTiming);
        if (e != hipSuccess) return (int)e;
    }
    *out = &o;
    return 0;
}

constexpr int kOverlapParts = 16;   // look-ahead workgroups of the overlapped chain

// Overlapped sharded chain.  recv holds two gather slots (step parity).  Per step k:
//   S2: wait(T_k ready) -> k_shard_la (records of k+1) -> k_pack_ahead -> all-gather into
//       recv[(k+1)&1] -> record ev_gather
//   S1: k_update<kShardFused> without look-ahead workgroups (T_k -> T_{k+1}, pivot from
//       recv[k&1]) -> wait(ev_gather) -> record ev_sweep
// S1 waiting for the gather before the next sweep also orders S2's reads of T_k before the
// sweep that overwrites it.  The last step computes the records of step k (for a continuation)
// but no pack/gather.
int shard_chain_overlap(double* buf0, double* buf1, const smx_shape& s, int parity, int k,
                        smx_ctl* ctl, smx_part* parts, double* send, double* recv, int nranks,
                        ncclComm_t comm, int32_t* log, int64_t log_cap, hipEvent_t* e_upd,
                        hipStream_t st, bool values) {
    Overlap* o = nullptr;
    int err = overlap_for_device(&o);
    if (err) return err;
    for (int q = 0; values && q < 2 && !o->sig[q]; ++q) {   // one 8-B signal each, zeroed
        hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&o->sig[q]),
                                             sizeof(uint64_t), hipMallocSignalMemory);
        if (e == hipSuccess) e = hipStreamWriteValue64(st, o->sig[q], 0, 0);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            o->sig[q] = nullptr;
            return (int)e;
        }
    }
    smx_shape sx = s;
    sx.nparts = s.nparts < kOverlapParts ? s.nparts : kOverlapParts;
    const int npx = sx.nparts;
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    const size_t rsz = (size_t)nranks * slot;
    double* T0 = parity ? buf1 : buf0;
    err = launch_prime(T0, sx, parity, ctl, parts, st);
    if (!err) err = launch_pack<true>(T0, sx, parity, ctl, parts + (size_t)parity * npx, send, st);
    if (!err) err = nccl_err(ncclAllGather(send, recv + (size_t)parity * rsz, slot, ncclFloat64,
                                           comm, st));
    // `values`: the two cross-stream dependencies as stream memory operations on monotonic
    // counters (sig[0] = sweeps done + 1, sig[1] = gathers done) instead of events
    const uint64_t base = o->seq;
    auto signal_sweep = [&](uint64_t v) {
        return values ? (int)hipStreamWriteValue64(st, o->sig[0], base + v, 0)
                      : (int)hipEventRecord(o->ev_sweep, st);
    };
    if (!err) err = signal_sweep(1);
    for (int step = 0; step < k && !err; ++step) {
        const int p = (parity + step) & 1;
        double* tin = p ? buf1 : buf0;
        double* tout = p ? buf0 : buf1;
        const double* rc = recv + (size_t)p * rsz;
        double* rn = recv + (size_t)(p ^ 1) * rsz;
        const bool more = step + 1 < k;
        err = values ? (int)hipStreamWaitValue64(o->s2, o->sig[0], base + step + 1,
                                                 hipStreamWaitValueGte, ~0ull)
                     : (int)hipStreamWaitEvent(o->s2, o->ev_sweep, 0);
        if (!err) err = launch_ahead(tin, sx, p, rc, nranks, ctl, parts, send, more, o->s2);
        if (!err && more)
            err = nccl_err(ncclAllGather(send, rn, slot, ncclFloat64, comm, o->s2));
        if (!err)
            err = values ? (int)hipStreamWriteValue64(o->s2, o->sig[1], base + step + 1, 0)
                         : (int)hipEventRecord(o->ev_gather, o->s2);
        if (err) break;
        if (e_upd) (void)hipEventRecord(e_upd[2 * step], st);
        err = launch_sweep(tin, tout, s, p, rc, nranks, ctl, log, log_cap, npx, st);
        if (e_upd) (void)hipEventRecord(e_upd[2 * step + 1], st);
        if (!err)
            err = values ? (int)hipStreamWaitValue64(st, o->sig[1], base + step + 1,
                                                     hipStreamWaitValueGte, ~0ull)
                         : (int)hipStreamWaitEvent(st, o->ev_gather, 0);
        if (!err) err = signal_sweep(step + 2);
    }
    o->seq = base + k + 2;
    if (!err) err = launch_publish(sx, (parity + k) & 1, ctl, parts, st);
    return err;
}

int shard_pivot(double* tin, double* tout, const smx_shape& s, int p, smx_ctl* ctl,
                smx_part* parts, double* send, double* recv, int nranks, ncclComm_t comm,
                int32_t* log, int64_t log_cap, hipEvent_t e0, hipEvent_t e1, hipStream_t st) {
    int err = launch_select(tin, s, p, ctl, parts, st);
    if (err) return err;
    err = smx_shard_pack(tin, &s, p, ctl, parts, send, st);
    if (err) return err;
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)s.ld;
    err = nccl_err(ncclAllGather(send, recv, slot, ncclFloat64, comm, st));
    if (err) return err;
    if (e0) (void)hipEventRecord(e0, st);
    err = smx_shard_update(tin, tout, recv, nranks, &s, p, ctl, log, log_cap, st);
    if (e1) (void)hipEventRecord(e1, st);
    return err;
}
}  // namespace

int smx_shard_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  smx_ctl* ctl, smx_part* parts, double* send, double* recv, int32_t nranks,
                  void* comm, int32_t* log, int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || !comm || nranks < 1 || k < 0) return (int)hipErrorInvalidValue;
    if (g_fused >= 2 && k > 0)
        return shard_chain_overlap(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                   nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap,
                                   nullptr, S(stream), g_fused == 3);
    if (g_fused && k > 0)
        return shard_chain_fused(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                 nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap,
                                 nullptr, S(stream));
    for (int step = 0; step < k; ++step) {
        const int p = (parity + step) & 1;
        const int err = shard_pivot(p ? buf1 : buf0, p ? buf0 : buf1, *shape, p, ctl, parts,
                                    send, recv, nranks, reinterpret_cast<ncclComm_t>(comm), log,
                                    log_cap, nullptr, nullptr, S(stream));
        if (err) return err;
    }
    return 0;
}

int smx_shard_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                        int32_t k, smx_ctl* ctl, smx_part* parts, double* send, double* recv,
                        int32_t nranks, void* comm, int32_t* log, int64_t log_cap, void* stream,
                        float* host_update_ms, float* host_total_ms) {
    if (!shape_ok(shape) || !comm || nranks < 1 || k < 1 || !host_update_ms || !host_total_ms)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    hipEvent_t* ev = nullptr;
    if (timer_events((size_t)(2 * k + 1), &ev)) return (int)hipErrorOutOfMemory;
    (void)hipEventRecord(ev[2 * k], st);
    int err = 0;
    if (g_fused >= 2)
        err = shard_chain_overlap(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                  nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap, ev,
                                  st, g_fused == 3);
    else if (g_fused)
        err = shard_chain_fused(buf0, buf1, *shape, parity & 1, k, ctl, parts, send, recv,
                                nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap, ev, st);
    for (int step = 0; step < k && !err && !g_fused; ++step) {
        const int p = (parity + step) & 1;
        err = shard_pivot(p ? buf1 : buf0, p ? buf0 : buf1, *shape, p, ctl, parts, send, recv,
                          nranks, reinterpret_cast<ncclComm_t>(comm), log, log_cap, ev[2 * step],
                          ev[2 * step + 1], st);
    }
    if (!err) err = (int)hipEventSynchronize(ev[2 * k - 1]);
    if (!err) {
        for (int step = 0; step < k; ++step)
            (void)hipEventElapsedTime(&host_update_ms[step], ev[2 * step], ev[2 * step + 1]);
        (void)hipEventElapsedTime(host_total_ms, ev[2 * k], ev[2 * k - 1]);
    }
    return err;
}

int smx_shard_fused_prime(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                          smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_prime(T, *shape, parity & 1, ctl, parts, S(stream));
}

int smx_shard_fused_begin(const double* T, const smx_shape* shape, int32_t parity,
                          const smx_ctl* ctl, const smx_part* parts, double* send, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_pack<true>(T, *shape, parity & 1, ctl,
                             parts + (size_t)(parity & 1) * shape->nparts, send, S(stream));
}

int smx_shard_fused_finish(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                           const smx_shape* shape, int32_t parity, smx_ctl* ctl, smx_part* parts,
                           double* send, int32_t* log, int64_t log_cap, void* ev_before,
                           void* ev_after, void* stream) {
    if (!shape_ok(shape) || Tin == Tout || nranks < 1) return (int)hipErrorInvalidValue;
    if (ev_before) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_before), S(stream));
    const int err = launch_update_mode<kShardFused>(Tin, Tout, *shape, parity & 1, ctl, parts,
                                                    log, nullptr, log_cap, recv, 0, nranks,
                                                    S(stream), 0,
                                                    folds_pack(*shape) ? send : nullptr);
    if (ev_after) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_after), S(stream));
    return err;
}

int smx_shard_folds_pack(const smx_shape* shape) {
    return shape_ok(shape) && folds_pack(*shape) ? 1 : 0;
}

int smx_shard_ahead(const double* T, const smx_shape* shape, int32_t parity, const double* recv,
                    int32_t nranks, smx_ctl* ctl, smx_part* parts, double* send, void* stream) {
    if (!shape_ok(shape) || nranks < 1) return (int)hipErrorInvalidValue;
    return launch_ahead(T, *shape, parity & 1, recv, nranks, ctl, parts, send, true, S(stream));
}

int smx_shard_sweep(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                    const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                    int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || Tin == Tout || nranks < 1) return (int)hipErrorInvalidValue;
    return launch_sweep(Tin, Tout, *shape, parity & 1, recv, nranks, ctl, log, log_cap, 0,
                        S(stream));
}

int smx_copy_probe(const double* src, double* dst, int64_t ndoubles, int32_t variant,
                   void* stream) {
    if (!src || !dst || ndoubles < 2 || (ndoubles & 1) || variant < 0 || variant > 1)
        return (int)hipErrorInvalidValue;
    const int64_t n2 = ndoubles / 2;
    const auto* a = reinterpret_cast<const dbl2*>(src);
    auto* b = reinterpret_cast<dbl2*>(dst);
    if (variant == 0)
        hipLaunchKernelGGL(k_copy<4>, dim3(num_cus()), dim3(256), 0, S(stream), a, b, n2);
    else
        hipLaunchKernelGGL(k_copy<1>, dim3(num_cus()), dim3(1024), 0, S(stream), a, b, n2);
    return (int)hipGetLastError();
}

int smx_fused_publish(const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                      const smx_part* parts, void* stream) {
    if (!shape_ok(shape)) return (int)hipErrorInvalidValue;
    return launch_publish(*shape, parity & 1, ctl, parts, S(stream));
}

int smx_shard_begin(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                    smx_part* parts, double* send, void* stream) {
    int err = smx_select(T, shape, parity, ctl, parts, stream);
    if (err) return err;
    return smx_shard_pack(T, shape, parity, ctl, parts, send, stream);
}

int smx_shard_finish(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                     const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                     int64_t log_cap, void* ev_before, void* ev_after, void* stream) {
    if (ev_before) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_before), S(stream));
    const int err = smx_shard_update(Tin, Tout, recv, nranks, shape, parity, ctl, log, log_cap,
                                     stream);
    if (ev_after) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_after), S(stream));
    return err;
}

int smx_tune_resident_overlap(int32_t on) {
    const int prev = g_resident_ovl;
    if (on >= 0 && on <= 2) g_resident_ovl = on;
    return prev;
}

int smx_tune_resident(int32_t workgroups) {
    const int prev = g_resident;
    if (workgroups >= -1) g_resident = workgroups > kResBlock ? kResBlock : workgroups;
    return prev;
}

int64_t smx_tune_resident_timeout(int64_t ticks) {
    int64_t prev = -1;
    if (hipMemcpyFromSymbol(&prev, HIP_SYMBOL(g_res_spin_ticks), sizeof prev) != hipSuccess)
        return -1;
    if (ticks >= 0 &&
        hipMemcpyToSymbol(HIP_SYMBOL(g_res_spin_ticks), &ticks, sizeof ticks) != hipSuccess)
        return -1;
    return prev;
}

int smx_resident_trace(void* trace, int32_t from_step) {
    g_resident_trace = static_cast<uint64_t*>(trace);
    g_resident_trace_from = from_step < 0 ? 0 : from_step;
    return 0;
}

int64_t smx_resident_bytes(const smx_shape* shape, int32_t* plan_out) {
    ResPlan p;
    if (!shape_ok(shape) || !resident_plan(*shape, &p)) return 0;
    if (plan_out) {
        plan_out[0] = p.G;
        plan_out[1] = p.rpw;
        plan_out[2] = p.ept;
        plan_out[3] = (int32_t)p.lds;
    }
    return p.bytes;
}

int smx_resident_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                     int32_t k, smx_ctl* ctl, void* xch, int64_t xch_bytes, int32_t epoch,
                     int32_t* log, double* xhist, int64_t log_cap, void* stream) {
    if (!shape_ok(shape) || buf0 == buf1 || k < 0) return (int)hipErrorInvalidValue;
    return launch_resident(buf0, buf1, *shape, parity & 1, k, ctl, xch, xch_bytes,
                           (uint32_t)epoch, log, xhist, log_cap, S(stream));
}

int smx_fastdiv_check(const double* num, const double* den, int64_t count,
                      unsigned long long* out, void* stream) {
    if (count < 0 || !num || !den || !out) return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), S(stream));
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_fastdiv_check, dim3(1024), dim3(256), 0, S(stream), num, den, count,
                       out);
    return (int)hipGetLastError();
}

int smx_fastdiv_check_bounded(const double* num, const double* den, int64_t count,
                              unsigned long long* out, void* stream) {
    if (count < 0 || !num || !den || !out) return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(out, 0, 4 * sizeof(unsigned long long), S(stream));
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_fastdiv_bounded_check, dim3(1024), dim3(256), 0, S(stream), num, den,
                       count, out);
    return (int)hipGetLastError();
}

int smx_diag_path_counts(int64_t* out, int32_t count, int32_t clear) {
#ifdef SMX_PATH_COUNT
    if (!out || count < 0) return (int)hipErrorInvalidValue;
    unsigned long long v[kPcCount];
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_path_cnt), sizeof v);
    if (e != hipSuccess) return (int)e;
    for (int k = 0; k < count && k < kPcCount; ++k) out[k] = (int64_t)v[k];
    if (clear) {
        static const unsigned long long zero[kPcCount] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_path_cnt), zero, sizeof zero);
    }
    return e == hipSuccess ? kPcCount : (int)e;
#else
    (void)out;
    (void)count;
    (void)clear;
    return -(int)hipErrorNotSupported;   // product build: no counters
#endif
}

int smx_tune_block_form(int32_t form) {
    const int prev = g_block_form;
    if (form == 0 || (form >= 4 && form <= 6)) g_block_form = form;
    return prev;
}

int smx_tune_block_planner(int32_t planner, int32_t nwin) {
    const int prev = g_block_planner;
    if (planner >= 0 && planner <= 2) g_block_planner = planner;
    if (nwin >= 2 && nwin <= kWin) g_block_nwin = nwin;
    else if (nwin == 0) g_block_nwin = kWin;
    return prev;
}

int smx_tune_block(int32_t pivots) {
    const int prev = g_block;
    if (pivots >= 0) g_block = pivots > kBlkMax ? kBlkMax : pivots;
    return prev;
}

int64_t smx_block_bytes(const smx_shape* shape, int32_t* pivots_inout) {
    // SMX_BLK_NOFREE=1 (A/B experiments): set once, here, outside any stream capture
    static const int nofree_env = [] {
        const char* e = getenv("SMX_BLK_NOFREE");
        const int v = (e && e[0] == '1') ? 1 : 0;
        if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_blk_nofree), &v, sizeof v);
        // SMX_SWEEP_ITEMS=K: work items per workgroup of the sweep's FORM 6 (default 16)
        const char* it = getenv("SMX_SWEEP_ITEMS");
        const int k = it ? atoi(it) : 0;
        if (k > 0) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sweep_items), &k, sizeof k);
        return v;
    }();
    (void)nofree_env;
    if (!shape_ok(shape)) return 0;
    const int req = pivots_inout ? *pivots_inout : 0;
    if (req < 0 || req > kBlkMax) return 0;
    const int P = req > 0 ? req : block_pivots(*shape);
    if (P < 1 || !block_args_ok(shape, 0, P, shape, INT64_MAX)) return 0;
    if (pivots_inout) *pivots_inout = P;
    return blk_layout(shape->rows + 1, shape->ld, blk_parts_of(shape->nparts, shape->rows)).bytes;
}

int smx_block_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes, int32_t* log,
                  double* xhist, int64_t log_cap, void* stream) {
    if (!block_args_ok(shape, k, pivots, blk, blk_bytes) || buf0 == buf1 || !ctl)
        return (int)hipErrorInvalidValue;
    if (k == 0) return 0;
    return launch_block_chain(buf0, buf1, *shape, parity & 1, k, pivots, ctl,
                            static_cast<char*>(blk), log, xhist, log_cap, S(stream));
}

static int block_timed_read(int nb, float* host_sweep_ms, float* host_total_ms) {
    hipEvent_t* ev = g_timer_ev;
    int err = (int)hipEventSynchronize(ev[2 * nb + 1]);
    if (!err) {
        for (int b = 0; b < nb; ++b)
            (void)hipEventElapsedTime(&host_sweep_ms[b], ev[2 * b], ev[2 * b + 1]);
        (void)hipEventElapsedTime(host_total_ms, ev[2 * nb], ev[2 * nb + 1]);
    }
    return err;
}

int smx_block_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                        int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                        int32_t* log, double* xhist, int64_t log_cap, void* stream,
                        float* host_sweep_ms, float* host_total_ms) {
    // both outputs NULL: launch only (asynchronous); smx_block_timed_read waits and reads
    const bool defer = !host_sweep_ms && !host_total_ms;
    if (!block_args_ok(shape, k, pivots, blk, blk_bytes) || buf0 == buf1 || !ctl || k < 1 ||
        (!defer && (!host_sweep_ms || !host_total_ms)))
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    const int nb = (k + pivots - 1) / pivots;
    hipEvent_t* ev = nullptr;
    if (timer_events((size_t)(2 * nb + 2), &ev)) return (int)hipErrorOutOfMemory;
    (void)hipEventRecord(ev[2 * nb], st);
    int err = launch_block_chain(buf0, buf1, *shape, parity & 1, k, pivots, ctl,
                               static_cast<char*>(blk), log, xhist, log_cap, st, ev);
    (void)hipEventRecord(ev[2 * nb + 1], st);
    if (defer) {
        if (!err) g_timed_blocks = nb;
        return err;
    }
    return err ? err : block_timed_read(nb, host_sweep_ms, host_total_ms);
}

int smx_block_timed_read(int32_t blocks, float* host_sweep_ms, float* host_total_ms) {
    if (blocks < 1 || blocks != g_timed_blocks || !host_sweep_ms || !host_total_ms)
        return (int)hipErrorInvalidValue;
    g_timed_blocks = 0;
    return block_timed_read(blocks, host_sweep_ms, host_total_ms);
}

int smx_block_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                           int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                           int32_t* log, double* xhist, int64_t log_cap, void* stream,
                           void** graph_out) {
    if (!block_args_ok(shape, k, pivots, blk, blk_bytes) || buf0 == buf1 || !ctl || k < 1 ||
        !graph_out)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    Graph* g = new Graph();
    hipError_t err = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    if (err != hipSuccess) {
        delete g;
        return (int)err;
    }
    int lerr = launch_block_chain(buf0, buf1, *shape, parity & 1, k, pivots, ctl,
                                static_cast<char*>(blk), log, xhist, log_cap, st);
    err = hipStreamEndCapture(st, &g->graph);
    if (lerr || err != hipSuccess) {
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return lerr ? lerr : (int)err;
    }
    err = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    if (err != hipSuccess) {
        (void)hipGraphDestroy(g->graph);
        delete g;
        return (int)err;
    }
    *graph_out = g;
    return 0;
}

int64_t smx_bshard_bytes(const smx_shape* shape) {
    if (!bshard_args_ok(shape, 1, shape, INT64_MAX)) return 0;
    return blk_layout(shape->rows + 1, shape->ld, blk_parts_of(shape->nparts, shape->rows)).bytes;
}

int smx_bshard_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                   int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes, double* send,
                   double* recv, int32_t nranks, void* comm, int32_t* log, double* xhist,
                   int64_t log_cap, void* stream) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || buf0 == buf1 || !ctl || !send ||
        !recv || nranks < 1 || !comm || k < 0)
        return (int)hipErrorInvalidValue;
    if (k == 0) return 0;
    return launch_block_chain(buf0, buf1, *shape, parity & 1, k, pivots, ctl,
                              static_cast<char*>(blk), log, xhist, log_cap, S(stream), nullptr,
                              send, recv, nranks, reinterpret_cast<ncclComm_t>(comm));
}

// The chain of smx_bshard_run captured once (prime; per block P x [pack -> RCCL exchange ->
// step], one sweep; publish) -- RCCL collectives are capturable, so one hipGraphLaunch replays
// the whole per-rank chain and the host enqueues O(1) work per k pivots instead of 3-5 calls per
// pivot.  The graph is bound to its buffers, comm and parity: a replay starts from
// buf[parity] and leaves the table in buf[(parity + k) & 1].
int smx_bshard_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                            int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                            double* send, double* recv, int32_t nranks, void* comm, int32_t* log,
                            double* xhist, int64_t log_cap, void* stream, void** graph_out) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || buf0 == buf1 || !ctl || !send ||
        !recv || nranks < 1 || !comm || k < 1 || !graph_out)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    Graph* g = new Graph();
    hipError_t err = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    if (err != hipSuccess) {
        delete g;
        return (int)err;
    }
    int lerr = launch_block_chain(buf0, buf1, *shape, parity & 1, k, pivots, ctl,
                                  static_cast<char*>(blk), log, xhist, log_cap, st, nullptr, send,
                                  recv, nranks, reinterpret_cast<ncclComm_t>(comm));
    err = hipStreamEndCapture(st, &g->graph);
    if (lerr || err != hipSuccess) {
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return lerr ? lerr : (int)err;
    }
    err = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    if (err != hipSuccess) {
        (void)hipGraphDestroy(g->graph);
        delete g;
        return (int)err;
    }
    *graph_out = g;
    return 0;
}

int smx_bshard_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                         int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                         double* send, double* recv, int32_t nranks, void* comm, int32_t* log,
                         double* xhist, int64_t log_cap, void* stream, float* host_sweep_ms,
                         float* host_total_ms) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || buf0 == buf1 || !ctl || !send ||
        !recv || nranks < 1 || !comm || k < 1 || !host_sweep_ms || !host_total_ms)
        return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    const int nb = (k + pivots - 1) / pivots;
    hipEvent_t* ev = nullptr;
    if (timer_events((size_t)(2 * nb + 2), &ev)) return (int)hipErrorOutOfMemory;
    (void)hipEventRecord(ev[2 * nb], st);
    int err = launch_block_chain(buf0, buf1, *shape, parity & 1, k, pivots, ctl,
                                 static_cast<char*>(blk), log, xhist, log_cap, st, ev, send,
                                 recv, nranks, reinterpret_cast<ncclComm_t>(comm));
    (void)hipEventRecord(ev[2 * nb + 1], st);
    if (!err) err = (int)hipEventSynchronize(ev[2 * nb + 1]);
    if (!err) {
        for (int b = 0; b < nb; ++b)
            (void)hipEventElapsedTime(&host_sweep_ms[b], ev[2 * b], ev[2 * b + 1]);
        (void)hipEventElapsedTime(host_total_ms, ev[2 * nb], ev[2 * nb + 1]);
    }
    return err;
}

int smx_bshard_prime(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                     void* blk, int64_t blk_bytes, void* stream) {
    if (!bshard_args_ok(shape, 1, blk, blk_bytes) || !ctl) return (int)hipErrorInvalidValue;
    return launch_blk_prime(true, T, *shape, parity & 1, parity & 1, ctl,
                            blk_ptrs(*shape, static_cast<char*>(blk)), S(stream));
}

int smx_bshard_pack(const double* T, const smx_shape* shape, int32_t step, int32_t pivots,
                    int32_t block, const smx_ctl* ctl, void* blk, int64_t blk_bytes, double* send,
                    void* stream) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || !ctl || !send || step < 0 ||
        step >= pivots || block < 0)
        return (int)hipErrorInvalidValue;
    return launch_bsh_pack(step, T, *shape, pivots, block, ctl,
                           blk_ptrs(*shape, static_cast<char*>(blk)), send, S(stream));
}

int smx_bshard_step(const double* T, const smx_shape* shape, int32_t step, int32_t pivots,
                    int32_t parity, int32_t block, const double* recv, int32_t nranks,
                    smx_ctl* ctl, void* blk, int64_t blk_bytes, int32_t* log, double* xhist,
                    int64_t log_cap, void* stream) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || !ctl || !recv || nranks < 1 ||
        step < 1 || step > pivots || block < 0)
        return (int)hipErrorInvalidValue;
    return launch_blk_step(true, step, T, *shape, pivots, parity & 1, block, ctl,
                           blk_ptrs(*shape, static_cast<char*>(blk)), recv, nranks, log, xhist,
                           log_cap, S(stream));
}

int smx_tune_shard_xchg(int32_t mode) {
    const int prev = g_shard_xchg;
    if (mode >= -1 && mode <= 1) g_shard_xchg = mode;
    return prev;
}

int smx_bshard_pick(const double* hdrs, const smx_shape* shape, int32_t nranks, int32_t rank,
                    const double* send, double* row, void* stream) {
    if (!shape_ok(shape) || !hdrs || !send || !row || nranks < 1 || rank < 0 || rank >= nranks)
        return (int)hipErrorInvalidValue;
    return launch_bsh_pick(hdrs, *shape, nranks, rank, send, row, S(stream));
}

int smx_bshard_step_light(const double* T, const smx_shape* shape, int32_t step, int32_t pivots,
                          int32_t parity, int32_t block, const double* hdrs, const double* row,
                          int32_t nranks, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                          int32_t* log, double* xhist, int64_t log_cap, void* stream) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || !ctl || !hdrs || !row || nranks < 1 ||
        step < 1 || step > pivots || block < 0)
        return (int)hipErrorInvalidValue;
    return launch_blk_step(true, step, T, *shape, pivots, parity & 1, block, ctl,
                           blk_ptrs(*shape, static_cast<char*>(blk)), hdrs, nranks, log, xhist,
                           log_cap, S(stream), row, SMX_SHARD_HDR);
}

int smx_bshard_sweep(double* Tin, double* Tother, const smx_shape* shape, int32_t pivots,
                     void* blk, int64_t blk_bytes, void* stream) {
    if (!bshard_args_ok(shape, pivots, blk, blk_bytes) || Tin == Tother)
        return (int)hipErrorInvalidValue;
    const BlkPtrs bp = blk_ptrs(*shape, static_cast<char*>(blk));
    return launch_block_sweep(true, Tin, Tother, *shape, pivots, static_cast<char*>(blk), bp.L,
                              S(stream));
}

int smx_bshard_publish(const smx_shape* shape, int32_t parity, int32_t block, smx_ctl* ctl,
                       void* blk, int64_t blk_bytes, void* stream) {
    if (!bshard_args_ok(shape, 1, blk, blk_bytes) || !ctl || block < 0)
        return (int)hipErrorInvalidValue;
    return launch_blk_publish(true, *shape, parity & 1, block, ctl,
                              blk_ptrs(*shape, static_cast<char*>(blk)), S(stream));
}

// Copy exchange of ranks that share one device (SimplexMethod(..., devices=[0] * N)): ONE launch
// on ranks[0]'s stream copies every rank's send slot into every rank's recv (grid.y = dst * N +
// src), instead of N^2 hipMemcpyAsync calls and N^2 event waits per pivot from the host
// (tools/mshard_host_cost.py: 418 us of host enqueue per pivot at 8 ranks, profiles/r04h/).
constexpr int kMsMaxRanks = 16;
struct MsSlots {
    const double* src[kMsMaxRanks];
    double* dst[kMsMaxRanks];
};
__global__ __launch_bounds__(256) void k_mshard_gather(MsSlots s, int nranks, int64_t slot) {
    const int q = blockIdx.y / nranks, o = blockIdx.y % nranks;
    const double* src = s.src[o];
    double* dst = s.dst[q] + (int64_t)o * slot;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < slot; j += (int64_t)gridDim.x * 256)
        dst[j] = src[j];
}

// ---- single-process multi-device row sharding (smx_mshard_*) --------------------------------
int smx_mshard_comms(void** comms_out, int32_t nranks, const int32_t* devices) {
    if (!comms_out || !devices || nranks < 1) return (int)hipErrorInvalidValue;
    ncclComm_t* c = new ncclComm_t[nranks];
    const ncclResult_t r = ncclCommInitAll(c, nranks, devices);
    if (r == ncclSuccess)
        for (int i = 0; i < nranks; ++i) comms_out[i] = c[i];
    delete[] c;
    return r == ncclSuccess ? 0 : -1000 - (int)r;
}

}  // extern "C"

namespace {
bool mshard_args_ok(const smx_rank* ranks, int32_t nranks, int32_t k, int32_t pivots,
                    int32_t exchange) {
    if (!ranks || nranks < 1 || k < 0 || pivots < 1 || pivots > kBlkMax ||
        (exchange != SMX_XCHG_RCCL && exchange != SMX_XCHG_COPY))
        return false;
    for (int q = 0; q < nranks; ++q) {
        const smx_rank& r = ranks[q];
        if (!bshard_args_ok(&r.shape, pivots, r.blk, r.blk_bytes) || !r.buf0 || !r.buf1 ||
            r.buf0 == r.buf1 || !r.ctl || !r.send || !r.recv || r.shape.ld != ranks[0].shape.ld ||
            (exchange == SMX_XCHG_RCCL && !r.comm))
            return false;
    }
    return true;
}

// Every launch of k chained pivots on every rank, enqueued from this thread (smx_mshard_run)
// ev_ext: the copy exchange's 2 * nranks events created by the caller, or NULL: created and
// destroyed here.
// pool (graph capture, one-device copy exchange only): every event record of the exchange takes
// a fresh event from it, never re-recording one inside the capture (round 4's capture re-recorded
// each rank's events once per pivot and crashed the host process in smx_mshard_graph_create,
// gpurun_out r04g / r04h); `pool_n` events, created by the caller on ranks[0]'s device.
int mshard_enqueue(const smx_rank* ranks, int32_t nranks, int32_t parity, int32_t k,
                   int32_t pivots, int32_t exchange, hipEvent_t* ev_ext = nullptr,
                   hipEvent_t* pool = nullptr, int pool_n = 0) {
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    const size_t slot = (size_t)SMX_SHARD_HDR + 2 * (size_t)ranks[0].shape.ld;
    BlkPtrs* bp = new BlkPtrs[nranks];
    // copy exchange: packed / received
    hipEvent_t* ev = ev_ext ? ev_ext : new hipEvent_t[2 * (size_t)nranks]();
    int err = 0;
    for (int q = 0; q < nranks && !err; ++q) {
        bp[q] = blk_ptrs(ranks[q].shape, static_cast<char*>(ranks[q].blk));
        if (exchange == SMX_XCHG_COPY && !ev_ext) {
            err = (int)hipSetDevice(ranks[q].device);
            if (!err) err = (int)hipEventCreateWithFlags(&ev[2 * q], hipEventDisableTiming);
            if (!err) err = (int)hipEventCreateWithFlags(&ev[2 * q + 1], hipEventDisableTiming);
        }
    }
    auto on = [&](int q) -> hipStream_t {
        (void)hipSetDevice(ranks[q].device);
        return S(ranks[q].stream);
    };
    auto buf = [&](int q, int p) { return p ? ranks[q].buf1 : ranks[q].buf0; };
    // light exchange (RCCL only; the copy exchange always moves whole slots)
    const bool light = exchange == SMX_XCHG_RCCL && xchg_light(nranks);
    // copy exchange on one device: one gather launch on ranks[0]'s stream (k_mshard_gather)
    bool one_dev = exchange == SMX_XCHG_COPY && nranks <= kMsMaxRanks;
    for (int q = 1; q < nranks; ++q) one_dev = one_dev && ranks[q].device == ranks[0].device;
    MsSlots ms{};
    for (int q = 0; q < nranks && one_dev; ++q) {
        ms.src[q] = ranks[q].send;
        ms.dst[q] = ranks[q].recv;
    }
    auto xrow = [&](int q) { return ranks[q].recv + (size_t)nranks * SMX_SHARD_HDR; };
    for (int q = 0; q < nranks && !err; ++q) {
        hipStream_t st = on(q);
        err = launch_blk_prime(true, buf(q, parity & 1), ranks[q].shape, parity & 1, parity & 1,
                               ranks[q].ctl, bp[q], st);
    }
    int p = parity & 1, done = 0, bn = 0;
    while (!err && done < k) {
        const int Pb = block_size(k, pivots, bn);
        for (int l = 1; l <= Pb && !err; ++l) {
            for (int q = 0; q < nranks && !err; ++q)
                err = launch_bsh_pack(l - 1, buf(q, p), ranks[q].shape, Pb, bn, ranks[q].ctl,
                                      bp[q], ranks[q].send, on(q));
            if (err) break;
            if (exchange == SMX_XCHG_RCCL && light) {
                // grouped header all-gather, every rank's pick, grouped max all-reduce of a row
                ncclResult_t rr = ncclGroupStart();
                for (int q = 0; q < nranks && rr == ncclSuccess; ++q)
                    rr = ncclAllGather(ranks[q].send, ranks[q].recv, SMX_SHARD_HDR, ncclFloat64,
                                       reinterpret_cast<ncclComm_t>(ranks[q].comm), on(q));
                ncclResult_t re = ncclGroupEnd();
                if (rr == ncclSuccess) rr = re;
                for (int q = 0; q < nranks && rr == ncclSuccess && !err; ++q)
                    err = launch_bsh_pick(ranks[q].recv, ranks[q].shape, nranks, q, ranks[q].send,
                                          xrow(q), on(q));
                if (rr == ncclSuccess && !err) {
                    rr = ncclGroupStart();
                    for (int q = 0; q < nranks && rr == ncclSuccess; ++q)
                        rr = ncclAllReduce(xrow(q), xrow(q), (size_t)ranks[q].shape.ld, ncclInt64,
                                           ncclMax, reinterpret_cast<ncclComm_t>(ranks[q].comm),
                                           on(q));
                    re = ncclGroupEnd();
                    if (rr == ncclSuccess) rr = re;
                }
                if (rr != ncclSuccess) err = -1000 - (int)rr;
            } else if (exchange == SMX_XCHG_RCCL) {   // one grouped all-gather of the slots
                ncclResult_t rr = ncclGroupStart();
                for (int q = 0; q < nranks && rr == ncclSuccess; ++q)
                    rr = ncclAllGather(ranks[q].send, ranks[q].recv, slot, ncclFloat64,
                                       reinterpret_cast<ncclComm_t>(ranks[q].comm), on(q));
                const ncclResult_t re = ncclGroupEnd();
                if (rr == ncclSuccess) rr = re;
                if (rr != ncclSuccess) err = -1000 - (int)rr;
            } else if (one_dev) {
                // ranks[0]'s stream waits for every pack, gathers every slot into every recv in
                // one launch, and every other rank waits for that launch: 3N - 1 host calls per
                // pivot.  A rank's next pack follows its wait, so no slot is overwritten early.
                hipStream_t st0 = on(0);
                auto pick = [&](hipEvent_t own) -> hipEvent_t {   // fresh event when capturing
                    if (!pool) return own;
                    if (pool_n <= 0) {
                        err = (int)hipErrorInvalidValue;
                        return own;
                    }
                    --pool_n;
                    return *pool++;
                };
                for (int q = 1; q < nranks && !err; ++q) {
                    const hipEvent_t e = pick(ev[2 * q]);
                    if (!err) err = (int)hipEventRecord(e, on(q));
                    if (!err) err = (int)hipStreamWaitEvent(st0, e, 0);
                }
                const int gx = (int)((slot + 256 * 8 - 1) / (256 * 8));
                if (!err) {
                    (void)hipSetDevice(ranks[0].device);
                    hipLaunchKernelGGL(k_mshard_gather, dim3(gx, nranks * nranks), dim3(256), 0,
                                       st0, ms, nranks, (int64_t)slot);
                    err = (int)hipGetLastError();
                }
                const hipEvent_t eg = err ? ev[1] : pick(ev[1]);
                if (!err) err = (int)hipEventRecord(eg, st0);
                for (int q = 1; q < nranks && !err; ++q)
                    err = (int)hipStreamWaitEvent(on(q), eg, 0);
            } else {   // every rank copies every send slot into its recv, ordered by events
                for (int q = 0; q < nranks && !err; ++q)
                    err = (int)hipEventRecord(ev[2 * q], on(q));
                for (int q = 0; q < nranks && !err; ++q) {
                    hipStream_t st = on(q);
                    for (int o = 0; o < nranks && !err; ++o)
                        err = (int)hipStreamWaitEvent(st, ev[2 * o], 0);
                    for (int o = 0; o < nranks && !err; ++o)
                        err = (int)hipMemcpyAsync(ranks[q].recv + (size_t)o * slot, ranks[o].send,
                                                  slot * sizeof(double), hipMemcpyDefault, st);
                    if (!err) err = (int)hipEventRecord(ev[2 * q + 1], st);
                }
                // no rank packs into its send slot again before every rank has copied it
                for (int q = 0; q < nranks && !err; ++q) {
                    hipStream_t st = on(q);
                    for (int o = 0; o < nranks && !err; ++o)
                        err = (int)hipStreamWaitEvent(st, ev[2 * o + 1], 0);
                }
            }
            for (int q = 0; q < nranks && !err; ++q)
                err = launch_blk_step(true, l, buf(q, p), ranks[q].shape, Pb, p, bn,
                                      ranks[q].ctl, bp[q], ranks[q].recv, nranks, ranks[q].log,
                                      ranks[q].xhist, ranks[q].log_cap, on(q),
                                      light ? xrow(q) : nullptr,
                                      light ? (int64_t)SMX_SHARD_HDR : 0);
        }
        for (int q = 0; q < nranks && !err; ++q)
            err = launch_block_sweep(true, buf(q, p), buf(q, p ^ 1), ranks[q].shape, Pb,
                                     static_cast<char*>(ranks[q].blk), bp[q].L, on(q), 0, 0, p);
        p = (p + Pb) & 1;
        done += Pb;
        ++bn;
    }
    for (int q = 0; q < nranks && !err; ++q)
        err = launch_blk_publish(true, ranks[q].shape, p, bn, ranks[q].ctl, bp[q], on(q));
    if (!ev_ext) {
        for (int q = 0; q < 2 * nranks; ++q)
            if (ev[q]) {
                (void)hipSetDevice(ranks[q / 2].device);
                (void)hipEventDestroy(ev[q]);   // released once its last record has completed
            }
        delete[] ev;
    }
    delete[] bp;
    (void)hipSetDevice(dev0);
    return err;
}
}  // namespace

extern "C" {

int smx_mshard_run(const smx_rank* ranks, int32_t nranks, int32_t parity, int32_t k,
                   int32_t pivots, int32_t exchange) {
    if (!mshard_args_ok(ranks, nranks, k, pivots, exchange)) return (int)hipErrorInvalidValue;
    if (k == 0) return 0;
    if (exchange == SMX_XCHG_RCCL) {
        // One host thread per device, each enqueuing its rank's whole chain on its own
        // communicator -- the multi-process protocol (launch_block_chain), no cross-device
        // group call: one thread driving N devices spends ~5 us of host time per launch, so at
        // 8 ranks its per-pivot enqueue (~3N launches) outgrows a rank's ~28-34 us of device
        // work (tools/mshard_host_cost.py, profiles/r04h/, r04j/); per thread it is 3 launches.
        std::vector<int> errs((size_t)nranks, 0);
        std::vector<std::thread> th;
        th.reserve((size_t)nranks);
        for (int q = 0; q < nranks; ++q)
            th.emplace_back([&, q] {
                const smx_rank& R = ranks[q];
                int e = (int)hipSetDevice(R.device);
                if (!e)
                    e = launch_block_chain(R.buf0, R.buf1, R.shape, parity & 1, k, pivots, R.ctl,
                                           static_cast<char*>(R.blk), R.log, R.xhist, R.log_cap,
                                           S(R.stream), nullptr, R.send, R.recv, nranks,
                                           reinterpret_cast<ncclComm_t>(R.comm));
                errs[(size_t)q] = e;
            });
        for (auto& t : th) t.join();
        int first = 0, first_rank = -1;
        for (int q = 0; q < nranks; ++q) {
            const int e = errs[(size_t)q];
            if (!e) continue;
            // every failing rank's own code, before the abort hides it behind one status
            fprintf(stderr, "smx_mshard_run: rank %d (device %d) failed: %s %d\n", q,
                    ranks[q].device, e <= -1000 ? "RCCL" : "hipError", e <= -1000 ? -1000 - e : e);
            if (!first) {
                first = e;
                first_rank = q;
            }
        }
        {
            std::lock_guard<std::mutex> lock(g_cache_mu);
            g_mshard_err = first;
            g_mshard_err_rank = first_rank;
        }
        if (first) {
            // a rank that failed mid-chain leaves the others' enqueued collectives waiting for
            // it forever: abort every communicator (the caller must not destroy them afterwards,
            // SMX_ERR_COMMS_ABORTED; smx_mshard_last_error returns the first rank's own code)
            for (int q = 0; q < nranks; ++q)
                (void)ncclCommAbort(reinterpret_cast<ncclComm_t>(ranks[q].comm));
            return SMX_ERR_COMMS_ABORTED;
        }
        return 0;
    }
    return mshard_enqueue(ranks, nranks, parity, k, pivots, exchange);
}

int smx_mshard_last_error(int32_t* rank_out) {
    std::lock_guard<std::mutex> lock(g_cache_mu);
    if (rank_out) *rank_out = g_mshard_err_rank;
    return g_mshard_err;
}

int smx_mshard_graph_create(const smx_rank* ranks, int32_t nranks, int32_t parity, int32_t k,
                            int32_t pivots, void** graph_out) {
    if (!mshard_args_ok(ranks, nranks, k, pivots, SMX_XCHG_COPY) || k < 1 || !graph_out ||
        nranks > kMsMaxRanks)
        return (int)hipErrorInvalidValue;
    for (int q = 1; q < nranks; ++q)
        if (ranks[q].device != ranks[0].device) return (int)hipErrorInvalidValue;
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    hipStream_t st0 = S(ranks[0].stream);
    // every event the capture records, created before it and destroyed after it, each recorded
    // exactly once: [0] the fork, [1 .. nranks) the joins, then nranks per pivot (the exchange)
    const int pool_n = nranks * k;
    const int nev = nranks + pool_n;
    std::vector<hipEvent_t> ev((size_t)nev, nullptr);
    std::vector<hipEvent_t> xev(2 * (size_t)nranks, nullptr);   // unused in pool mode
    int err = (int)hipSetDevice(ranks[0].device);
    for (int q = 0; q < nev && !err; ++q)
        err = (int)hipEventCreateWithFlags(&ev[(size_t)q], hipEventDisableTiming);
    Graph* g = new Graph();
    if (!err) err = (int)hipStreamBeginCapture(st0, hipStreamCaptureModeThreadLocal);
    if (!err) {
        int lerr = (int)hipEventRecord(ev[0], st0);   // fork: every rank's stream joins
        for (int q = 1; q < nranks && !lerr; ++q)
            lerr = (int)hipStreamWaitEvent(S(ranks[q].stream), ev[0], 0);
        if (!lerr)
            lerr = mshard_enqueue(ranks, nranks, parity, k, pivots, SMX_XCHG_COPY, xev.data(),
                                  ev.data() + nranks, pool_n);
        for (int q = 1; q < nranks && !lerr; ++q) {   // join back into ranks[0]'s stream
            lerr = (int)hipEventRecord(ev[(size_t)q], S(ranks[q].stream));
            if (!lerr) lerr = (int)hipStreamWaitEvent(st0, ev[(size_t)q], 0);
        }
        (void)hipSetDevice(ranks[0].device);
        const hipError_t e2 = hipStreamEndCapture(st0, &g->graph);
        err = lerr ? lerr : (int)e2;
    }
    if (!err) err = (int)hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    (void)hipSetDevice(dev0);
    if (err) {
        if (g->exec) (void)hipGraphExecDestroy(g->exec);
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return err;
    }
    *graph_out = g;
    return 0;
}

int smx_int_first_fix(const double* T0, double* T1, int64_t ld, int32_t rows, int32_t cols,
                      int32_t r_local, int32_t c, const double* prow, const uint8_t* mask,
                      int64_t ldm, const uint8_t* maskr, void* stream) {
    if (!int_first_args_ok(T0, T1, ld, rows, cols, r_local, c, prow, mask, ldm))
        return (int)hipErrorInvalidValue;
    const int grid = rows < 4096 ? rows : 4096;
    hipLaunchKernelGGL(k_int_first_fix, dim3(grid), dim3(256), 0, S(stream), T0, T1, ld, rows,
                       cols, r_local, c, prow, mask, ldm, maskr);
    return (int)hipGetLastError();
}

int smx_host_int_first_fix(const double* T0, double* T1, int64_t ld, int32_t rows, int32_t cols,
                           int32_t r_local, int32_t c, const double* prow, const uint8_t* mask,
                           int64_t ldm, const uint8_t* maskr) {
    if (!int_first_args_ok(T0, T1, ld, rows, cols, r_local, c, prow, mask, ldm)) return -1;
    host_int_first_fix(T0, T1, ld, rows, cols, r_local, c, prow, mask, ldm, maskr);
    return 0;
}

}  // extern "C"
