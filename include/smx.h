/*
 * smx.h -- C ABI of the MI355X simplex pivot engine (libsmx.so, gfx950).
 *
 * Drop-in boundary for the hot path of jqnfxa/Simplex-Method-Solver, src/simplex.py:
 *   smx_reset      <- the tableau set-up of SimplexMethod.__init__ (simplex.py:25-39): primes
 *                     the device control block with the first-negative "-b" row and the first
 *                     negative f-row column of a freshly uploaded tableau
 *   smx_select     <- SimplexMethod.pick_element (simplex.py:70-141), per-workgroup partials
 *   smx_finalize   <- the return/raise of pick_element (simplex.py:89, 91, 101-103, 138-141)
 *   smx_update     <- SimplexMethod.recalculate_matrix (simplex.py:143-177), steps 1-4,
 *                     out of place like the reference's deepcopy (simplex.py:149, 177)
 *   smx_run        <- the pivot loop of SimplexMethod.get_solution (simplex.py:184-198),
 *                     k chained select+update pairs, no host synchronisation
 *   smx_graph_*    <- the same loop captured once as a hipGraph and replayed
 *   smx_shard_*    <- row-sharded variant for 1 process per GPU (exchange done by the caller's
 *                     RCCL all-gather between smx_shard_begin and smx_shard_finish)
 * The reference is pure Python; it has no FFI of its own.  The Python binding a maintainer would
 * add is in INTEGRATION.md (ctypes), and simplex-method-solver_amd/simplex_mi355x/_lib.py is it.
 *
 * Conventions
 *   - All pointers are DEVICE pointers owned by the caller (torch tensors in the Python host),
 *     except where a name says host.  Every call is asynchronous on `stream` (a hipStream_t).
 *   - Tableau: row-major fp64, R = n+1 rows (n constraint rows, then the f-row), C = m+1 used
 *     columns (m variables, then the "-b" column), leading dimension `ld` (a multiple of 4 doubles,
 *     >= C rounded up to 4).  f-row entries j >= flen are padding: computed, never read by a selection.
 *   - Two tableau buffers ping-pong: step s reads buf[s & 1] and writes buf[(s + 1) & 1];
 *     `parity` = s & 1 selects the control-block slots of that step.
 *   - Return value: 0 on success, otherwise a hipError_t (no exceptions cross this ABI).
 *     The pivot outcome is device-side in smx_ctl.sel_status (SMX_* codes below), mapped by the
 *     host to the reference's ValueError strings (simplex.py:89, 139).
 */
#ifndef SMX_H
#define SMX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* outcome codes (also used by oracle/) */
#define SMX_PIVOT 0         /* (r, c) selected; simplex.py:91, 141                          */
#define SMX_OPTIMUM 1       /* no negative f-row coefficient; simplex.py:101-103             */
#define SMX_INCORRECT 2     /* ValueError("incorrect system"); simplex.py:88-89              */
#define SMX_NOT_CONVERGE 3  /* ValueError("simplex method does not converge"); :138-139      */
#define SMX_FSHORT 4        /* len(function) < m and the f-row scan ran off its end (IndexError) */
#define SMX_IDLE 5          /* no selection made yet                                         */

#define SMX_NONE 0x7f7f7f7f /* "no index" sentinel (memset byte 0x7f)                        */
#define SMX_ABSENT ((int32_t)0x80000000) /* label position code: label does not exist      */

/* Device control block (caller allocates sizeof(smx_ctl) bytes of device memory).
 * Fields indexed [parity] are double-buffered: step s reads slot s&1 and its update kernel writes
 * slot (s+1)&1, so no kernel ever reads a word another block of the same launch is writing. */
typedef struct smx_ctl {
    int32_t negb[2];    /* per parity slot: first row i < n with T[i][m] < 0 (global index)  */
    int32_t negf[2];    /* per parity slot: first j < min(m, flen) with f[j] < 0             */
    int32_t term;       /* != 0: a terminal outcome was reached; chained kernels do nothing  */
    int32_t sel_status; /* last selection: SMX_* code                                         */
    int32_t sel_r;      /* last selection: pivot row (global)                                 */
    int32_t sel_c;      /* last selection: pivot column                                       */
    double sel_e;       /* last selection: pivot element T[r][c]                              */
    int64_t npivots;    /* pivots applied since smx_reset(..., clear_count=1)                 */
    int32_t sel_owner;  /* sharded: rank whose candidate row is the pivot row                 */
    int32_t nla;        /* sharded fused update: look-ahead workgroups done (0 between launches) */
    int64_t shard_off;  /* sharded: offset (doubles) of the pivot row in the receive buffer   */
    int32_t xpos[2][2]; /* [parity][x1, x2]: position code of labels 'x1', 'x2' (simplex.py:
                           58-59): p >= 0 row p (basic), -(j+1) column j, SMX_ABSENT none      */
    int64_t npiv[2];    /* [parity]: pivot index of the step (history ring position)          */
    int32_t dec[2][4];  /* dec[0][0]: smx_resident_run hand-off timeout flag; rest reserved   */
} smx_ctl; /* 128 bytes */

/* One per select workgroup (caller allocates 2 * nparts * sizeof(smx_part) bytes: the fused
 * chain double-buffers them by parity; the unfused calls use the first nparts). */
typedef struct smx_part {
    int32_t p1col;    /* phase 1: first column j with T[r][j] > 0 in this workgroup's slice  */
    int32_t first;    /* phase 2: first row with T[i][c] != 0 (its ratio may be NaN)         */
    double first_v;   /* ratio T[first][m] / T[first][c]                                     */
    int32_t best_cls; /* best non-NaN candidate: 0 (v<0), 1 (v==0), 2 (v>0), 3 none          */
    int32_t best_i;
    double best_v;
} smx_part; /* 32 bytes */

/* Shape of one (possibly sharded) tableau. */
typedef struct smx_shape {
    int64_t ld;     /* leading dimension in doubles                                         */
    int32_t rows;   /* local constraint rows (n when unsharded)                              */
    int32_t n;      /* global constraint rows                                                */
    int32_t m;      /* variables                                                             */
    int32_t flen;   /* len(function) of the reference's f-row                                */
    int32_t row0;   /* global index of local row 0 (0 when unsharded)                        */
    int32_t nparts; /* select workgroups (smx_part records)                                  */
} smx_shape;

/* Create (once, reused by every *_run_timed call) at least `events` timing events, so that no
 * event is created or destroyed inside a caller's timed region; the timed calls grow the pool
 * themselves when it is too small. */
int smx_timer_reserve(int32_t events);

/* Library/ABI identification; returns the number of kernels built into the library. */
int smx_version(char* buf, int len);
/* Recommended number of select partials for a shape (host-only helper). */
int smx_nparts_for(int32_t rows, int32_t m);

/* Tuning of the update kernel (process-wide): variant index (16-B loads in flight per lane,
 * non-temporal stores; see smx_tune_get) and resident blocks per CU (0 = occupancy API).
 * -1 keeps the current value; variant -2 restores the automatic choice (the default: plain
 * loads for a tableau buffer of at most 16 MiB, which stays cache-resident, non-temporal
 * loads above).  smx_tune_get reports variant -1 while automatic. */
int smx_tune_set(int32_t variant, int32_t blocks_per_cu);
int smx_tune_get(int32_t* variant, int32_t* blocks_per_cu, int32_t* nvariants,
                 int32_t* units_in_flight, int32_t* vec, int32_t* nt);

/* Scan a freshly uploaded tableau into ctl slot `parity`; clears term, sets sel_status = IDLE,
 * zeroes npivots when clear_count != 0, and places labels x1/x2 at columns 0/1 (simplex.py:30). */
int smx_reset(const double* T, const smx_shape* shape, int32_t parity, int32_t clear_count,
              smx_ctl* ctl, void* stream);

/* Set the x1/x2 position codes of slot `parity` (after the host re-labelled a tableau). */
int smx_set_xpos(smx_ctl* ctl, int32_t parity, int32_t x1code, int32_t x2code, void* stream);

/* pick_element, part 1: per-workgroup partials of the selection for the tableau T. */
int smx_select(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
               smx_part* parts, void* stream);

/* Fused chain (default for smx_run / smx_run_timed / smx_graph_*; `on`: 0 off, 1 on, 2 on plus
 * the overlapped form of smx_shard_run): ONE kernel per pivot --
 * the update of step k, whose first nparts workgroups also compute step k+1's select inputs
 * (first negative new "-b" row, entering column, ratio-test partials) from T_k with the update's
 * own arithmetic (bit-identical); a chain is primed by one small kernel and ends with a one-wave
 * publish of ctl->negb.  Records are double-buffered: `parts` must hold 2 * nparts of them.
 * smx_tune_fused(0) restores the select + update pair; returns the previous setting. */
int smx_tune_fused(int32_t on);
/* Smallest local tableau buffer (bytes) for which the sharded fused update packs the next step
 * itself (smx_shard_folds_pack; default INT64_MAX = never, it measured slower); -1 keeps it;
 * returns the previous value. */
int64_t smx_tune_fold(int64_t min_bytes);

/* pick_element, part 2: reduce the partials into ctl->sel_* (does not set term, logs nothing). */
int smx_finalize(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                 const smx_part* parts, void* stream);

/* recalculate_matrix: reduce the partials, record the outcome in ctl (sel_*, term, npivots,
 * log[k % log_cap] = (r, c)), and on SMX_PIVOT write the pivoted tableau to Tout.  Also primes
 * ctl slot parity^1 for the next step (fused first-negative scans) and, when xhist != NULL,
 * records xhist[k % log_cap] = (x1, x2) of the new tableau (find_optimum, simplex.py:51-68;
 * 0.0 for a non-basic label) -- the device-resident history of get_solution (:197-198). */
int smx_update(const double* Tin, double* Tout, const smx_shape* shape, int32_t parity,
               smx_ctl* ctl, const smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
               void* stream);

/* k pivots (select + update each), buffers buf0/buf1, first step's parity `parity`. */
int smx_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
            smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
            void* stream);

/* The same k-pivot chain captured as a hipGraph (opaque handle); replay with smx_graph_launch. */
int smx_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                     int32_t k, smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist,
                     int64_t log_cap, void* stream, void** graph_out);
int smx_graph_launch(void* graph, void* stream);
int smx_graph_destroy(void* graph);

/* smx_run with HIP events recorded on `stream` around every update kernel; synchronises, then
 * writes each update kernel's duration (ms) to host_update_ms[0..k-1] and the whole chain's
 * device time (first select start -> last update end) to *host_total_ms. */
int smx_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  smx_ctl* ctl, smx_part* parts, int32_t* log, double* xhist, int64_t log_cap,
                  void* stream, float* host_update_ms, float* host_total_ms);

/* Forced-pivot microbenchmark of the update kernel alone: applies pivot (r, c) from Tin to Tout
 * without any selection (used to measure the kernel against the HBM roofline). */
int smx_update_forced(const double* Tin, double* Tout, const smx_shape* shape, int32_t r,
                      int32_t c, void* stream);

/* ---- batched small LPs (one wavefront per LP; the UI's workload) --------------------------
 * B problems, each packed as rows 0..n_b (f-row = row n_b) of a Rmax x ldb fp64 block (Rmax <=
 * 64, ldb <= 64, ldb >= m_b + 1); dims = int32 [B][3] = (n, m, len(function)).  Runs the whole
 * get_solution loop (simplex.py:184-198) per problem, at most max_pivots pivots.  Outputs per
 * problem: final table (out, same layout), status (SMX_* ; SMX_PIVOT = cap reached), pivot count,
 * rc = int32 [B][max_pivots][2], xv = fp64 [B][max_pivots][2] (x1, x2 after each pivot), and when
 * snaps != NULL the table after each pivot, fp64 [B][max_pivots][Rmax][ldb]. */
int smx_batch_solve(const double* tabs, const int32_t* dims, int32_t B, int32_t Rmax,
                    int32_t ldb, int32_t max_pivots, double* out, int32_t* rc, double* xv,
                    double* snaps, int32_t* status, int32_t* npivots, void* stream);

/* ---- row-sharded engine (one process per GPU; exchange = caller's all-gather) ----------
 * Local tableau: shape->rows constraint rows (global rows row0 .. row0+rows-1) + a replica
 * of the f-row as local row `rows`.  Per pivot:
 *   smx_select(T, shape, parity, ...)             local ratio-test / phase-1 partials
 *   smx_shard_pack(T, ..., send)                  header + candidate rows -> send slot
 *   all_gather(send -> recv[P][slot])             RCCL over xGMI, by the caller
 *   smx_shard_update(Tin, Tout, recv, P, ...)     every block merges the P headers (identical
 *                                                 decision on every rank), then pivots with the
 *                                                 winning row read straight from recv
 * Slot layout (doubles): [SMX_SHARD_HDR header][row A: ld][row B: ld]; header =
 *   {local first-negative-b row | NONE, first ratio candidate | NONE, its ratio, best class,
 *    best row, best ratio, entering column, first positive column of row B (phase 1)}.
 * smx_shard_merge only records the selection in ctl (like smx_finalize). */
#define SMX_SHARD_HDR 8
int smx_shard_pack(const double* T, const smx_shape* shape, int32_t parity, const smx_ctl* ctl,
                   const smx_part* parts, double* send, void* stream);
int smx_shard_merge(const double* recv, int32_t nranks, const smx_shape* shape,
                    int32_t parity, smx_ctl* ctl, int32_t* log, int64_t log_cap, void* stream);
int smx_shard_update(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                     const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                     int64_t log_cap, void* stream);
/* One pivot = smx_shard_begin (select + pack) -> all-gather -> smx_shard_finish (update, with
 * optional hipEvent_t records around it, may be NULL). */
int smx_shard_begin(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                    smx_part* parts, double* send, void* stream);
int smx_shard_finish(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                     const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                     int64_t log_cap, void* ev_before, void* ev_after, void* stream);

/* The same pivot with the fused look-ahead (no select kernel): smx_shard_fused_begin packs the
 * header and candidate rows from this step's look-ahead records (parts slot `parity`, written by
 * smx_shard_fused_prime for the first step of a sequence, by the previous fused finish after
 * that); smx_shard_fused_finish merges, updates and writes the next step's records -- and, when
 * `send` is not NULL and smx_shard_folds_pack(shape) (off by default, see smx_tune_fold),
 * already packs the next step into it: then skip the next begin.  Before switching
 * back to the unfused calls, smx_fused_publish(next parity) restores ctl->negb. */
int smx_shard_folds_pack(const smx_shape* shape);
int smx_shard_fused_prime(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                          smx_part* parts, void* stream);
int smx_shard_fused_begin(const double* T, const smx_shape* shape, int32_t parity,
                          const smx_ctl* ctl, const smx_part* parts, double* send, void* stream);
int smx_shard_fused_finish(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                           const smx_shape* shape, int32_t parity, smx_ctl* ctl, smx_part* parts,
                           double* send, int32_t* log, int64_t log_cap, void* ev_before,
                           void* ev_after, void* stream);
int smx_fused_publish(const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                      const smx_part* parts, void* stream);
/* Streaming copy of `ndoubles` (even) doubles src -> dst, for measuring the box's read+write
 * ceiling beside the update (bench.py): variant 0 = 4 x 16-B loads in flight per lane, 256
 * threads x 1 block per CU; variant 1 = 1 load, 1024 threads x 1 block per CU. */
int smx_copy_probe(const double* src, double* dst, int64_t ndoubles, int32_t variant,
                   void* stream);

/* The two halves of a step of the overlapped chain (smx_shard_run's default form), for callers
 * that drive the exchange themselves: after step k's all-gather into `recv`,
 * smx_shard_ahead computes step k+1's records (parts slot parity^1) and packs step k+1's header
 * and candidate rows into `send` from T_k (it may run concurrently with the sweep, on another
 * stream); smx_shard_sweep is step k's update.  Start a sequence with smx_shard_fused_prime +
 * smx_shard_fused_begin. */
int smx_shard_ahead(const double* T, const smx_shape* shape, int32_t parity, const double* recv,
                    int32_t nranks, smx_ctl* ctl, smx_part* parts, double* send, void* stream);
int smx_shard_sweep(const double* Tin, double* Tout, const double* recv, int32_t nranks,
                    const smx_shape* shape, int32_t parity, smx_ctl* ctl, int32_t* log,
                    int64_t log_cap, void* stream);

/* Native RCCL driver (one communicator per rank; the unique id is created on rank 0 and
 * shipped to the others by any bootstrap, e.g. torch.distributed.broadcast_object_list).
 * smx_shard_run = k x {select, pack, ncclAllGather on `stream`, update}; with smx_tune_fused(1)
 * (the default) prime + pack + k x {ncclAllGather, fused update that also packs the next step}
 * + publish; with
 * smx_tune_fused(2) the overlapped form: the update sweeps on `stream` while an internal exchange
 * stream computes the next step's look-ahead records, header and candidate rows from T_k and
 * gathers them (two events per step).  No host synchronisation.  `recv` must hold
 * 2 * nranks * (SMX_SHARD_HDR + 2 * ld) doubles (the second half is used by the overlapped form).  RCCL failures are returned as -1000 - ncclResult_t. */
int smx_comm_unique_id(void* id_out /* 128 bytes */);
int smx_comm_init(void** comm_out, int32_t nranks, const void* id, int32_t rank);
int smx_comm_destroy(void* comm);
/* What RCCL formed: the communicator's rank count (ncclCommCount), this rank (ncclCommUserRank)
 * and its device (ncclCommCuDevice) -- the multi-GPU bench line records them for every rank. */
int smx_comm_info(void* comm, int32_t* count, int32_t* rank, int32_t* device);
int smx_shard_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  smx_ctl* ctl, smx_part* parts, double* send, double* recv, int32_t nranks,
                  void* comm, int32_t* log, int64_t log_cap, void* stream);
int smx_shard_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                        int32_t k, smx_ctl* ctl, smx_part* parts, double* send, double* recv,
                        int32_t nranks, void* comm, int32_t* log, int64_t log_cap, void* stream,
                        float* host_update_ms, float* host_total_ms);

/* The resident loop's hand-off spin bound in s_memrealtime ticks (100 MHz; default 2 s) on the
 * current device: ticks >= 0 sets it, < 0 only queries.  Returns the previous bound (-1 on a HIP
 * error).  A spin past the bound latches ctl.dec[0][0] and the grid drains; the Python host then
 * restores the chain's input from its snapshot and reruns the pivots on the launch chain
 * (device.py).  Test support: a bound of 0 forces that path. */
int64_t smx_tune_resident_timeout(int64_t ticks);

/* ---- on-chip resident pivot loop ---------------------------------------------------------
 * The whole get_solution pivot loop (simplex.py:184-198) for k pivots in ONE persistent launch:
 * G workgroups (one per CU, 1024 threads) each hold ceil(n/G) constraint rows and a replica of
 * the f-row in LDS for the whole run and exchange one 32-B record ({payload, tag} granules) +
 * one pivot row per pivot through `xch` (agent-coherent sc1 hand-offs, double-buffered).  Same decisions,
 * same per-element arithmetic, same ctl / log / xhist bookkeeping and ping-pong convention as
 * smx_run: the table after the d pivots actually applied is left in buf[(parity + d) & 1].
 * Only unsharded tableaux whose rows fit in LDS (about R x C <= 2048^2, n <= 65534, C <= 4096)
 * are eligible: smx_resident_bytes returns the `xch` size (0 when not eligible) and optionally
 * plan_out[4] = {workgroups, rows per workgroup, elements per thread, LDS bytes}.
 * `epoch` (1..4095) tags this launch's hand-offs: the caller zeroes `xch` when it allocates it,
 * uses a different epoch for each of 4095 consecutive launches on it, and zeroes it again
 * before an epoch value comes round again; k < 2^20 - 1.  A hand-off that does not complete
 * within 2 s sets ctl->dec[0][0] = 1 and the kernel returns (the table is then undefined).
 * smx_tune_resident: -1 never, 0 automatic, > 0 that many workgroups (<= 256), -2 keeps;
 * returns the previous setting.
 * smx_resident_trace (diagnostic): device buffer of 64 x G x 8 uint64 s_memrealtime stamps for
 * steps from_step .. from_step+63 of later launches (NULL disables). */
int smx_tune_resident(int32_t workgroups);
/* smx_tune_resident_overlap: 2 (default) automatic -- the overlapped resident loop from 768
 * columns: step s's bulk update runs on the non-polling waves during step s+1's hand-off, the
 * records read T_{s+1} on the fly -- 1 always overlapped, 0 the round-3 loop (every step fully
 * updated before the next record); -1 query only; returns the previous setting.  Bit-identical
 * either way. */
int smx_tune_resident_overlap(int32_t on);
int smx_resident_trace(void* trace, int32_t from_step);
int64_t smx_resident_bytes(const smx_shape* shape, int32_t* plan_out);
int smx_resident_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                     int32_t k, smx_ctl* ctl, void* xch, int64_t xch_bytes, int32_t epoch,
                     int32_t* log, double* xhist, int64_t log_cap, void* stream);
/* Self-check of the resident loop's division by the pivot element (the hardware division
 * sequence with its denominator half hoisted, inside an exponent window) against the
 * compiler's x / e on `count` device operand pairs: out[0] = pairs inside the window,
 * out[1] = pairs whose results differ in any bit (device unsigned long long[2]). */
int smx_fastdiv_check(const double* num, const double* den, int64_t count,
                      unsigned long long* out, void* stream);
/* The block sweep's unchecked divisions (smx_block.hpp, kBndSpan: no per-element window when the
 * pivot elements, pivot-row values and multipliers are bounded) against num / den on the domains
 * those bounds guarantee, den in [2^-100, 2^101): out[0] = pairs with num = +0 or |num| in
 * [2^-254, 2^410), out[1] = those the hoisted-reciprocal form gets wrong in any bit; out[2] =
 * pairs with num = +-0 or |num| in [2^-456, 2^410) (zeros allowed), out[3] = those the
 * zero-safe form (fd_zero: the same plus v_div_fixup_f64) gets wrong.  Device unsigned long
 * long[4].  Test support. */
int smx_fastdiv_check_bounded(const double* num, const double* den, int64_t count,
                              unsigned long long* out, void* stream);
/* Diagnostic: the block sweep's units (one row x 128 columns) per path, summed over every
 * k_blk_sweep launch since the last clear -- out[0..count) = fast, zero-extended, window-tracked,
 * window vote failed (-> exact), exact directly, units in chunks not free / not zero-safe, units of
 * rows flagged 0 / 3, inputs out of bounds on a free chunk and flag-1 row, units in chunks whose
 * pivots / pivot-row values fail the bounds, then per wave the shader clock (s_memtime) and the
 * 100 MHz real time (s_memrealtime) over its sweep body -- their ratio is the clock the sweep
 * ran at (smx_block.hpp kPc*).
 * Synchronises the device.  Returns the number of counters, or -hipErrorNotSupported in the
 * product build (the counters exist only in libsmx_diag.so, `make -C csrc diag`). */
int smx_diag_path_counts(int64_t* out, int32_t count, int32_t clear);

/* ---- block pivots: P pivots per HBM sweep ------------------------------------------------
 * k pivots of the get_solution loop (simplex.py:184-198) in blocks of `pivots` (1..24): per block,
 * `pivots` planning steps each decide one pivot (pick_element, simplex.py:70-141) from the block's
 * input table T_k -- every value of T_{k+l} they need is re-derived from T_k with the update's own
 * expression chained l times -- then ONE sweep applies all of them to every element
 * (recalculate_matrix, simplex.py:143-177, the same operations in the same order per element),
 * so a block moves 16*R*C bytes for `pivots` pivots.  Same decisions, bits, ctl / log / xhist
 * bookkeeping and ping-pong convention as smx_run: the table after the d pivots actually applied
 * is in buf[(parity + d) & 1] (the sweep works in place when a block applies an even count).
 * Unsharded tableaux only (row0 = 0, rows = n).  `blk` is device scratch of smx_block_bytes
 * bytes (no initialisation needed).  smx_block_bytes: with *pivots_inout = 0 it asks the
 * library's policy (smx_tune_block: 0 automatic = from 48 MiB on, 24 pivots where the persistent
 * window planner runs, else 10 up to 256 MiB, 12 from 256 MiB, 20 from 1 GiB; 1 never, 2..24
 * that many) and returns 0 when chains of
 * `shape` would not use blocks; with 1..24 it asks for that many (0: `shape` not eligible).  Otherwise it returns the scratch size and sets
 * *pivots_inout to the pivots per block.  smx_block_run_timed also returns each sweep's HIP-event time (ceil(k/pivots)
 * entries) and the chain's total. */
int smx_tune_block(int32_t pivots);
/* Planner of unsharded block chains: 0 (default) the window planner -- T_{k+D} at the first
 * nwin - 1 columns and the "-b" column of every row, kept current pivot by pivot over up to 256
 * workgroups: ONE persistent launch per block (k_blk_wplan: the window in registers, the steps
 * handing off through tagged granules) where its workgroups fit one per CU and its rows in
 * registers (up to 32,768 rows), else one launch per pivot (k_blk_wstep); then the pivot rows at
 * every column once per block (k_blk_prows; columns outside the window through chains from the
 * block's input table); 2 the window planner's launch form always; 1 the register-form chains
 * (k_blk_step).  nwin: window slots 2..64 (0 = 64, the default; -1 keeps it).  Same decisions
 * and bits either way.  Returns the previous planner. */
int smx_tune_block_planner(int32_t planner, int32_t nwin);
/* Layout of the block sweep (k_blk_sweep, csrc/smx_block.hpp): 0 automatic (the default: pivot-
 * row slices in registers up to 12 pivots per sweep, in LDS shared by a workgroup's waves beyond,
 * and wherever the register layout's grid cannot give every wave one column chunk), 4 registers,
 * 5 LDS, 6 LDS in work items (every workgroup's rows in K segments, each at another column chunk:
 * SMX_SWEEP_ITEMS=K, default 16); any other value keeps the setting.  Returns the previous one.
 * Same bits either way. */
int smx_tune_block_form(int32_t form);
int64_t smx_block_bytes(const smx_shape* shape, int32_t* pivots_inout);
int smx_block_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                  int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes, int32_t* log,
                  double* xhist, int64_t log_cap, void* stream);
int smx_block_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                        int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                        int32_t* log, double* xhist, int64_t log_cap, void* stream,
                        float* host_sweep_ms, float* host_total_ms);
/* With host_sweep_ms = host_total_ms = NULL, smx_block_run_timed only enqueues (asynchronous);
 * smx_block_timed_read(ceil(k/pivots), ...) then waits for that chain's last event and returns
 * the same times (a caller's timed region can end at its own synchronize, before the readout). */
int smx_block_timed_read(int32_t blocks, float* host_sweep_ms, float* host_total_ms);
int smx_block_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                           int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                           int32_t* log, double* xhist, int64_t log_cap, void* stream,
                           void** graph_out);

/* ---- block pivots, row-sharded (one rank per GPU) -----------------------------------------
 * The block chain of smx_block_run on this rank's row block (shape.row0 / rows; a rank may own
 * no rows), with ONE all-gather per pivot of the send slots (layout of smx_shard_*: header +
 * row A + row B, SMX_SHARD_HDR + 2*ld doubles per rank; rows as values of T_{k+D} derived from
 * the block's input table).  smx_bshard_run issues the all-gathers itself through `comm`
 * (smx_comm_init) on `stream`; the step-wise calls let a driver do its own exchange:
 *   prime once per chain; per block `block` = 0, 1, ... (block start parity `parity`), for
 *   step = 1..pivots: pack(step - 1) -> all-gather send -> recv -> step(step); then sweep(T of
 *   the block, the other buffer) -- in place for an even count, so the table after d pivots is in
 *   buf[(parity0 + d) & 1]; after the last block publish(block count).
 * x-history: each rank writes (x1, x2) after every pivot into ITS ring for the label rows it
 * owns, and 0 for a label that is not basic (simplex.py:60-66); the slot of a basic label owned
 * by another rank is left untouched -- the host takes each value from the owner of the label's
 * row (it knows the positions from the pivot log).  `xhist` may be NULL.
 * `blk` is smx_bshard_bytes bytes. */
int64_t smx_bshard_bytes(const smx_shape* shape);
int smx_bshard_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity, int32_t k,
                   int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes, double* send,
                   double* recv, int32_t nranks, void* comm, int32_t* log, double* xhist,
                   int64_t log_cap, void* stream);
int smx_bshard_run_timed(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                         int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                         double* send, double* recv, int32_t nranks, void* comm, int32_t* log,
                         double* xhist, int64_t log_cap, void* stream, float* host_sweep_ms,
                         float* host_total_ms);
/* smx_bshard_run's chain of k pivots captured as a hipGraph (the RCCL collectives included):
 * smx_graph_launch replays it with one host call, smx_graph_destroy frees it.  A replay starts
 * from buf[parity] and leaves the table in buf[(parity + k) & 1]; every rank of the job captures
 * and replays its own graph in the same order. */
int smx_bshard_graph_create(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                            int32_t k, int32_t pivots, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                            double* send, double* recv, int32_t nranks, void* comm, int32_t* log,
                            double* xhist, int64_t log_cap, void* stream, void** graph_out);
int smx_bshard_prime(const double* T, const smx_shape* shape, int32_t parity, smx_ctl* ctl,
                     void* blk, int64_t blk_bytes, void* stream);
int smx_bshard_pack(const double* T, const smx_shape* shape, int32_t step, int32_t pivots,
                    int32_t block, const smx_ctl* ctl, void* blk, int64_t blk_bytes, double* send,
                    void* stream);
int smx_bshard_step(const double* T, const smx_shape* shape, int32_t step, int32_t pivots,
                    int32_t parity, int32_t block, const double* recv, int32_t nranks,
                    smx_ctl* ctl, void* blk, int64_t blk_bytes, int32_t* log, double* xhist,
                    int64_t log_cap, void* stream);
int smx_bshard_sweep(double* Tin, double* Tother, const smx_shape* shape, int32_t pivots,
                     void* blk, int64_t blk_bytes, void* stream);
/* The light exchange (smx_tune_shard_xchg): instead of all-gathering the whole send slots, a
 * driver all-gathers the SMX_SHARD_HDR-double headers only (hdrs = [nranks][SMX_SHARD_HDR]),
 * calls smx_bshard_pick (every rank: the same decision; the owner of the winning row copies it
 * into `row`, ld doubles, the others fill it with the bit pattern 0x8000000000000000), reduces
 * `row` over the ranks with MAX on int64 (an all-reduce: the owner's bits survive), and
 * decides the step with smx_bshard_step_light.  `rank` = this rank's index in the gather order.
 * Per pivot and rank: 64 B per rank + one row (all-reduce) instead of 64 B + 2 rows per rank. */
int smx_bshard_pick(const double* hdrs, const smx_shape* shape, int32_t nranks, int32_t rank,
                    const double* send, double* row, void* stream);
int smx_bshard_step_light(const double* T, const smx_shape* shape, int32_t step, int32_t pivots,
                          int32_t parity, int32_t block, const double* hdrs, const double* row,
                          int32_t nranks, smx_ctl* ctl, void* blk, int64_t blk_bytes,
                          int32_t* log, double* xhist, int64_t log_cap, void* stream);
/* Exchange of smx_bshard_run / smx_mshard_run (SMX_XCHG_RCCL): -1 automatic (light from 4 ranks
 * on), 0 full send slots, 1 light; -2 keeps; returns the previous setting.  recv must hold
 * nranks * (SMX_SHARD_HDR + 2 * ld) doubles either way (the light form uses its first
 * nranks * SMX_SHARD_HDR + ld). */
int smx_tune_shard_xchg(int32_t mode);
int smx_bshard_publish(const smx_shape* shape, int32_t parity, int32_t block, smx_ctl* ctl,
                       void* blk, int64_t blk_bytes, void* stream);

/* ---- row sharding across the devices of ONE process (SimplexMethod(..., devices=[...])) ------
 * The block protocol of smx_bshard_* for all ranks of a single-process job: every rank is a row
 * block on its own device and stream (the smx_bshard_* buffers of that rank), and per pivot the
 * ranks exchange their send slots by
 *   SMX_XCHG_RCCL -- the communicators of smx_mshard_comms (ncclCommInitAll over distinct
 *                    devices); one host thread per rank enqueues that rank's whole chain with
 *                    its own collectives, exactly as a rank of a multi-process job does.  Should
 *                    any rank fail to enqueue, every communicator is aborted (ncclCommAbort, so
 *                    no rank waits forever for the failed one's collectives) and the call returns
 *                    SMX_ERR_COMMS_ABORTED: the handles are gone, do not destroy them;
 *   SMX_XCHG_COPY -- one host thread; device copies of every send slot into every recv (one
 *                    gather launch per pivot on rank 0's stream when all ranks share a device),
 *                    ordered by events (any devices, also several ranks on ONE device, where
 *                    RCCL refuses).
 * Stream-ordered, no host synchronisation; the per-rank state afterwards is exactly what
 * smx_bshard_run leaves on each rank of a multi-process job. */
#define SMX_XCHG_RCCL 0
#define SMX_XCHG_COPY 1
#define SMX_ERR_COMMS_ABORTED (-2000)
typedef struct smx_rank {
    int32_t device;     /* HIP device ordinal of this row block                              */
    int32_t reserved;
    void* stream;       /* hipStream_t on that device                                        */
    double* buf0;       /* ping-pong local tableaux: the rank's rows, then its f-row replica */
    double* buf1;
    smx_ctl* ctl;
    void* blk;          /* smx_bshard_bytes(&shape) bytes                                    */
    int64_t blk_bytes;
    double* send;       /* SMX_SHARD_HDR + 2 * ld doubles                                    */
    double* recv;       /* nranks send slots                                                 */
    int32_t* log;       /* pivot log ring (may be NULL when log_cap = 0)                     */
    double* xhist;      /* x-history ring, see smx_bshard_* (may be NULL)                    */
    int64_t log_cap;
    void* comm;         /* ncclComm_t of this rank (SMX_XCHG_RCCL), else NULL                */
    smx_shape shape;    /* the rank's local shape (rows, row0; ld equal on every rank)        */
} smx_rank;
int smx_mshard_comms(void** comms_out, int32_t nranks, const int32_t* devices);
int smx_mshard_run(const smx_rank* ranks, int32_t nranks, int32_t parity, int32_t k,
                   int32_t pivots, int32_t exchange);
/* The first rank's own error of the last smx_mshard_run that returned SMX_ERR_COMMS_ABORTED
 * (a hipError_t, or -1000 - ncclResult_t), 0 if that call succeeded; *rank_out = that rank's
 * index (-1: none).  Every failing rank is also reported on stderr. */
int smx_mshard_last_error(int32_t* rank_out);
/* smx_mshard_run's k pivots with the copy exchange, every rank on ranks[0]'s device (the host-
 * bound case: ~3N host calls per pivot), captured once as ONE graph on ranks[0].stream -- the
 * other ranks' streams fork from and join back into it, and every event the capture records is
 * its own, recorded exactly once.  Replay with smx_graph_launch(graph, ranks[0].stream), free
 * with smx_graph_destroy.  Opt-in (SimplexMethod(..., devices=[d] * N) with graph_chain=True). */
int smx_mshard_graph_create(const smx_rank* ranks, int32_t nranks, int32_t parity, int32_t k,
                            int32_t pivots, void** graph_out);
/* ---- Host engine (no device): the same pick_element / recalculate_matrix on a HOST tableau --
 * For machines without an MI355X (the reference UI's 2-variable LPs, BASELINE.json configs[0]).
 * Pointers here are HOST pointers (same layout as the device tableau: row-major fp64, R = n + 1
 * rows, leading dimension shape->ld, f-row entries j >= flen are padding); synchronous; the
 * decisions and per-element arithmetic are the device engine's, bit for bit.
 *   smx_host_select <- SimplexMethod.pick_element (simplex.py:70-141): returns the SMX_* status,
 *                      rc_out[0..1] = (r, c) of the pivot (r also set for SMX_INCORRECT)
 *   smx_host_pivot  <- recalculate_matrix after its pick (simplex.py:149-177): Tout from Tin,
 *                      out of place; -1 for an (r, c) outside the tableau
 *   smx_host_run    <- get_solution's loop (simplex.py:184-198) for k pivots starting at
 *                      buf[parity]; the table after d pivots is buf[(parity + d) & 1]; returns
 *                      the pivots applied, status_out = SMX_IDLE when all k were applied, else
 *                      the terminal SMX_* outcome; log[2 * d .. 2 * d + 1] = (r, c) of pivot d */
int smx_host_select(const double* T, const smx_shape* shape, int32_t* rc_out);
int smx_host_pivot(const double* Tin, double* Tout, const smx_shape* shape, int32_t r, int32_t c);
int64_t smx_host_run(double* buf0, double* buf1, const smx_shape* shape, int32_t parity,
                     int64_t k, int32_t* log, int32_t* status_out);

/* ---- Integer inputs: the first pivot's zero signs (smx_intfirst.hpp) ------------------------
 * The reference holds the caller's Python ints as ints until its first recalculate_matrix
 * (simplex.py:36-39, :155-175), and int arithmetic gives some zero results of that pivot the
 * opposite sign from fp64 (-0 is the int 0; an int product 0 * -3 is +0).  After the regular
 * first pivot T0 -> T1 (any engine: update, block, resident, sharded), this rewrites the entries
 * of T1 that are +-0 with the int semantics; every other entry already agrees in every bit
 * (|ints| < 2^26).  rows x cols local entries (ld doubles per row), r_local = the pivot row's
 * local index or -1 when another rank holds it, prow = T0's pivot row (cols doubles, e =
 * prow[c]), mask = 1 byte per T0 entry (ldm per row; nonzero = the caller passed an int) or
 * NULL when every entry is an int, maskr = the pivot row's mask (NULL likewise).  Device
 * pointers and `stream` for smx_int_first_fix, host pointers (synchronous) for the host form. */
int smx_int_first_fix(const double* T0, double* T1, int64_t ld, int32_t rows, int32_t cols,
                      int32_t r_local, int32_t c, const double* prow, const uint8_t* mask,
                      int64_t ldm, const uint8_t* maskr, void* stream);
int smx_host_int_first_fix(const double* T0, double* T1, int64_t ld, int32_t rows, int32_t cols,
                           int32_t r_local, int32_t c, const double* prow, const uint8_t* mask,
                           int64_t ldm, const uint8_t* maskr);

#ifdef __cplusplus
}
#endif
#endif /* SMX_H */
