"""Benchmark: pivots/s and achieved HBM GB/s of the MI355X simplex pivot engine.

Workload (BASELINE.json configs[3], the north-star target config): a 16384 x 16384 dense fp64
tableau (n = m = 16383; seeded uniform random LP A~U(-1,1), b~U(0.1,1), c~U(-1,1), feasible at
the origin so the trajectory is a long phase-2 run), resident in HBM before timing starts.
A "step" is one pivot of the reference's get_solution loop (simplex.py:184-198): its selection
(pick_element, :70-141) and its Jordan step over every element (recalculate_matrix, :143-177).
At N = 1 on this table the steps run as block pivots: up to P pivots (the library's policy,
smx_tune_block: 24 where the persistent window planner runs -- this table's 2 GiB --, else 20 from
1 GiB, 12 from 256 MiB, 10 from 48 MiB) are decided by ONE persistent planner launch per block
(k_blk_wplan: the first columns of every row kept current pivot by pivot in registers, the steps
handing off through tagged granules, csrc/smx_wplan.hpp; it also derives the pivot rows at every
column), and ONE sweep of the tableau (k_blk_sweep) applies all of them, so a sweep moves 16 B per
element for P pivots (a chain of k pivots is cut into blocks of near-equal size: the driver's 20
pivots are ONE sweep of 20, the sustained 200 nine of 22-23);
bit-identical to one pivot per sweep.  After the timed region the
line adds `sustained` (the next 200 pivots, HIP events around every sweep: the steady-state rate
beside the burst) and times the one-pivot chain (k_update<kFused>, one kernel per pivot) as
"single_pivot_update".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--size S]

N = 1: one process.  N > 1: launched by torch.distributed.run, one rank per GPU; the tableau's
constraint rows are block-partitioned (strong scaling of the same tableau) and run the
block-sharded chain (sharded.py, smx_bshard_*): every pivot of a block exchanges one all-gather
of (header + candidate rows) over RCCL -- from 4 ranks on the light form, an all-gather of the
headers plus one max all-reduce of the pivot row -- and each rank sweeps its rows once per block.  Timing: barrier +
synchronize on both sides of exactly K pivots, max over ranks.  Rank 0 prints ONE JSON line.

roofline: algorithmic bytes of the dominant kernel = 16 B per tableau element per launch
(read + write every element once; a block sweep applies P pivots per launch), divided by that
kernel's average duration measured with HIP events on the solver stream inside the timed region
(block chain: events around every sweep; graph paths: events around the replay / K, so
inter-kernel gaps count as kernel time; N > 1: events around every update kernel).  traffic: HBM bytes per launch from
the committed rocprofv3 PMC summary (profiles/), FETCH_SIZE doubled per the gfx950 correction.
cpu_baseline: the numpy restatement of the same pivot (oracle/numpy_oracle.py, bit-identical to
the reference) on the same tableau, single thread, a bounded number of pivots.
parity: after the timed region the line checks itself against the C oracle's run of the same LP
(tests/golden/bench16k.json, made in the build container by tests/golden/make_bench16k.py): every
pivot (r, c) so far, and the SHA-256 of the whole table when the line stops at a pivot count the
fixture hashes (25 = the driver's --warmup 5 --steps 20; 220 = the defaults).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "simplex-method-solver_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "pivots/sec + achieved HBM GB/s, dense fp64 tableau, 1/2/4/8 MI355X"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
PEAK_CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)


L2_AGG_GBS = 36900.0   # aggregate L2 read rate, 8 XCDs (MI355X_MICROARCH.md, L2 section)
MALL_BYTES = 256 << 20  # Infinity Cache: a working set beyond it streams from HBM


def physical_limit_gbs(footprint_bytes):
    """The fastest rate any kernel can move bytes over a working set of `footprint_bytes`:
    HBM peak (8 TB/s) beyond the Infinity Cache, the aggregate L2 rate within it."""
    return PEAK_HBM_GBS if footprint_bytes > MALL_BYTES else L2_AGG_GBS


def physical_check(name, bytes_per_launch, seconds_per_launch, footprint_bytes):
    """Refuse a measurement whose implied rate (bytes one launch moves / its duration) exceeds
    what the memory system can deliver: a kernel that did no work, a graph that captured nothing
    or events that bracket the wrong stream all show up here.  Returns the rate in GB/s; raises
    ValueError for an impossible one."""
    if not seconds_per_launch > 0.0:
        raise ValueError(f"{name}: non-positive launch time {seconds_per_launch!r}")
    gbs = bytes_per_launch / seconds_per_launch / 1e9
    lim = physical_limit_gbs(footprint_bytes)
    if gbs > lim:
        raise ValueError(f"{name}: {bytes_per_launch:.4g} B in {seconds_per_launch * 1e6:.4g} us "
                         f"= {gbs:.0f} GB/s exceeds the physical limit {lim:.0f} GB/s for a "
                         f"{footprint_bytes / 2**20:.1f} MiB working set: the measurement is "
                         f"broken (no work done, or the wrong stream timed)")
    return gbs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=16384, help="tableau is size x size (n=m=size-1)")
    ap.add_argument("--rows", type=int, default=None, help="tableau rows R (default: --size)")
    ap.add_argument("--cols", type=int, default=None, help="tableau columns C (default: --size)")
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=None, help="PMC summary json (default: profiles/)")
    ap.add_argument("--sharded", action="store_true",
                    help="use the row-sharded RCCL path even at world size 1")
    ap.add_argument("--pivots", type=int, default=None,
                    help="row-sharded path: pivots per sweep at most (block pivots; 1 = one "
                         "pivot per sweep, the fused one-pivot protocol; default: 12 / 10 / 8 by "
                         "the size of each rank's table, as the single-GPU policy)")
    ap.add_argument("--xchg", choices=("auto", "full", "light"), default="auto",
                    help="row-sharded block path: exchange per pivot (full = all-gather of every "
                         "rank's header + 2 candidate rows; light = header all-gather + one "
                         "max all-reduce of the pivot row; auto = light from 4 ranks on)")
    ap.add_argument("--block-pivots", type=int, default=0,
                    help="N = 1: pivots per sweep (smx_tune_block; 0 = the library's policy, "
                         "20 at 16384^2)")
    ap.add_argument("--sustained", type=int, default=200,
                    help="block path, N = 1: after the timed region, time this many further "
                         "pivots with HIP events around every sweep (the steady-state rate beside "
                         "the timed burst), then one more block after 1 s idle; 0 = off")
    ap.add_argument("--enqueue-probe", action="store_true",
                    help="row-sharded block path: after the timed region, time the host enqueue "
                         "per pivot of the eager and graph-captured chains (host_enqueue)")
    return ap.parse_args()


def load_traffic(path, workload):
    if path is None:
        path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as fh:
            d = json.load(fh)
        rec = d.get(workload)
        return None if rec is None else float(rec["bytes_per_launch"])
    except Exception:
        return None


def load_valu(workload):
    """VALU lane-instructions per element-pivot of a block sweep, from SQ_INSTS_VALU
    (profiles/valu_instr.json, written by tools/valu_instr.py from the committed counter passes)."""
    path = os.path.join(REPO, "profiles", "valu_instr.json")
    try:
        with open(path) as fh:
            return float(json.load(fh)[workload]["instr_per_element_pivot"])
    except Exception:
        return None


def load_clock(workload):
    """The shader clock (GHz) the dominant sweep runs at, from a committed rocprofv3 GRBM pass
    (profiles/sweep_clock.json: GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / the dispatch's
    duration, written by tools/sweep_clock.py)."""
    try:
        with open(os.path.join(REPO, "profiles", "sweep_clock.json")) as fh:
            rec = json.load(fh)[workload]
        return float(rec["clock_ghz"]), rec.get("source")
    except Exception:
        return None, None


def two_term(R, C, pivots_per_launch, instr, avg_kernel, hbm_bytes):
    """The sweep's two-term bound: fp64 VALU issue (one wave64 instruction per
    CU per clock, 256 CUs at the 2.4 GHz peak clock) against HBM (8 TB/s); frac = the larger
    term over the measured average sweep."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    wave_instr = R * C * pivots_per_launch * instr / 64.0
    t_valu = wave_instr / (cus * PEAK_CLOCK_HZ)
    t_hbm = hbm_bytes / (PEAK_HBM_GBS * 1e9)
    return {"instr_per_element_pivot": instr, "wave_instr_per_launch": wave_instr,
            "valu_peak_ms": t_valu * 1e3, "hbm_peak_ms": t_hbm * 1e3,
            "bound": "valu" if t_valu > t_hbm else "hbm",
            "frac": max(t_valu, t_hbm) / avg_kernel,
            "valu_frac": t_valu / avg_kernel, "cus": cus, "peak_clock_ghz": PEAK_CLOCK_HZ / 1e9,
            "source": "SQ_INSTS_VALU passes, profiles/valu_instr.json"}


def shape_of(args):
    R = args.rows if args.rows else args.size
    C = args.cols if args.cols else args.size
    return R - 1, C - 1


def cycle_report(n, m, log):
    """Opt-in cycle detection over the pivots just run (host side, outside the timed region)."""
    from simplex_mi355x.basis import BasisTracker
    tr = BasisTracker(n, m)
    for r, c in log:
        if tr.pivot(int(r), int(c)):
            break
    return None if tr.cycle is None else {"first_step": tr.cycle[0], "period": tr.cycle[1]}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _timed_pivots(pick, pivot, A, n, m, seconds, min_done=2):
    done = 0
    t0 = time.perf_counter()
    while True:
        st, r, c = pick(A, n, m, m)
        if st != 0:
            break
        A = pivot(A, r, c)
        done += 1
        if time.perf_counter() - t0 >= seconds and done >= min_done:
            break
    return done, time.perf_counter() - t0


def cpu_baseline(T, n, m, seconds):
    """The reference's CPU path, restated (it is pure Python and cannot ship to the GPU box),
    timed on this host on a bounded sample of the same workload:
      value  -- numpy port (oracle/numpy_oracle.py, bit-identical), 1 thread, ~`seconds` s;
      omp    -- C port (oracle/simplex_oracle.c, bit-identical), OpenMP on the CPU share;
      python -- pure-Python list restatement incl. deepcopy (oracle/restated.py, the reference's
                own algorithm) at 1024x1024, its ns/element scaled to this tableau."""
    import numpy as np
    from oracle import c_oracle, numpy_oracle, restated
    A = np.ascontiguousarray(T)
    done, dt = _timed_pivots(numpy_oracle.pick, numpy_oracle.pivot, A, n, m, seconds)
    out = {"value": done / dt, "unit": "pivots/s", "cores": 1, "kind": "port",
           "sample": f"{done} pivots of the same {n + 1}x{m + 1} tableau from step 0 "
                     f"(numpy restatement, single thread), {dt:.1f} s",
           "cpu_model": _cpu_model()}
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16"))))
    done_c, dt_c = _timed_pivots(
        c_oracle.pick, lambda X, r, c: c_oracle.pivot(X, r, c, threads=threads), A, n, m,
        seconds / 3)
    out["omp"] = {"value": done_c / dt_c, "unit": "pivots/s", "cores": threads, "kind": "port",
                  "sample": f"{done_c} pivots, C restatement with OpenMP, {dt_c:.1f} s"}
    # pure Python on a 1024^2 replica of the generator (the reference's own per-element cost)
    from simplex_mi355x import lp
    nn = mm = 1023
    S = lp.dense_tableau("uniform", 0, nn, mm)
    tab = [list(map(float, row)) for row in S[:nn]] + [list(map(float, S[nn, :mm]))]
    t0 = time.perf_counter()
    k = 0
    while k < 2:
        st = restated.pick(tab, nn, mm, 1 + max(nn, mm))
        if st[0] != "pivot":
            break
        tab = restated.pivot(tab, st[1], st[2])
        k += 1
    dt_p = time.perf_counter() - t0
    if k:
        ns_el = dt_p / k / ((nn + 1) * (mm + 1)) * 1e9
        out["python"] = {"value": 1e9 / (ns_el * (n + 1) * (m + 1)), "unit": "pivots/s",
                         "cores": 1, "kind": "port",
                         "sample": f"{k} pivots (pick + pivot with deepcopy) at 1024x1024: "
                                   f"{ns_el:.0f} ns/element, scaled to {n + 1}x{m + 1}"}
        # the restatement is faster per element than the reference itself (hoisted row reads):
        # the ratio measured beside the reference in the build container (tools/cpu_rate_check.py)
        try:
            with open(os.path.join(REPO, "profiles", "r02", "cpu_rate_check.json")) as fh:
                ratio = {r["size"]: r["ratio_restated_over_reference"]
                         for r in json.load(fh)["rows"]}[1024]
            out["python"]["restated_over_reference_ns"] = ratio
            out["python"]["reference_estimate"] = out["python"]["value"] * ratio
        except (OSError, KeyError, ValueError):
            pass
    return out


def copy_ceiling(nbytes):
    """Best read+write rate of smx_copy_probe on this GPU for nbytes per buffer (GB/s)."""
    import torch
    from simplex_mi355x import _lib
    L = _lib.load()
    nd = (int(nbytes) // 16) * 2
    a = torch.ones(nd, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    s = torch.cuda.current_stream()
    best = 0.0
    for variant in (0, 1):
        for _ in range(3):
            _lib.check(L.smx_copy_probe(a.data_ptr(), b.data_ptr(), nd, variant, s.cuda_stream),
                       "smx_copy_probe")
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            L.smx_copy_probe(a.data_ptr(), b.data_ptr(), nd, variant, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        best = max(best, 2.0 * nd * 8 / (e0.elapsed_time(e1) / 10) / 1e6)
    del a, b
    torch.cuda.empty_cache()
    return best


def _single_pivot_line(dev, R, C, k):
    """The one-pivot-per-sweep chain (k_update<kFused>, a hipGraph of k launches) continued from
    the current table, outside the timed region: the rank-1 update kernel's own roofline."""
    import torch
    prev_block = dev.block
    dev.block = 0
    try:
        dev.prepare(k)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(dev.stream)
        dev.run(k, graph=True)
        e1.record(dev.stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        dev.sync_state()
    finally:
        dev.block = prev_block
    ach = physical_check("single_pivot_update", 16.0 * R * C, ms * 1e-3 / k, 16.0 * R * C)
    return {"kernel": "k_update<kFused>", "pivots_per_launch": 1, "pivots": k,
            "pivots_s": k / ms * 1e3, "avg_kernel_ms": ms / k, "achieved": ach,
            "unit": "GB/s", "frac": ach / PEAK_HBM_GBS}


def sustained_record(dev, P, k, idle_s=1.0):
    """The steady state beside the timed burst (outside the timed region, continuing the same
    trajectory): k more pivots in blocks of at most P with HIP events around every sweep, then,
    after `idle_s` seconds with the GPU idle, one more block of P.  A sweep that is slower in the
    sustained run than in the burst but fast again after the pause points at the clock (power /
    thermal state under a long fp64 load); one that stays slow points at the data (units leaving
    the sweep's fast path as the table's values spread)."""
    import numpy as np
    from simplex_mi355x import _lib
    L = _lib.load()
    nb = -(-k // P)
    _lib.check(L.smx_timer_reserve(2 * nb + 2), "smx_timer_reserve")
    t0 = time.perf_counter()
    sw, tot = dev.run_block_timed(k, P)
    wall = time.perf_counter() - t0
    ctl = dev.sync_state()
    out = {"pivots": k, "pivots_s": k / (tot * 1e-3), "wall_pivots_s": k / wall,
           "device_ms": tot, "sweeps": len(sw), "sweep_ms": [round(float(x), 4) for x in sw],
           "mean_sweep_ms": float(np.mean(sw)), "first_sweep_ms": float(sw[0]),
           "last_sweep_ms": float(sw[-1]),
           "planner_ms_per_pivot": (tot - float(np.sum(sw))) / k,
           "trajectory_valid": not bool(ctl["term"])}
    if not ctl["term"]:
        time.sleep(idle_s)
        sw2, tot2 = dev.run_block_timed(P, P)
        ctl = dev.sync_state()
        out["after_idle"] = {"idle_s": idle_s, "pivots": P, "sweep_ms": float(sw2[0]),
                             "device_ms": tot2, "trajectory_valid": not bool(ctl["term"])}
    return out


BENCH_FIXTURE = os.path.join(REPO, "tests", "golden", "bench16k.json")


def table_sha256(T, n, m):
    """SHA-256 of rows 0..n-1 (m + 1 values each, C order) then the f-row's first m values: the
    hash of tests/golden/make_config5.table_sha256."""
    import numpy as np
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(T[:n, :m + 1]))
    h.update(np.ascontiguousarray(T[n, :m]))
    return h.hexdigest()


def parity_check(dev, args, n, m, done):
    """The line against the C oracle's run of the same LP: the pivots logged
    so far and, at a pivot count the fixture hashes, the whole table.  None when the workload is
    not the fixture's (another size, generator or seed)."""
    if not os.path.exists(BENCH_FIXTURE):
        return None
    with open(BENCH_FIXTURE) as fh:
        fx = json.load(fh)
    if (n, m, args.kind, args.seed) != (fx["n"], fx["m"], fx["kind"], fx["seed"]):
        return None
    k = min(done, int(fx["pivots"]))
    log_ok = dev.read_log(0, k).tolist() == fx["log"][:k]
    sha_ok = None
    if str(done) in fx["sha256"]:
        sha_ok = table_sha256(dev.download(), n, m) == fx["sha256"][str(done)]
    return {"ok": bool(log_ok and sha_ok is not False), "pivots_checked": k,
            "log_equal": bool(log_ok), "sha256_at": done if sha_ok is not None else None,
            "sha256_equal": sha_ok, "fixture": "tests/golden/bench16k.json (C oracle)"}


def run_single(args):
    import numpy as np
    import torch
    from simplex_mi355x import _lib, lp
    from simplex_mi355x.device import DeviceTableau

    n, m = shape_of(args)
    R, C = n + 1, m + 1
    if args.block_pivots:
        _lib.tune_block(args.block_pivots)
    T = lp.dense_tableau(args.kind, args.seed, n, m)
    dev = DeviceTableau(T, n, m, m, device="cuda:0", log_cap=max(1 << 16, args.warmup + args.steps))
    if args.warmup:
        dev.run(args.warmup, graph=True)
        dev.sync_state()
    resident = dev.resident_plan()
    bplan = None if resident is not None else dev.block_plan()
    bytes_per_sweep = 16.0 * R * C   # read + write every element once
    extra = {}
    if bplan is not None:
        # block pivots: P pivots planned from the sweep's input table, then one sweep applies
        # them all.  The timed region launches the chain eagerly with HIP events around every
        # sweep on the solver stream (the host stays ahead: ~P+1 launches per ~1.5 ms of work),
        # so the sweep average comes from the timed run itself.
        P = bplan[1]
        nb = -(-args.steps // P)              # blocks of near-equal size (block_size in libsmx)
        P_top = -(-args.steps // nb)          # the largest block: the dominant sweep kernel
        # the per-sweep timing events exist before the timed region (no hipEventCreate inside)
        _lib.check(_lib.load().smx_timer_reserve(2 * nb + 2), "smx_timer_reserve")
        # host preparation (shape, plan, scratch) before the timed region; the events are read
        # after it (the region is: enqueue the K pivots, wait for them)
        launch, read = dev.block_timed_launcher(args.steps, P)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        sw, tot_ms = read()
        dev_ms = tot_ms
        avg_kernel = float(np.mean(sw)) * 1e-3
        kernel = f"k_blk_sweep<{P_top}>"
        traffic = load_traffic(args.traffic, f"{R}x{C}/k_blk_sweep<{P_top}>")
        instr = load_valu(f"{R}x{C}/{kernel}")
        extra = {"pivots_per_launch": args.steps / len(sw), "max_pivots_per_launch": P,
                 "launches": len(sw),
                 "planner_ms_per_pivot": (tot_ms - float(np.sum(sw))) / args.steps,
                 "algorithmic_bytes_per_pivot": bytes_per_sweep * len(sw) / args.steps}
        if instr is not None:
            extra["two_term"] = two_term(R, C, args.steps / len(sw), instr, avg_kernel,
                                         bytes_per_sweep)
            ghz, src = load_clock(f"{R}x{C}/{kernel}")
            if ghz is not None:
                # the VALU term at the clock the sweep actually holds (power-managed)
                tt = extra["two_term"]
                t_clk = tt["wave_instr_per_launch"] / (tt["cus"] * ghz * 1e9)
                tt["clock_ghz"] = ghz
                tt["clock_source"] = src
                tt["valu_ms_at_clock"] = t_clk * 1e3
                tt["valu_frac_at_clock"] = t_clk / avg_kernel
        # every launch of the chain: k_blk_start, per block Pb k_blk_step and k_blk_sweep +
        # k_blk_sweep_rest (the last one also publishes the chain's state)
        kernels_per_pivot = (args.steps + 2 * len(sw) + 1) / args.steps
    else:
        # the timed region replays one pre-captured hipGraph of K chained pivots (one fused
        # k_update per pivot, or the LDS-resident loop for tableaux that fit on chip); HIP events
        # on the solver stream bracket it, so the kernel average includes the inter-kernel gaps
        dev.prepare(args.steps)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(dev.stream)
        dev.run(args.steps, graph=True)
        ev1.record(dev.stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        dev_ms = ev0.elapsed_time(ev1)
        avg_kernel = dev_ms * 1e-3 / args.steps   # s per pivot (prime/publish included)
        if resident is not None:
            # one launch runs all K pivots: per launch K x 16 B per element, algorithmic only
            # (the tableau stays in LDS for the whole chain; HBM sees it once in, once out)
            kernel = "k_resident"
            avg_kernel = dev_ms * 1e-3
            bytes_per_sweep *= args.steps
            extra = {"pivots_per_launch": args.steps,
                     "note": "tableau held in LDS for the whole chain: the bytes are "
                             "algorithmic (16 B per element per pivot), not HBM traffic"}
            kernels_per_pivot = 1.0 / args.steps
        else:
            kernel = "k_update<kFused>" if _lib.fused_enabled() else "k_update<kSingle>"
            # fused: k_la_prime, K k_update, k_publish; unfused: k_select + k_update per pivot
            kernels_per_pivot = (args.steps + 2) / args.steps if _lib.fused_enabled() else 2
            extra = {"pivots_per_launch": 1}
        traffic = load_traffic(args.traffic, f"{R}x{C}")
    ctl = dev.sync_state()
    done = int(ctl["npivots"])
    valid = done == args.warmup + args.steps and not ctl["term"]
    cycle = cycle_report(n, m, dev.read_log(0, done))
    parity = parity_check(dev, args, n, m, done)
    if resident is not None:
        # algorithmic bytes of a chain held in LDS: not an HBM rate, no physical bound applies
        achieved = bytes_per_sweep / avg_kernel / 1e9
    else:
        # the sweep / update moves every element in and out once per launch; an in-place sweep's
        # working set is one buffer (8 B per element), so that is the footprint that decides
        # whether HBM or the caches bound it
        achieved = physical_check(kernel, bytes_per_sweep, avg_kernel, 8.0 * R * C)
    workload =f"{R}x{C} dense fp64 tableau, {args.kind} random LP seed {args.seed}"
    sustained = None
    if bplan is not None and valid and args.sustained > 0:
        sustained = sustained_record(dev, bplan[1], args.sustained)
    copy_gbs = copy_ceiling(8.0 * R * C)   # same bytes as one sweep (outside timing)
    single = None
    if bplan is not None and valid:
        single = _single_pivot_line(dev, R, C, 20)
    out = {
        "metric": METRIC,
        "value": args.steps / wall,
        "unit": "pivots/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: seeded dense random LP generated on the host, uploaded to HBM "
                "before timing (no dataset)",
        "config": {"workload": workload, "rows": R, "cols": C, "n": n, "m": m,
                   "parallelism": "single GPU", "kernels_per_pivot": kernels_per_pivot},
        # NOT an HBM rate: the bytes one pivot would move in a pass of its own (16 B per
        # element) over the time per pivot; a block sweep applies P pivots per pass, so this can
        # exceed the HBM peak.  roofline.achieved is the real HBM rate of the dominant kernel.
        "equiv_one_pass_gbs": 16.0 * R * C / (wall / args.steps) / 1e9,
        "equiv_one_pass_note": "16 B/element/pivot over wall time per pivot; a block sweep "
                               "moves 16 B/element once per P pivots, so this is not HBM traffic",
        "device_ms_per_step": dev_ms / args.steps,
        "parity": None if parity is None else parity["ok"],
        "parity_detail": parity,
        "roofline": dict({"bound": (extra.get("two_term") or {}).get("bound", "hbm"),
                          "achieved": achieved, "peak": PEAK_HBM_GBS,
                          "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                          "kernel": kernel, "algorithmic_bytes_per_launch": bytes_per_sweep,
                          "avg_kernel_ms": avg_kernel * 1e3,
                          "copy_ceiling_gbs": copy_gbs, "frac_of_copy": achieved / copy_gbs},
                         **extra),
        "single_pivot_update": single,
        "sustained": sustained,
        "trajectory_valid": bool(valid),
        "basis_cycle": cycle,
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(T, n, m, args.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


def check_world(args, env=None):
    """--gpus N must match the world torch.distributed.run formed: a bare
    `python bench.py --gpus 8` would otherwise run one rank and print an n_gpus 1 line.  Runs
    before anything touches the GPU; returns an error message or None."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in env and args.gpus > 1:
        return (f"bench.py --gpus {args.gpus}: launch one rank per GPU with `python -m "
                f"torch.distributed.run --nnodes=1 --nproc-per-node {args.gpus} --master-addr "
                f"127.0.0.1 --master-port <port> bench.py --gpus {args.gpus} ...`")
    if world != args.gpus:
        return (f"bench.py --gpus {args.gpus} but torch.distributed.run formed WORLD_SIZE={world}: "
                "refusing to report a line for a different GPU count")
    return None


def main():
    args = parse()
    msg = check_world(args)
    if msg:
        print(msg, file=sys.stderr, flush=True)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1 or args.sharded:
        from simplex_mi355x import sharded
        sharded.bench_main(args, METRIC, PEAK_HBM_GBS, cpu_baseline, load_traffic)
    else:
        run_single(args)


if __name__ == "__main__":
    main()
