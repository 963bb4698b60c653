"""The committed bench evidence keeps the driver's contract (CPU only: reads profiles/).

profiles/r03c/bench20_default.json is a `python bench.py --steps 20 --warmup 5` line (the
driver's command) of the final round-3 build's GPU run, with its cpu_baseline;
profiles/r03c/bench_steps{20,200}_rocprof.json and kernel_stats_16384_steps{20,200}.csv are the
bench lines and rocprofv3 kernel-trace stats of the same commands (tools/profile_r03.sh),
profiles/r03c/pmc/ the FETCH_SIZE / WRITE_SIZE passes of the --steps 20 line.  The checks: the
JSON line's keys and types, the roofline arithmetic (achieved = algorithmic bytes / average
launch, frac = achieved / peak), the cpu_baseline block, and that the HIP-event launch average
agrees with rocprofv3's.
"""
import csv
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")


def _line(name):
    with open(os.path.join(PROF, name)) as fh:
        lines = [ln for ln in fh.read().splitlines() if ln.startswith("{")]
    assert lines, name
    return json.loads(lines[-1])


def _rocprof_avg_ms(name, needle):
    with open(os.path.join(PROF, name)) as fh:
        rows = [r for r in csv.DictReader(fh) if needle in r["Name"]]
    assert rows, needle
    calls = sum(int(r["Calls"]) for r in rows)
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    return total / calls * 1e-6


def test_default_line_keys():
    rec = _line("r03c/bench20_default.json")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in rec, k
    assert rec["unit"] == "pivots/s" and rec["dtype"] == "f64" and rec["n_gpus"] == 1
    assert rec["higher_is_better"] is True and rec["vs_baseline"] is None
    assert "workload" in rec["config"] and rec["config"]["rows"] == 16384
    assert rec["trajectory_valid"] is True
    assert rec["value"] == pytest.approx(1e3 / rec["ms_per_step"], rel=1e-6)


def test_roofline_arithmetic():
    r = _line("r03c/bench20_default.json")["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    ach = r["algorithmic_bytes_per_launch"] / (r["avg_kernel_ms"] * 1e-3) / 1e9
    assert r["achieved"] == pytest.approx(ach, rel=1e-9)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-9)
    assert r["algorithmic_bytes_per_launch"] == 16.0 * 16384 * 16384
    # PMC traffic within a few percent of the algorithmic bytes (no re-reads)
    assert r["traffic"] is not None
    assert 1.0 <= r["traffic"] / r["algorithmic_bytes_per_launch"] < 1.03


def test_cpu_baseline_block():
    cb = _line("r03c/bench20_default.json")["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1
    assert cb["value"] > 0 and cb["unit"] == "pivots/s" and cb["sample"]


@pytest.mark.parametrize("steps,kernel", [(20, "k_blk_sweep<10>"), (200, "k_blk_sweep<12>")])
def test_event_average_agrees_with_rocprof(steps, kernel):
    rec = _line(f"r03c/bench_steps{steps}_rocprof.json")
    r = rec["roofline"]
    prof = _rocprof_avg_ms(f"r03c/kernel_stats_16384_steps{steps}.csv", "k_blk_sweep<")
    assert r["kernel"] == kernel
    assert abs(r["avg_kernel_ms"] - prof) / prof < 0.10, (r["avg_kernel_ms"], prof)


def test_pmc_summary_matches_csv_passes():
    with open(os.path.join(PROF, "pmc_traffic.json")) as fh:
        t = json.load(fh)["16384x16384/k_blk_sweep<10>"]
    assert t["bytes_per_launch"] == pytest.approx(t["read_bytes_corrected"] + t["write_bytes"])
    assert t["read_bytes_corrected"] == pytest.approx(2 * 1024 * t["fetch_size_kib_median"])
    assert t["write_bytes"] == pytest.approx(1024 * t["write_size_kib_median"])
    # and it is the median of the committed counter passes
    import importlib.util
    import statistics
    spec = importlib.util.spec_from_file_location(
        "pmc_traffic", os.path.join(REPO, "tools", "pmc_traffic.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    d = os.path.join(PROF, "r03c", "pmc")
    assert statistics.median(mod.per_dispatch(d, "FETCH_SIZE", "k_blk_sweep<10")) == \
        t["fetch_size_kib_median"]
    assert statistics.median(mod.per_dispatch(d, "WRITE_SIZE", "k_blk_sweep<10")) == \
        t["write_size_kib_median"]


def test_valu_table_matches_counter_summaries():
    """profiles/valu_instr.json (bench.py's two-term bound) is tools/valu_instr.py over the
    committed SQ_INSTS_VALU summaries: lane-instructions per element-pivot of the sweep."""
    import subprocess
    import sys
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "valu_instr.py")],
                         check=True, capture_output=True, text=True).stdout
    with open(os.path.join(PROF, "valu_instr.json")) as fh:
        committed = json.load(fh)
    assert json.loads(out) == committed
    for key, rec in committed.items():
        assert key.startswith("16384x16384/k_blk_sweep<")
        # ~3 f64 ops per element-pivot (a FMA-shaped update plus the exact rounding fix-ups) and
        # the loads/stores/index arithmetic around them
        assert 6.0 < rec["instr_per_element_pivot"] < 12.0
        # the merged multi-pass summaries know the fp64 share; a single SQ_INSTS_VALU pass not
        if "f64_fma_mul_add_share" in rec:
            assert rec["f64_fma_mul_add_share"] > 0.6
        else:
            assert rec["source"].endswith(")") and "_counter_collection.csv" in rec["source"]


def test_two_term_arithmetic(monkeypatch):
    """bench.two_term (the block path's VALU-vs-HBM bound) on CPU, the device query stubbed."""
    import importlib.util

    import torch
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    class Props:
        multi_processor_count = 256
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: Props())
    R = C = 16384
    hbm = 16.0 * R * C
    t = bench.two_term(R, C, 12, 8.15, 1.2e-3, hbm)
    t_valu = R * C * 12 * 8.15 / 64 / (256 * 2.4e9)
    t_hbm = hbm / 8e12
    assert t["valu_peak_ms"] == pytest.approx(t_valu * 1e3)
    assert t["hbm_peak_ms"] == pytest.approx(t_hbm * 1e3)
    assert t["bound"] == "valu" and t["frac"] == pytest.approx(max(t_valu, t_hbm) / 1.2e-3)
    assert bench.two_term(R, C, 4, 8.15, 1.0e-3, hbm)["bound"] == "hbm"


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_physical_guard_rejects_impossible_rates():
    """bench.physical_check refuses a launch that would move bytes faster than the memory system
    can (the round-3 forced-update record: 1.07 GB in 0.26 us); accepts the real ones."""
    bench = _bench_module()
    R = 8192
    b = 16.0 * R * R
    with pytest.raises(ValueError, match="physical limit"):
        bench.physical_check("forced 8192^2", b, 0.2624e-6, b)
    # 200 us for the same pivot: 5.4 TB/s, below 8 TB/s
    assert bench.physical_check("forced 8192^2", b, 200.6e-6, b) == pytest.approx(b / 200.6e-6 / 1e9)
    # a 16384^2 sweep: HBM-bound working set, limit 8 TB/s (0.5 ms for 4.3 GB would be 8.6 TB/s)
    b16 = 16.0 * 16384 * 16384
    with pytest.raises(ValueError):
        bench.physical_check("sweep", b16, 0.5e-3, 8.0 * 16384 * 16384)
    assert bench.physical_check("sweep", b16, 0.84e-3, 8.0 * 16384 * 16384) < 8000.0
    # a cache-resident 1024^2 update (16.8 MB): bounded by the L2 rate, not HBM -- 4.7 us is
    # legal (3.6 TB/s), the 0.36 us "record" is not (47 TB/s)
    b1 = 16.0 * 1024 * 1024
    assert bench.physical_limit_gbs(b1) == bench.L2_AGG_GBS
    bench.physical_check("forced 1024^2", b1, 4.7e-6, b1)
    with pytest.raises(ValueError):
        bench.physical_check("forced 1024^2", b1, 0.3576e-6, b1)
    with pytest.raises(ValueError):
        bench.physical_check("zero", b1, 0.0, b1)


def test_committed_config_records_are_physical():
    """Every forced-update / chain record committed from round 4 on passes the guard."""
    import glob
    bench = _bench_module()
    paths = sorted(glob.glob(os.path.join(PROF, "r04*", "configs_2_3*.jsonl")))
    assert paths, "no round-4 configs record"
    for p in paths:
        with open(p) as fh:
            for ln in fh:
                if not ln.startswith("{"):
                    continue
                rec = json.loads(ln)
                if "forced_update_us" in rec:
                    b = 16.0 * rec["size"] ** 2
                    bench.physical_check(p, b, rec["forced_update_us"] * 1e-6, b)


def test_forced_record_agrees_with_rocprof():
    """The 8192^2 forced-update line (HIP events around the graph replay on the solver stream)
    agrees with the rocprofv3 kernel trace of the same tool run (k_update<kForced = 2, ...>)."""
    with open(os.path.join(PROF, "r04a", "configs_2_3.jsonl")) as fh:
        rec = [json.loads(ln) for ln in fh if '"forced_update_us"' in ln and '"size": 8192' in ln][0]
    prof_us = _rocprof_avg_ms("r04a/kernel_stats_run_configs3.csv", "k_update<2,") * 1e3
    assert abs(rec["forced_update_us"] - prof_us) / prof_us < 0.05, (rec, prof_us)


def test_world_guard_refuses_a_bare_multi_gpu_launch():
    """`python bench.py --gpus 2` without torch.distributed.run exits non-zero before touching the
    GPU (it used to fall into the sharded path at WORLD_SIZE 1 and print an n_gpus 1 line), and a
    torchrun world that differs from --gpus is refused too."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert out.returncode == 2, out
    assert "torch.distributed.run" in out.stderr
    bench = _bench_module()

    class A:
        gpus = 4
    assert bench.check_world(A(), {"WORLD_SIZE": "2"}) is not None
    assert bench.check_world(A(), {"WORLD_SIZE": "4"}) is None
    A.gpus = 1
    assert bench.check_world(A(), {}) is None


def test_parity_check_against_the_bench_fixture():
    """bench.parity_check: the line's own pivots (and, at 25 / 220 pivots, the table's SHA-256)
    against tests/golden/bench16k.json (the C oracle's run of the bench LP); a wrong pivot or a
    wrong table fails it, another workload is not checked."""
    import numpy as np
    bench = _bench_module()
    with open(os.path.join(REPO, "tests", "golden", "bench16k.json")) as fh:
        fx = json.load(fh)
    assert fx["n"] == fx["m"] == 16383 and fx["kind"] == "uniform" and fx["seed"] == 0
    assert set(fx["sha256"]) >= {"25", "220"} and len(fx["log"]) == fx["pivots"] >= 220

    class Dev:
        def __init__(self, log, table=None):
            self._log, self._t = np.array(log, dtype=np.int32), table

        def read_log(self, a, b):
            return self._log[a:b]

        def download(self):
            return self._t

    class A:
        kind, seed = "uniform", 0
    ok = bench.parity_check(Dev(fx["log"][:30]), A(), 16383, 16383, 30)
    assert ok["ok"] and ok["pivots_checked"] == 30 and ok["sha256_equal"] is None
    bad = [list(x) for x in fx["log"][:30]]
    bad[7][1] += 1
    assert bench.parity_check(Dev(bad), A(), 16383, 16383, 30)["ok"] is False
    # at 25 pivots the table is hashed: a wrong table fails (a small stand-in table)
    wrong = np.zeros((16384, 16384), dtype=np.float64)
    r = bench.parity_check(Dev(fx["log"][:25], wrong), A(), 16383, 16383, 25)
    assert r["sha256_at"] == 25 and r["sha256_equal"] is False and r["ok"] is False
    assert bench.parity_check(Dev([]), A(), 8191, 8191, 0) is None
    # the hash is the fixture generator's
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "mk5", os.path.join(REPO, "tests", "golden", "make_config5.py"))
    T = np.arange(7 * 5, dtype=np.float64).reshape(7, 5)
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    assert mk.table_sha256(T, 6, 4) == bench.table_sha256(T, 6, 4)


def test_roofline_bound_follows_the_two_term_bound():
    """The block line's roofline.bound is the two-term bound's (fp64 VALU issue for the 20-pivot
    sweep), with the VALU fraction at the committed shader clock beside it."""
    import re
    src = open(os.path.join(REPO, "bench.py")).read()
    assert re.search(r'"bound": \(extra\.get\("two_term"\) or \{\}\)\.get\("bound", "hbm"\)', src)
    bench = _bench_module()
    ghz, source = bench.load_clock("16384x16384/k_blk_sweep<20>")
    assert ghz is not None and 1.0 < ghz < 2.5 and source
