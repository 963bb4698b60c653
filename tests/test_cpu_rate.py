"""The cpu_baseline's pure-Python leg stands in for the reference's own CPU cost.

profiles/r02/cpu_rate_check.json was written by tools/cpu_rate_check.py in the build container:
the reference's pick_element + recalculate_matrix (simplex.py:70-177, imported from
/root/reference) and oracle/restated.py's pick + pivot, timed interleaved on the same seeded LPs.
The restatement hoists the row and column reads out of the inner loop, so it is faster per element
than the reference: the python leg of bench.py's cpu_baseline OVERSTATES the reference's CPU rate
(a conservative baseline), by the factor recorded here."""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_restatement_rate_is_pinned_and_conservative():
    with open(os.path.join(REPO, "profiles", "r02", "cpu_rate_check.json")) as fh:
        rec = json.load(fh)
    sizes = {r["size"] for r in rec["rows"]}
    assert 1024 in sizes          # the size bench.py times the python leg at
    for r in rec["rows"]:
        assert r["ratio_restated_over_reference"] == (
            r["restated_ns_per_element"] / r["reference_ns_per_element"])
        # never slower than the reference (the baseline does not flatter the GPU) and within
        # the same order: a stand-in, not a different algorithm
        assert 0.4 < r["ratio_restated_over_reference"] <= 1.0
        assert 100.0 < r["reference_ns_per_element"] < 5000.0
