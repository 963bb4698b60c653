"""CPU-side checks of the C ABI library (no compute calls: there is no GPU here)."""
from __future__ import annotations

import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "smx.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^int(?:64_t)? (smx_[a-z_]+)\(", text, flags=re.M)))


def test_header_declares_the_path():
    names = _declared()
    for need in ("smx_select", "smx_finalize", "smx_update", "smx_run", "smx_reset",
                 "smx_graph_create", "smx_shard_pack", "smx_shard_merge", "smx_shard_update"):
        assert need in names


def test_library_exports_every_declared_symbol():
    from simplex_mi355x import _lib
    L = _lib.load()
    for name in _declared():
        assert hasattr(L, name), name
    assert set(_declared()) == set(_lib.EXPORTS)


def test_library_is_gfx950_code_object():
    from simplex_mi355x import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert "gfx950" in _lib.version()


def test_library_stamp_matches_sources():
    """The library carries the stamp of the sources it was built from (csrc/Makefile SRC_HASH) and
    the loader refuses a stale one (the box must run what HEAD builds)."""
    from simplex_mi355x import _lib
    L = _lib.load()
    assert _lib.source_stamp() is not None
    assert _lib.library_stamp(L) == _lib.source_stamp()


def test_stale_library_is_refused(monkeypatch):
    from simplex_mi355x import _lib
    L = _lib.load()
    monkeypatch.setattr(_lib, "source_stamp", lambda: "0000000000000000")
    with pytest.raises(OSError, match="stale"):
        _lib.check_stamp(L, _lib.LIB_PATH)
    _lib.check_stamp(L, "/elsewhere/libsmx_ab_variant.so")   # an A/B build is not checked


def test_struct_layouts_match_header():
    from simplex_mi355x import _lib
    assert ctypes.sizeof(_lib.Shape) == 32
    assert _lib.CTL_DTYPE.itemsize == 128
    # offsets used by the host and the kernels (include/smx.h)
    f = _lib.CTL_DTYPE.fields
    assert (f["term"][1], f["npivots"][1], f["shard_off"][1], f["xpos"][1], f["npiv"][1],
            f["dec"][1]) == (16, 40, 56, 64, 80, 96)


def test_host_helpers_without_gpu():
    from simplex_mi355x import _lib
    L = _lib.load()
    assert L.smx_nparts_for(16383, 16383) == 64
    assert L.smx_nparts_for(3, 2) == 1


def test_device_tableau_refuses_to_run_without_gpu():
    """A device tableau never falls back: asking for the MI355X without one raises; only the
    explicit host engine (chosen by default when no HIP device exists) runs on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import simplex
    with pytest.raises(RuntimeError, match="no CPU path"):
        simplex.SimplexMethod([[1.0, 1.0, -2.0]], [-1.0, -1.0], device="cuda:0")
    assert simplex.SimplexMethod([[1.0, 1.0, -2.0]], [-1.0, -1.0]).backend == "host"


def test_reference_entry_errors_before_device():
    """IndexError on an empty problem comes from the same line as in the reference (:27)."""
    import simplex
    with pytest.raises(IndexError):
        simplex.SimplexMethod([], [-1.0])


def test_ragged_rows_rejected_before_device():
    import simplex
    with pytest.raises(ValueError, match="ragged"):
        simplex.SimplexMethod([[1.0, 2.0, 3.0], [1.0, 2.0]], [-1.0, -1.0])


def test_ops_registered_as_torch_custom_ops():
    import torch
    import simplex_mi355x.ops  # noqa: F401
    for name in ("reset", "select", "finalize", "update", "run", "update_forced",
                 "shard_pack", "shard_merge", "shard_update"):
        assert hasattr(torch.ops.smx, name)


def test_lp_generator_is_shardable():
    import numpy as np
    from simplex_mi355x import lp
    full = lp.dense_rows("uniform", 5, 3000, 40)
    part = lp.dense_rows("uniform", 5, 3000, 40, 1000, 2500)
    assert np.array_equal(full[1000:2500], part)
    T = lp.dense_tableau("degenerate", 2, 50, 30)
    assert T.shape == (51, 31) and np.all(T[-1, 30] == 0)


def _integration_stub():
    """The ctypes binding block of INTEGRATION.md, bound to the in-tree libsmx.so."""
    from simplex_mi355x import _lib
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(# src/simplex_hip.py.*?)```", text, flags=re.S).group(1)
    ns = {}
    exec(compile(block.replace('"libsmx.so"', repr(_lib.LIB_PATH)), "INTEGRATION.md", "exec"),
         ns)
    return ns


def test_integration_stub_matches_library_signatures():
    from simplex_mi355x import _lib
    ns = _integration_stub()
    L = _lib.load()
    for name in ("smx_reset", "smx_select", "smx_finalize", "smx_update", "smx_run"):
        stub = getattr(ns["L"], name).argtypes
        assert len(stub) == len(getattr(L, name).argtypes), name
    assert ctypes.sizeof(ns["Shape"]) == ctypes.sizeof(_lib.Shape)
