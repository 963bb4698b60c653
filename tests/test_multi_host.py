"""Host-side error handling of the single-process multi-device driver (simplex_mi355x/multi.py)
without a GPU: the library call is stubbed."""
from __future__ import annotations

import pytest


def test_aborted_communicators_are_not_reused(monkeypatch):
    """After smx_mshard_run aborted (and so freed) every RCCL communicator, the rank table no
    longer carries their handles and a later run refuses instead of passing freed handles to RCCL
    (ADVICE r5); the failing rank's own code reaches the message (smx_mshard_last_error)."""
    from simplex_mi355x import _lib, multi

    calls = []

    class FakeLib:
        def smx_mshard_run(self, structs, world, parity, k, pivots, xchg):
            calls.append([structs[p].comm for p in range(world)])
            return _lib.ERR_COMMS_ABORTED

        def smx_mshard_last_error(self, rank):
            rank._obj.value = 1
            return -1000 - 5

    monkeypatch.setattr(_lib, "load", lambda: FakeLib())
    mt = multi.MultiTableau.__new__(multi.MultiTableau)
    mt.world, mt.exchange, mt.step, mt.graph_chain = 2, "rccl", 0, False
    mt._structs = (_lib.Rank * 2)()
    mt._structs[0].comm, mt._structs[1].comm = 0x1000, 0x2000
    mt._comms = [0x1000, 0x2000]
    mt._aborted = False
    with pytest.raises(RuntimeError, match=r"rank 1: RCCL ncclInvalidUsage"):
        mt._native(4, 2)
    assert calls == [[0x1000, 0x2000]]
    assert mt._comms is None and [mt._structs[p].comm for p in range(2)] == [None, None]
    with pytest.raises(RuntimeError, match="aborted by an earlier"):
        mt._native(4, 2)
    assert len(calls) == 1
