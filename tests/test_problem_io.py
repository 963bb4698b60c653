"""Problem files: the reference's .txt format (main.py:386-495) and the binary .smx sibling."""
from __future__ import annotations

import numpy as np
import pytest

from golden_util import dec_input, load
from simplex_mi355x import problem_io


def test_txt_roundtrip_of_reference_examples(tmp_path):
    for name, case in load("examples.json").items():
        cons, func = dec_input(case["input"])
        if len(cons[0]) != 3:
            continue
        grad = list(func)[:2] + [0.0]                 # the UI keeps a 3rd gradient entry
        p = str(tmp_path / f"{name}.txt")
        problem_io.save_txt(p, cons, grad, 7)
        c2, g2, lim = problem_io.load_txt(p)
        assert c2 == [list(map(float, r)) for r in cons] and g2 == list(map(float, grad))
        assert lim == 7
        y, c = problem_io.solver_inputs_txt(p)
        assert c == list(map(float, grad))[:-1]       # main.py:312: grad[:-1]


def test_txt_written_format_matches_reference_writer(tmp_path):
    p = tmp_path / "p.txt"
    problem_io.save_txt(str(p), [[1.0, 1.0, -2.0], [-1.0, 1.0, 1.5]], [-1.0, -1.0, 0.0], 10)
    assert p.read_text(encoding="utf-8") == "1.0,1.0,-2.0\n-1.0,1.0,1.5\n-1.0,-1.0,0.0\n10"


@pytest.mark.parametrize("text,msg", [
    ("5", "Неверный формат файла"),
    ("1,2\n1,1,1\n3", "Неверный формат в строке 1: 1,2"),
    ("1,2,3\n1,1\n3", "Неверный формат градиента: 1,1"),
])
def test_txt_errors_use_reference_messages(tmp_path, text, msg):
    p = tmp_path / "bad.txt"
    p.write_text(text, encoding="utf-8")
    with pytest.raises(ValueError) as ei:
        problem_io.load_txt(str(p))
    assert str(ei.value) == msg


def test_smx_roundtrip_and_row_blocks(tmp_path):
    from simplex_mi355x import lp
    n, m = 300, 77
    T = lp.dense_tableau("uniform", 9, n, m)
    p = str(tmp_path / "t.smx")
    problem_io.save_smx(p, T, n, m, m, rows_per_chunk=64)
    assert problem_io.read_header(p) == (n, m, m, 80)
    full, n2, m2, flen = problem_io.load_host(p)
    assert (n2, m2, flen) == (n, m, m)
    assert np.array_equal(full.view(np.int64), T.view(np.int64))
    part, *_ = problem_io.load_host(p, 100, 200)
    assert np.array_equal(part[:-1], T[100:200]) and np.array_equal(part[-1], T[n])


def test_smx_rejects_garbage(tmp_path):
    p = tmp_path / "x.smx"
    p.write_bytes(b"not a tableau" * 10)
    with pytest.raises(ValueError):
        problem_io.read_header(str(p))


@pytest.mark.parametrize("name", list(load("examples.json")))
def test_from_file_txt_host_engine_vs_reference_examples(tmp_path, name):
    """The .txt path through the host engine (device="cpu") equals the reference's own
    get_solution() of every example LP (examples.json); the GPU twin is in test_gpu_parity.py."""
    import simplex
    from golden_util import check_txt_example
    check_txt_example(simplex.SimplexMethod, tmp_path, name, device="cpu")


def test_batch_eligibility_excludes_int_inputs():
    """solve_batch sends int / mixed problems to SimplexMethod (the int first-pivot fix), floats
    to the batch kernel (CPU: eligibility only)."""
    import numpy as np
    from simplex_mi355x.batch import _eligible
    fl = [[1.0, 1.0, -2.0], [-1.0, 1.0, 1.5], [1.0, -2.0, 4.0]]
    assert _eligible(fl, [-1.0, -1.0])
    assert not _eligible([[1, 1, -2], [-1, 1, 1.5], [1, -2, 4]], [-1, -1])
    assert not _eligible(fl, [-1, -1.0])
    assert not _eligible(fl[:2] + [[1.0, True, 4.0]], [-1.0, -1.0])
    assert not _eligible([np.array([1, 1, -2])] + fl[1:], [-1.0, -1.0])
    assert _eligible([np.array([1.0, 1.0, -2.0])] + fl[1:], [np.float64(-1.0), -1.0])
    assert not _eligible(fl, [np.int32(-1), -1.0])
