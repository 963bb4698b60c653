"""Problem files: the reference's ``.txt`` format and a binary sibling for HBM.

``.txt`` -- exactly the reference UI's format (main.py:386-393 writes, main.py:402-495 reads):
one ``a1,a2,b`` line per constraint (``y = a1*x1 + a2*x2 + b >= 0``), then the gradient line
``g1,g2,g3``, then the integer plot scale.  The solver's objective is ``grad[:-1]``
(main.py:312).  The reader raises ``ValueError`` with the reference's own messages where the UI
would show them in a message box.  The format is limited to 3 columns (main.py:439).

``.smx`` -- binary tableau for large LPs: a 64-byte little-endian header
``b"SMXTAB01", n, m, flen, ld, reserved*3`` (int64) followed by ``(n+1) x ld`` fp64 rows
(constraint rows, then the f-row, zero-padded).  ``load_device`` streams it from a memory map
into a ``DeviceTableau`` in row chunks (any size up to HBM, no Python lists, no full host copy);
``row_lo/row_hi`` read one rank's row block plus the f-row for the sharded engine.
"""
from __future__ import annotations

import os
import struct

import numpy as np

MAGIC = b"SMXTAB01"
HEADER = 64


# --------------------------------------------------------------------------- .txt (reference)
def save_txt(path: str, constraints, grad, lim: int) -> None:
    """main.py:386-393: coefficient lines, gradient line, scale (no trailing newline)."""
    with open(path, "w", encoding="utf-8") as f:
        for coeffs in constraints:
            f.write(",".join(map(str, coeffs)) + "\n")
        f.write(",".join(map(str, grad)) + "\n")
        f.write(str(lim))


def load_txt(path: str):
    """main.py:415-481 parsing rules; returns ``(constraints, grad, lim)``."""
    with open(path, "r", encoding="utf-8") as f:
        lines = f.readlines()
    if len(lines) < 2:
        raise ValueError("Неверный формат файла")                    # main.py:419-421
    data_lines = lines[:-1]
    num_lines = len(data_lines) - 1
    constraints, grad = [], []
    for row_idx, line in enumerate(data_lines):
        row_values = line.strip().split(",")
        if row_idx < num_lines:
            if len(row_values) != 3:                                # main.py:436-437
                raise ValueError(f"Неверный формат в строке {row_idx + 1}: {line.strip()}")
            constraints.append(list(map(float, row_values)))
        else:
            if len(row_values) != 3:                                # main.py:442-443
                raise ValueError(f"Неверный формат градиента: {line.strip()}")
            grad = list(map(float, row_values))
    lim = int(lines[-1].strip())                                     # main.py:478
    return constraints, grad, lim


def solver_inputs_txt(path: str):
    """What main.py:308-313 hands to SimplexMethod for this file: (y, grad[:-1])."""
    constraints, grad, _ = load_txt(path)
    return [list(map(float, r)) for r in constraints], list(grad)[:-1]


# --------------------------------------------------------------------------- .smx (binary)
def _ld(C: int) -> int:
    return ((C + 15) // 16) * 16


def save_smx(path: str, T: np.ndarray, n: int, m: int, flen: int, rows_per_chunk: int = 4096):
    """Write a dense tableau (rows 0..n-1 constraints, row n the f-row) as .smx."""
    C = m + 1
    ld = _ld(C)
    with open(path, "wb") as f:
        f.write(MAGIC + struct.pack("<7q", n, m, flen, ld, 0, 0, 0))
        buf = np.zeros((min(rows_per_chunk, n + 1), ld), dtype="<f8")
        for lo in range(0, n + 1, rows_per_chunk):
            hi = min(n + 1, lo + rows_per_chunk)
            blk = buf[:hi - lo]
            blk[:] = 0.0
            blk[:, :C] = T[lo:hi, :C]
            f.write(blk.tobytes())


def read_header(path: str):
    with open(path, "rb") as f:
        head = f.read(HEADER)
    if len(head) != HEADER or head[:8] != MAGIC:
        raise ValueError(f"{path}: not an .smx tableau")
    n, m, flen, ld = struct.unpack("<4q", head[8:40])
    if ld < m + 1 or os.path.getsize(path) < HEADER + (n + 1) * ld * 8:
        raise ValueError(f"{path}: truncated or inconsistent .smx header")
    return int(n), int(m), int(flen), int(ld)


def memmap(path: str):
    n, m, flen, ld = read_header(path)
    mm = np.memmap(path, dtype="<f8", mode="r", offset=HEADER, shape=(n + 1, ld))
    return mm, n, m, flen


def load_host(path: str, row_lo: int = 0, row_hi: int | None = None) -> tuple:
    """Rows [row_lo, row_hi) plus the f-row as a dense host array ``(rows+1, m+1)``."""
    mm, n, m, flen = memmap(path)
    row_hi = n if row_hi is None else row_hi
    T = np.empty((row_hi - row_lo + 1, m + 1), dtype=np.float64)
    T[:-1] = mm[row_lo:row_hi, :m + 1]
    T[-1] = mm[n, :m + 1]
    return T, n, m, flen


def load_device(path: str, device=None, row_lo: int = 0, row_hi: int | None = None,
                rows_per_chunk: int = 2048):
    """Stream an .smx file into a DeviceTableau (rows [row_lo, row_hi) + the f-row) in chunks."""
    import torch

    from .device import DeviceTableau
    mm, n, m, flen = memmap(path)
    row_hi = n if row_hi is None else row_hi
    rows = row_hi - row_lo
    C = m + 1
    stub = np.zeros((rows + 1, 0), dtype=np.float64)   # shape carrier, no payload
    dev = DeviceTableau(stub, n, m, flen, device=device, row0=row_lo,
                        n_global=n, defer_upload=True)
    with torch.cuda.stream(dev.stream):
        dev.buf.zero_()
        for lo in range(0, rows, rows_per_chunk):
            hi = min(rows, lo + rows_per_chunk)
            blk = torch.from_numpy(np.array(mm[row_lo + lo:row_lo + hi, :C]))
            dev.buf[0, lo:hi, :C].copy_(blk)
        dev.buf[0, rows, :C].copy_(torch.from_numpy(np.array(mm[n, :C])))
    dev.reset_state()
    return dev
