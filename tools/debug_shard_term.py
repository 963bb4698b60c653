import sys, os
sys.path[:0] = ['tests', 'simplex-method-solver_amd', '.']
import numpy as np, torch
from test_gpu_sharded import _simulate
from simplex_mi355x import lp
from oracle import c_oracle
n, m = 40, 30
T = lp.dense_tableau("uniform", 2, n, m)
for k in (78, 79, 80, 81, 400):
    states, logs, tables, full = _simulate(T, n, m, k, 3)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k)
    print(k, "oracle", st, done, "hip", states, "logs_eq", [np.array_equal(l, log) for l in logs],
          "table_eq", np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64)), flush=True)
