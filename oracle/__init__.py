"""CPU oracle for the simplex pivot path — TEST INFRASTRUCTURE ONLY.

Restatements of /root/reference/src/simplex.py used as the parity checker (tests/, smoke())
and as the timed CPU baseline (bench.py cpu_baseline).  The product package never imports it.
"""
