#!/usr/bin/env python3
"""One ugpu_find_records pass over a host buffer with the pipeline's per-chunk
timestamps (UGPU_REC_TRACE=1 on stderr): where the records path's time goes.
    python tools/rec_trace.py CONFIG MIB"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import ugrep_amd as U  # noqa: E402
from oracle_lib import gen  # noqa: E402

PATS = {"c2": ("foo|bar|baz", 1), "c3": ("[A-Za-z_][A-Za-z0-9_]*", 3), "c4": (r"\w+", 4)}
rx, kind = PATS[sys.argv[1]]
n = int(sys.argv[2]) << 20
pat = U.Pattern(U.compile_regex(rx))
buf = np.ascontiguousarray(gen(kind, 1, 0, n))
for rep in range(3):
    t0 = time.perf_counter()
    rr = U.Records(pat, buf)
    t1 = time.perf_counter()
    got = rr.drain()
    t2 = time.perf_counter()
    rr.close()
    print("rep %d: find_records %.3f ms, drained %.3f ms (%.1f GB/s), %d records" %
          (rep, (t1 - t0) * 1e3, (t2 - t0) * 1e3, n / (t2 - t0) / 1e9, got[0]), file=sys.stderr, flush=True)
