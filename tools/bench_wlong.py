#!/usr/bin/env python3
"""Option W over long word runs (DESIGN 3.15 'not covered'): COUNT wall time
of U.find_all for W patterns over 64 MiB of the C2 corpus with letter runs of
150 KB and 1 MiB planted in it, and over the corpus alone; one JSON line per
pattern.  Run once per library (UGPU_LIB=libugrep_amd_wr0.so: the byte-load
walk) and compare; the counts must agree."""
import json
import os
import sys
import time

import numpy as np
import torch

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "tests")]
import ugrep_amd as U  # noqa: E402
from oracle_lib import gen  # noqa: E402

base = np.asarray(gen(1, 7, 0, 64 << 20)).copy()
runs = base.copy()
for k, (pos, n) in enumerate(((1 << 20, 150000), (9 << 20, 150000), (20 << 20, 1 << 20), (40 << 20, 400000))):
    seg = np.frombuffer((b" " + b"abcdefghij" * (n // 10) + (b"ing" if k % 2 == 0 else b"") + b" "), np.uint8)
    runs[pos:pos + seg.size] = seg
for rx in ("[a-z]+ing", "[A-Za-z]+tion", "[a-z]+[0-9]*", "\\w+x", "foo|bar|baz"):
    pat = U.Pattern(rx, word=True)
    out = dict(lib=os.environ.get("UGPU_LIB", "libugrep_amd.so"), pattern=rx, kernel=pat.info()["kernel"])
    for name, host in (("corpus", base), ("runs", runs)):
        dev = torch.from_numpy(host).to("cuda")
        r = U.find_all(pat, dev, offsets=False)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = U.find_all(pat, dev, offsets=False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = dict(ms=round(1e3 * sorted(ts)[1], 3), count=r.count, digest=r.digest)
    print(json.dumps(out), flush=True)
