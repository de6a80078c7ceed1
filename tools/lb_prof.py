"""Loop-needle lookback: the slow inputs alone, for a kernel-trace profile (debug aid)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

import ugrep_amd as U  # noqa: E402
import test_lookback as T  # noqa: E402

rx, needle, f = T.CASES[0]
host = T._text(3, 400000, needle, f)
which = sys.argv[1] if len(sys.argv) > 1 else "all"
os.environ["UGPU_LB"] = "1"
pat = U.Pattern(rx)
patw = U.Pattern(rx, word=True)
for name, h, p in (("text1M", host[:1 << 20], pat), ("rand", host[:800000], pat), ("tail", host[800000:1 << 20], pat),
                   ("word", host, patw)):
    if which not in ("all", name):
        continue
    dev = torch.from_numpy(h.copy()).to("cuda")
    t0 = time.time()
    r = U.find_all(p, dev)
    print(name, r.count, f"{(time.time() - t0) * 1e3:.1f} ms", flush=True)
