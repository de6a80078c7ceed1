"""Round 6 diagnostic: needle-free runs of 5000 bytes (tests/test_dom.py) per
pattern, dominated restarts on and off (UGPU_DOM=0), wall ms per COUNT scan."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ugrep_amd as U  # noqa: E402

rng = np.random.default_rng(11)
base = np.frombuffer((b"the sailing boat passed qux abcdx " * 32000)[:1 << 20], np.uint8).copy()
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for pos in (4096 - 2500, 65536 - 100, 300001, (1 << 20) - 5000)[:runs]:
    base[pos:pos + 5000] = rng.choice(np.frombuffer(b"abcdfghjklmnopstuvwz", np.uint8), 5000)
dev = torch.from_numpy(base).cuda()
for rx in ["[a-z]+(ing|ed)", "[a-z]*q[a-z]*x", "a[a-z]*(ing|ed)", "[a-z]+(ab|cd|ef)x"]:
    for d in ("1", "0"):
        os.environ["UGPU_DOM"] = d
        pat = U.Pattern(U.compile_regex(rx))
        U.find_all(pat, dev, offsets=False)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = U.find_all(pat, dev, offsets=False)
            ts.append((time.perf_counter() - t0) * 1e3)
        print(rx, "dom", d, r.count, "ms", [round(t, 2) for t in ts], flush=True)
