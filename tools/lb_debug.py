"""Loop-needle lookback: step-by-step GPU check with progress lines (debug aid)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

import ugrep_amd as U  # noqa: E402
from oracle_lib import OracleDfa  # noqa: E402
import test_lookback as T  # noqa: E402


def check(rx, host, lb, what, **kw):
    t0 = time.time()
    os.environ["UGPU_LB"] = lb
    pat = U.Pattern(rx, word=kw.pop("word", False))
    os.environ.pop("UGPU_LB", None)
    dev = torch.from_numpy(host).to("cuda")
    o = OracleDfa(U.compile_regex(rx))
    want = (o.find_w if pat.word else o.find)(host, want_list=True)
    print(f"{what} rx={rx} lb={lb} n={host.size} oracle={want[0]} ({time.time() - t0:.2f}s)", flush=True)
    r = U.find_all(pat, dev, offsets=kw.get("offsets", True))
    ok = (r.count, r.digest, r.dcap) == want[:3]
    print(f"   gpu={r.count} ok={ok} ({time.time() - t0:.2f}s)", flush=True)
    if not ok and kw.get("offsets", True):
        got = r.triples()
        for i, (a, b) in enumerate(zip(got, want[3])):
            if a != b:
                print("   first diff", i, a, b, bytes(host[max(0, b[0] - 20):b[0] + 30]), flush=True)
                break
        else:
            print("   lengths", len(got), len(want[3]), got[-3:], want[3][-3:], flush=True)
    return ok


def timed(rx, host, lb, what, start=0, word=False):
    os.environ["UGPU_LB"] = lb
    pat = U.Pattern(rx, word=word)
    os.environ.pop("UGPU_LB", None)
    dev = torch.from_numpy(host).to("cuda")
    o = OracleDfa(U.compile_regex(rx))
    want = (o.find_w if word else o.find)(host, start=start, want_list=True)
    U.find_all(pat, dev, start=start)
    torch.cuda.synchronize()
    t0 = time.time()
    r = U.find_all(pat, dev, start=start)
    dt = time.time() - t0
    print(f"{what} rx={rx} lb={lb} start={start} n={host.size} ok={r.triples() == want[3]} gpu {dt * 1e3:.1f} ms",
          flush=True)


rx, needle, f = T.CASES[0]
rng = np.random.default_rng(1)
toks = " ".join(["abc", "xing", "sing", "walking", "the", "a", "of"][int(i)] for i in rng.integers(0, 7, 300000))
segs = {"r70k": f * 70000 + needle, "r3k": f * 3000, "n50k": needle * 50000, "r150k": f * 150000 + needle,
        "r20k": f * 20000 + needle, "r5k": f * 5000 + needle, "r5kx": f * 5000}
for lb in ("1", "0"):
    for name, seg in segs.items():
        h = np.frombuffer((toks[:600000] + " " + seg + " " + toks[600000:]).encode(), np.uint8).copy()
        timed(rx, h, lb, name)
        timed(rx, h, lb, name + "-W", word=True)
host = T._text(3, 400000, needle, f)
for lb in ("1", "0"):
    timed(rx, host, lb, "text")
    timed(rx, host, lb, "text-W", word=True)
print("done", flush=True)
