"""U mode where it is the default: a code-point run table without a gap
transducer ([^a]+: no sync bytes), on 1 GiB of the C4 corpus, against the
kernel it replaces (UGPU_XU=0: dense_kernel).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ugrep_amd as U  # noqa: E402


def run(rx, n, reps=5):
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    U.gen(U.GEN_UTF8, 1, 0, buf.data_ptr(), n)
    torch.cuda.synchronize()
    out = {}
    for xu in ("1", "0"):
        os.environ["UGPU_XU"] = xu
        pat = U.Pattern(rx)
        sc = U.Scanner(pat)
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            sc.scan(buf.data_ptr(), 0, n, n, True, 0, torch.cuda.current_stream().cuda_stream)
            tot = sc.totals()
            best = min(best, time.perf_counter() - t)
        out["xu" if xu == "1" else "fallback"] = dict(kernel=pat.info()["kernel"], ms=round(best * 1e3, 3),
                                                     gbs=round(n / best / 1e9, 1), count=tot.count,
                                                     digest=tot.digest)
    os.environ.pop("UGPU_XU", None)
    out["equal"] = (out["xu"]["count"], out["xu"]["digest"]) == (out["fallback"]["count"], out["fallback"]["digest"])
    return out


if __name__ == "__main__":
    res = {rx: run(rx, 1 << 30) for rx in ("[^a]+", "[^\\n]+")}
    print(json.dumps(res))
