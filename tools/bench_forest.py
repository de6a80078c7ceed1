#!/usr/bin/env python3
"""Non-resynchronising FIND chains on the GPU: `\\D\\D` over
the C4 word corpus (no digits, so the two match phases never meet) resolved by
the forest FIND, against the reference matcher on the same bytes.

    python tools/bench_forest.py [--mib 1024] [--ref-mib 256]

Prints one JSON line: GPU time per whole-buffer scan (ugpu_scan + totals, which
falls to the forest after the speculative stitch gives up), count/digest/dcap,
and the reference harness (oracle/_ref, 1 thread: its newline-split threads
would cut \\D\\D matches that span a newline) on a prefix, with its result
compared to the GPU scan of that same prefix."""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import ugrep_amd as U  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--ref-mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--regex", default=r"\D\D")
    a = ap.parse_args()
    n = a.mib << 20
    dev = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    U.gen(4, 1, 0, dev.data_ptr(), n, st)
    torch.cuda.synchronize()
    pat = U.Pattern(U.compile_regex(a.regex))
    sc = U.Scanner(pat)

    def scan(m):
        sc.scan(dev.data_ptr(), 0, m, m, True, 0, st)
        t = sc.totals()
        return t

    t = scan(n)
    best = 1e30
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t = scan(n)
        best = min(best, time.perf_counter() - t0)
    out = {"regex": a.regex, "bytes": n, "seconds": round(best, 4), "gbps": round(n / best / 1e9, 2),
           "count": t.count, "digest": t.digest, "dcap": t.dcap, "forest": bool(t.flags & 8), "kernel": pat.info()["kernel"]}
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness_avx2")
    if a.ref_mib and os.path.exists(exe):
        m = min(a.ref_mib << 20, n)
        r = json.loads(subprocess.run([exe, "bench", "re", a.regex, "gen:4:1:0:%d" % m, "1", "1"], capture_output=True,
                                      check=True, timeout=900).stdout.decode().strip().splitlines()[-1])
        g = scan(m)
        out["reference"] = {"bytes": m, "threads": 1, "gbps": round(m / r["seconds"] / 1e9, 4),
                            "count": r["count"], "digest": r["digest"], "dcap": r["dcap"],
                            "gpu_equal": (g.count, g.digest, g.dcap) == (r["count"], r["digest"], r["dcap"])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
