#!/usr/bin/env python3
"""Records path (ugpu_find_records + ugpu_records_drain) at 256 MiB over its
knobs: chunk size (UGPU_REC_CHUNK), 2-byte dense pieces (UGPU_REC_DENSE),
drain threads (UGPU_REC_DRAIN_THREADS) and borrowed buffers.  One JSON line
per setting, best of --reps; every result checked against ugpu_find_all.

    python tools/rec_sweep.py [--mib 256] [--reps 5]"""
import argparse
import itertools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import ugrep_amd as U  # noqa: E402

PATS = [("c3", "[A-Za-z_][A-Za-z0-9_]*", 3), ("c4", r"\w+", 4)]
CHUNKS = [int(x) for x in os.environ.get("SWEEP_CHUNKS", "16,32,64").split(",")]
DENSE = [int(x) for x in os.environ.get("SWEEP_DENSE", "0,1").split(",")]
THREADS = [int(x) for x in os.environ.get("SWEEP_THREADS", "8,16").split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from oracle_lib import gen
    n = a.mib << 20
    for name, rx, kind in PATS:
        pat = U.Pattern(U.compile_regex(rx))
        buf = gen(kind, 1, 0, n)
        want = U.find_all(pat, buf, offsets=False)
        want = (want.count, want.digest, want.dcap)
        for chunk, dense, threads, borrow in itertools.product(CHUNKS, DENSE, THREADS, (False, True)):
            os.environ["UGPU_REC_CHUNK"] = str(chunk << 20)
            os.environ["UGPU_REC_DENSE"] = str(dense)
            os.environ["UGPU_REC_DRAIN_THREADS"] = str(threads)
            U.Records(pat, buf, borrow=borrow).drain()
            best = 1e30
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = U.Records(pat, buf, borrow=borrow)
                got = r.drain()
                best = min(best, time.perf_counter() - t0)
                r.close()
                assert got == want, (name, chunk, dense, threads, borrow)
            print(json.dumps({"config": name, "chunk_mib": chunk, "dense": dense, "drain_threads": threads,
                              "borrow": borrow, "ms": round(best * 1e3, 3), "gbps": round(n / best / 1e9, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
