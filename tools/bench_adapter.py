#!/usr/bin/env python3
"""Latency of the drop-in adapter's host-buffer path (ugpu_find_all on a host
buffer: H2D copy + scan + records back, what reflex::GpuMatcher does for a
buffer()-fed file) against the reference CPU matcher on the same bytes, over
input sizes from 4 KiB to 256 MiB.  Prints one JSON line per (pattern, size)
and a summary line with the crossover sizes (the
adapter's UGPU_ADAPTER_MIN_BYTES / UGPU_ADAPTER_SPARSE defaults).

    python tools/bench_adapter.py [--max-mib 256] [--reps 5]

The reference CPU leg runs oracle/_ref/ref_harness_avx2 (libreflex compiled from
the reference sources, 1 thread: one matcher, as the adapter replaces one)."""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import ugrep_amd as U  # noqa: E402

PATS = [("c2", "foo|bar|baz", 1), ("c3", "[A-Za-z_][A-Za-z0-9_]*", 3), ("c4", r"\w+", 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from oracle_lib import gen
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness_avx2")
    sizes = [4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20]
    sizes = [s for s in sizes if s <= a.max_mib << 20]
    summary = {}
    for name, rx, kind in PATS:
        pat = U.Pattern(U.compile_regex(rx))
        data = gen(kind, 1, 0, sizes[-1])
        cross = None
        for n in sizes:
            buf = np.ascontiguousarray(data[:n])
            U.find_all(pat, buf.tobytes(), offsets=True)  # warm
            best = 1e30
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = U.find_all(pat, buf, offsets=True)
                best = min(best, time.perf_counter() - t0)
            line = {"pattern": rx, "config": name, "bytes": n, "gpu_ms": round(best * 1e3, 4),
                    "gpu_gbps": round(n / best / 1e9, 3), "matches": r.count}
            # the records path the drop-in matcher pops from (ugpu_find_records:
            # pipelined H2D + scans + packed records into pinned memory), every
            # record decoded natively (ugpu_records_drain)
            U.Records(pat, buf).drain()  # warm (pinned pool, workspaces)
            bestr = 1e30
            for _ in range(a.reps):
                t0 = time.perf_counter()
                rr = U.Records(pat, buf)
                got = rr.drain()
                bestr = min(bestr, time.perf_counter() - t0)
                rr.close()
            line["records_ms"] = round(bestr * 1e3, 4)
            line["records_gbps"] = round(n / bestr / 1e9, 3)
            line["records_equal"] = got == (r.count, r.digest, r.dcap)
            # the same with a borrowed buffer (UGPU_REC_BORROW: the consumer
            # starts at the first piece, not after the whole H2D; a native
            # consumer that owns its buffer, not ugrep's mmap)
            bestb = 1e30
            for _ in range(a.reps):
                t0 = time.perf_counter()
                rr = U.Records(pat, buf, borrow=True)
                gotb = rr.drain()
                bestb = min(bestb, time.perf_counter() - t0)
                rr.close()
            line["records_borrow_ms"] = round(bestb * 1e3, 4)
            line["records_borrow_gbps"] = round(n / bestb / 1e9, 3)
            line["records_borrow_equal"] = gotb == (r.count, r.digest, r.dcap)
            if os.path.exists(exe):
                j = json.loads(subprocess.run([exe, "bench", "re", rx, "gen:%d:1:0:%d" % (kind, n), "1", str(a.reps)],
                                              capture_output=True, check=True, timeout=600).stdout.decode()
                               .strip().splitlines()[-1])
                line["cpu_ms"] = round(j["seconds"] * 1e3, 4)
                line["cpu_gbps"] = round(n / j["seconds"] / 1e9, 3)
                line["equal_count"] = j["count"] == r.count
                if cross is None and j["seconds"] > min(best, bestr):
                    cross = n
            print(json.dumps(line), flush=True)
        summary[name] = cross
    print(json.dumps({"crossover_bytes": summary, "note": "smallest size where the GPU host-buffer path beats one "
                      "reference CPU matcher (None: never within the sizes measured)"}), flush=True)


if __name__ == "__main__":
    main()
