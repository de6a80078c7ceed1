#!/usr/bin/env python3
"""Condense a tools/profile.sh run (rocprofv3 rocpd SQLite output) into JSON:
per-kernel stats from the kernel-trace pass (the --stats summary) and, for the
dominant scan kernel, the PMC counters of its last dispatch.

FETCH_SIZE is reported in KB by rocprofv3 and, on gfx950, counts half the bytes
of 16 B/lane streaming reads (MI355X_MICROARCH.md, HBM section): the HBM bytes
are FETCH_SIZE * 1024 * 2."""
import glob
import json
import os
import sqlite3
import sys


def db(d, sub):
    f = glob.glob(os.path.join(d, sub, "**", "*.db"), recursive=True)
    return sqlite3.connect(f[0]) if f else None


def main(d, match=("sparse_kernel", "dense_kernel", "xi_kernel", "xg_kernel", "xc_kernel", "scan_kernel")):
    kernels = []
    c = db(d, "trace")
    if c:
        for name, calls, total, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            kernels.append({"name": name, "calls": calls, "total_us": round(total, 3), "avg_us": round(avg, 3),
                            "pct": round(pct, 3)})
    scan = [k for k in kernels if any(n in k["name"] for n in match)]
    dom = max(scan, key=lambda k: k["total_us"]) if scan else None
    counters = {}
    for sub in ("pmc1", "pmc2", "pmc3"):
        c = db(d, sub)
        if not c or not dom:
            continue
        last = c.execute("select max(dispatch_id) from counters_collection where kernel_name = ?",
                         (dom["name"],)).fetchone()[0]
        for name, val in c.execute("select counter_name, sum(value) from counters_collection "
                                   "where kernel_name = ? and dispatch_id = ? group by counter_name",
                                   (dom["name"], last)):
            counters[name] = val
    bench = None
    try:
        with open(os.path.join(d, "bench.json")) as fh:
            bench = json.loads(fh.read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        pass
    res = {"kernels": kernels, "dominant": dom, "counters_last_dispatch": counters}
    if bench:
        res["bench"] = {k: bench[k] for k in ("value", "ms_per_step", "matches", "roofline", "config") if k in bench} \
            if "roofline" in bench else bench
    if "FETCH_SIZE" in counters:
        res["hbm_bytes_per_launch"] = int(counters["FETCH_SIZE"] * 1024 * 2)
        if bench and "roofline" in bench:
            alg = bench["roofline"]["algorithmic_bytes_per_launch"]
            res["algorithmic_bytes_per_launch"] = alg
            res["traffic_over_algorithmic"] = round(res["hbm_bytes_per_launch"] / alg, 4)
    if "GRBM_GUI_ACTIVE" in counters and dom:
        res["effective_clock_ghz"] = round(counters["GRBM_GUI_ACTIVE"] / 8 / (dom["avg_us"] * 1e3), 3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    # usage: pmc_summary.py DIR [kernel-name-substring ...]
    main(sys.argv[1], tuple(sys.argv[2:]) or ("sparse_kernel", "dense_kernel", "xi_kernel", "xg_kernel", "xc_kernel", "scan_kernel"))
