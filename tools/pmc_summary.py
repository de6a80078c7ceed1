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


def main(d, match=("sparse_kernel", "dense_kernel", "xi_kernel", "xg_kernel", "xc_kernel", "xu_kernel", "scan_kernel")):
    kernels = []
    c = c_trace = db(d, "trace")
    if c:
        for name, calls, total, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            kernels.append({"name": name, "calls": calls, "total_us": round(total, 3), "avg_us": round(avg, 3),
                            "pct": round(pct, 3)})
    scan = [k for k in kernels if any(n in k["name"] for n in match)]
    dom = max(scan, key=lambda k: k["total_us"]) if scan else None
    # the bench's own scan dispatches only: the persistent grids do not tell a
    # full-size launch from a smaller one (a PCIe-leg or reference-check
    # sample), so keep the dispatches within 25 % of the longest one
    if c and dom:
        durs = [r[0] / 1e3 for r in c.execute("select duration from kernels where name = ? order by dispatch_id",
                                              (dom["name"],))]
        if durs:
            top = max(durs)
            main_ = [x for x in durs if x >= 0.75 * top]
            dom["main_dispatches"] = len(main_)
            dom["other_dispatches"] = len(durs) - len(main_)
            dom["main_avg_us"] = round(sum(main_) / len(main_), 3)
    counters = {}
    for sub in ("pmc1", "pmc2", "pmc3"):
        c = db(d, sub)
        if not c or not dom:
            continue
        rows = c.execute("select dispatch_id, max(duration) from counters_collection where kernel_name = ? "
                         "group by dispatch_id order by dispatch_id", (dom["name"],)).fetchall()
        if not rows:
            continue
        top = max(r[1] for r in rows)
        last = [r[0] for r in rows if r[1] >= 0.75 * top][-1]  # the last full-size dispatch
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
    # the timed steps' dispatches: the last `steps` full-size ones (before them
    # come the warmup steps and the first launch, slower while clocks ramp)
    if dom and bench and "main_dispatches" in dom and c_trace:
        steps = int(bench.get("steps", 0))
        durs = [r[0] / 1e3 for r in c_trace.execute("select duration from kernels where name = ? order by dispatch_id",
                                                    (dom["name"],))]
        top = max(durs)
        main_ = [x for x in durs if x >= 0.75 * top]
        if steps and len(main_) >= steps:
            dom["timed_dispatches"] = steps
            dom["timed_avg_us"] = round(sum(main_[-steps:]) / steps, 3)
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
        res["effective_clock_ghz"] = round(counters["GRBM_GUI_ACTIVE"] / 8 / (dom.get("main_avg_us", dom["avg_us"]) * 1e3), 3)
    if dom and "main_avg_us" in dom:
        res["kernel_ms"] = round(dom.get("timed_avg_us", dom["main_avg_us"]) / 1e3, 4)
        if bench and "roofline" in bench:
            # the trace's average against the bench line's HIP-event time of the same command
            res["kernel_ms_bench"] = bench["roofline"].get("kernel_ms")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    # usage: pmc_summary.py DIR [kernel-name-substring ...]
    main(sys.argv[1], tuple(sys.argv[2:]) or ("sparse_kernel", "dense_kernel", "xi_kernel", "xg_kernel", "xc_kernel", "xu_kernel", "scan_kernel"))
