#!/usr/bin/env python3
"""Summarise a tools/gpu_sweep.sh run: per library, kernel ms, HBM fraction and
FETCH_SIZE bytes (x1024 x2, gfx950) of the dominant scan kernel's last dispatch."""
import glob
import json
import os
import sqlite3
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    lib = os.path.basename(f)[:-5]
    try:
        b = json.load(open(f))
    except ValueError:
        continue
    k = b["roofline"]["kernel"]
    fetch = None
    dbs = glob.glob(os.path.join(d, "pmc_" + lib, "**", "*.db"), recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        row = c.execute("select kernel_name, max(dispatch_id) from counters_collection where kernel_name like ? ",
                        ("%" + k + "%",)).fetchone()
        if row and row[1] is not None:
            v = c.execute("select sum(value) from counters_collection where dispatch_id = ? and counter_name = "
                          "'FETCH_SIZE'", (row[1],)).fetchone()[0]
            fetch = v * 1024 * 2
    alg = b["roofline"]["algorithmic_bytes_per_launch"]
    print("%-28s %s ms %.2f frac %.4f fetch/alg %s digest %s" % (lib, k, b["roofline"]["kernel_ms"], b["roofline"]["frac"],
                                                               "%.3f" % (fetch / alg) if fetch else "-", b["digest"]))
