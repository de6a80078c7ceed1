#!/usr/bin/env python3
"""Update profiles/traffic.json (read by bench.py for roofline.traffic) from a
tools/profile.sh summary: python tools/traffic_from_summary.py CONFIG SUMMARY.json

HBM bytes per launch = FETCH_SIZE (KB, last dispatch of the dominant scan
kernel) x 1024 x 2 -- the gfx950 wide-read correction of MI355X_MICROARCH.md's
HBM / rocprofv3 section."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg, summ = sys.argv[1], sys.argv[2]
d = json.load(open(summ))
fetch = d["counters_last_dispatch"]["FETCH_SIZE"] * 1024 * 2
alg = d["bench"]["roofline"]["algorithmic_bytes_per_launch"]
names = [k["name"] for k in d["kernels"] if d["bench"]["roofline"]["kernel"] in k["name"]]
path = os.path.join(REPO, "profiles", "traffic.json")
t = json.load(open(path))
t[cfg] = {"hbm_bytes_per_launch": int(fetch), "algorithmic_bytes_per_launch": alg,
          "traffic_over_algorithmic": round(fetch / alg, 4), "kernel": names[0] if names else "",
          "source": "%s: rocprofv3 --kernel-trace --pmc FETCH_SIZE, last dispatch, KB x 1024 x 2 (gfx950 wide-read "
                    "correction)" % os.path.relpath(summ, REPO)}
json.dump(t, open(path, "w"), indent=1)
print(cfg, t[cfg])
