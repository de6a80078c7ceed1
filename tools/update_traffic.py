#!/usr/bin/env python3
"""Write a profiles/traffic.json entry from a tools/profile.sh summary
(tools/pmc_summary.py output): HBM bytes per launch of the dominant kernel's
last full-size dispatch, and that kernel's trace-average time, which bench.py
compares with its own HIP-event time before using the entry (±5 %).

    python tools/update_traffic.py CONFIG profiles/rNN_cX_summary.json"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(cfg, summary):
    s = json.load(open(os.path.join(REPO, summary)))
    p = os.path.join(REPO, "profiles", "traffic.json")
    t = json.load(open(p)) if os.path.exists(p) else {}
    t[cfg] = {"hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
              "algorithmic_bytes_per_launch": s["algorithmic_bytes_per_launch"],
              "traffic_over_algorithmic": s["traffic_over_algorithmic"],
              "kernel": s["dominant"]["name"], "kernel_ms": s.get("kernel_ms"),
              "source": "%s: rocprofv3 --kernel-trace --pmc FETCH_SIZE, last full-size dispatch, KB x 1024 x 2 "
                        "(gfx950 wide-read correction)" % summary}
    json.dump(t, open(p, "w"), indent=1)
    print(json.dumps(t[cfg]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
