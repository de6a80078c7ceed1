#!/usr/bin/env python3
"""Throughput of the line-level consumers (ugpu_lines)
over a config's synthetic corpus resident in HBM.

The match starts come from one FIND scan (ugpu_scan + ugpu_scan_offsets) into
device arrays, as a line-mode ugrep consumer would get them; then each timed
step is one ugpu_lines call (newline count pass, host prefix of the per-wave
counts, line assignment pass, -c stitch).  Algorithmic bytes: the buffer is
read once plus 16 B per match (start read, line
written).  Prints one JSON line.  Profile with rocprofv3 --kernel-trace --stats
for the nl_count_kernel / nl_assign_kernel durations.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import ugrep_amd  # noqa: E402

CONFIGS = {"c2": ("c2_foobarbaz", 1, 16 << 30), "c3": ("c3_ident", 3, 4 << 30), "c4": ("c4_word", 4, 4 << 30)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--bytes", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    pkey, kind, size = CONFIGS[args.config]
    n = args.bytes or size
    with open(os.path.join(REPO, "ugrep_amd", "data", "config_patterns.json")) as f:
        opc = json.load(f)[pkey]["opc"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    buf = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    ugrep_amd.gen(kind, 1, 0, buf.data_ptr(), n, sptr)
    pat = ugrep_amd.Pattern(opc)
    sc = ugrep_amd.Scanner(pat)
    sc.scan(buf.data_ptr(), 0, n, n, True, 0, sptr)
    t = sc.totals()
    m = t.count
    starts = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
    lens = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    caps = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    sc.offsets(starts.data_ptr(), lens.data_ptr(), caps.data_ptr(), m, sptr)
    del lens, caps
    lines = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        nl, ml = ugrep_amd.lines(buf.data_ptr(), n, starts.data_ptr(), m, lines.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nl, ml = ugrep_amd.lines(buf.data_ptr(), n, starts.data_ptr(), m, lines.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / args.steps
    # sanity (not timed): newline count against torch, line numbers non-decreasing
    nl_torch = int((buf[:n] == 10).sum().item())
    mono = bool((lines[1:m] >= lines[:m - 1]).all().item()) if m > 1 else True
    alg = n + 16 * m  # every byte read once + start read + line written per match
    print(json.dumps({
        "what": "ugpu_lines (newline count + match line numbers + matching-line count)",
        "config": args.config, "bytes": n, "matches": m, "newlines": nl, "matching_lines": ml,
        "newlines_ok": nl == nl_torch, "lines_monotone": mono,
        "ms_per_call": round(el * 1e3, 4), "GBps_input": round(n / el / 1e9, 1),
        "GBps_algorithmic": round(alg / el / 1e9, 1), "algorithmic_bytes": alg}), flush=True)


if __name__ == "__main__":
    main()
