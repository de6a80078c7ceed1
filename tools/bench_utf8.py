#!/usr/bin/env python3
"""Throughput of binary-file detection (ugpu_check_utf8 / ugpu_find_nul,
SURVEY.md §8f row 4) over a synthetic corpus resident in HBM.

Each timed step is one synchronous call over the whole buffer (memset of the
result slot, utf8_kernel, 8-byte read-back).  The corpus is valid (no failing
byte), so the whole buffer is read: algorithmic bytes = buffer bytes.
--config c4 = UTF-8 words (every tile takes the exact per-byte test),
c3 = ASCII source code (the pure-ASCII fast path).  Prints one JSON line;
profile with rocprofv3 --kernel-trace --stats for utf8_kernel's duration.
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

KINDS = {"c2": 1, "c3": 3, "c4": 4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=sorted(KINDS))
    ap.add_argument("--bytes", type=int, default=16 << 30)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nul", action="store_true", help="time the NUL search (-a/-U) instead of isutf8")
    args = ap.parse_args()
    n = args.bytes
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    buf = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    ugrep_amd.gen(KINDS[args.config], 1, 0, buf.data_ptr(), n, sptr)
    torch.cuda.synchronize(dev)
    fn = ugrep_amd.find_nul if args.nul else ugrep_amd.check_utf8
    for _ in range(args.warmup):
        r = fn(buf.data_ptr(), n, sptr)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = fn(buf.data_ptr(), n, sptr)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / args.steps
    print(json.dumps({
        "what": "ugpu_find_nul (memchr NUL)" if args.nul else "ugpu_check_utf8 (reflex::isutf8)",
        "config": args.config, "bytes": n, "result": r, "ms_per_call": round(el * 1e3, 4),
        "GBps": round(n / el / 1e9, 1), "hbm_frac": round(n / el / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
