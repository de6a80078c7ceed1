#!/bin/bash
# round 6: where a 5000-byte needle-free run's time goes (dominated restarts on/off)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r6c; rm -rf $out; mkdir -p $out
timeout -k 10 300 python3 -u tools/dbg_dom.py > $out/dbg.txt 2>&1 || { tail -30 $out/dbg.txt; exit 1; }
cat $out/dbg.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 -u tools/dbg_dom.py 1 > $out/prof.txt 2>&1 || { tail -30 $out/prof.txt; exit 1; }
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); head -20 "$f"
