#!/bin/bash
# round 6: trace-only kernel summaries of the needle-set lookback bench lines
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6pl; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/inged -o run -- python3 bench.py --config c2 --regex '[a-z]+(ing|ed)' --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/inged.json 2> $out/inged.err || { tail -5 $out/inged.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tion -o run -- python3 bench.py --config c2 --regex '[A-Za-z]+(tion|sion|ment|ness)' --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/tion.json 2> $out/tion.err || { tail -5 $out/tion.err; exit 1; }
find $out -name '*kernel_stats.csv' | head
