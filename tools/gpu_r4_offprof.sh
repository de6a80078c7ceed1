#!/bin/bash
# round 4: kernel trace of the OFFSETS steps (bitmap expansion on)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in c4 c3; do
  UGPU_XC_BITMAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_offprof_$c -o run --output-format csv -- python3 bench.py --config $c --offsets --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_offprof_$c.log 2>&1 || { tail -5 gpurun_out/r4_offprof_$c.log; exit 1; }
  f=$(ls gpurun_out/r4_offprof_$c/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && head -8 "$f" | cut -d, -f1-4
done
