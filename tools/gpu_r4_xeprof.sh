#!/bin/bash
# round 4: kernel times of the OFFSETS passes (trace only)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xeprof_$c -o run -- python3 -u bench.py --config $c --offsets --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/xeprof_$c.json 2> gpurun_out/xeprof_$c.err || { tail gpurun_out/xeprof_$c.err; exit 1; }
  f=$(find gpurun_out/xeprof_$c -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
r.sort(key=lambda x:-float(x['TotalDurationNs']))
for x in r[:6]: print('$c', x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e6,4))
"
done
