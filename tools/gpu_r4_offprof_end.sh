#!/bin/bash
# round 4 closing: trace-only kernel summaries of the exact OFFSETS commands
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r04o
rm -rf $out; mkdir -p $out
for c in c4 c3; do
  d=$out/$c; mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/trace -o run -- python3 -u bench.py --config $c --offsets --no-cpu-baseline --pcie-sample-mib 0 > $d/bench.json 2> $d/bench.err || { tail $d/bench.err; exit 1; }
  python3 tools/pmc_summary.py $d xc_expand_kernel > $d/summary.json
  python3 -c "
import json;s=json.load(open('$d/summary.json'))
print('$c', s['bench']['ms_per_step'] if 'ms_per_step' in s['bench'] else s['bench'])
for k in s['kernels'][:5]: print('   ', k['name'][:50], k['calls'], k['avg_us'])"
done
