#!/bin/bash
# round 5 closing measurement (one MI355X):
#   per config (c2 = the default command, c3, c4): the exact bench command under a
#   trace-only rocprofv3 pass (the line and its kernel times come from the same
#   run), then one FETCH_SIZE pass (HBM bytes per launch); the OFFSETS lines;
#   tools/pmc_summary.py condenses each config into gpurun_out/r05e/<c>/summary.json
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r05e
rm -rf $out; mkdir -p $out
for c in c2 c3 c4; do
  d=$out/$c; mkdir -p $d
  if [ $c = c2 ]; then a=""; else a="--config $c"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/trace -o run -- python3 -u bench.py $a > $d/bench.json 2> $d/bench.err || { tail $d/bench.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $d/pmc1 -o run -- python3 -u bench.py $a --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $d/pmc1.json 2> $d/pmc1.err || { tail $d/pmc1.err; exit 1; }
  python3 tools/pmc_summary.py $d > $d/summary.json
  python3 -c "import json;s=json.load(open('$d/summary.json'));b=s['bench'];print('$c', b['ms_per_step'], b['value'], s.get('kernel_ms'), s.get('kernel_ms_bench'), s.get('traffic_over_algorithmic'))"
done
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --offsets --no-cpu-baseline --pcie-sample-mib 0 > $out/offsets_$c.json 2> $out/offsets_$c.err || { tail $out/offsets_$c.err; exit 1; }
  python3 -c "import json;j=json.load(open('$out/offsets_$c.json'));print('$c offsets', j['ms_per_step'], j['offsets'])"
done
