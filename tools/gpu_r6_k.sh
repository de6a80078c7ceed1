#!/bin/bash
# round 6: OFFSETS with the next batch's COUNT overlapping the record expansion (bench --offsets-pipeline), A/B
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6k; rm -rf $out; mkdir -p $out
for cfg in c4 c3; do
  for mode in on off on off; do
    timeout -k 10 300 python3 bench.py --config $cfg --offsets --offsets-pipeline $mode --no-cpu-baseline --pcie-sample-mib 0 --steps 10 --warmup 3 > $out/b_${cfg}_$mode.json 2> $out/b_${cfg}_$mode.err || { tail -20 $out/b_${cfg}_$mode.err; exit 1; }
    python3 -c "import json;j=json.load(open('$out/b_${cfg}_$mode.json'));print('$cfg', '$mode', j['ms_per_step'], j['roofline']['kernel_ms'], j['offsets'])" | tee -a $out/summary.txt
  done
done
