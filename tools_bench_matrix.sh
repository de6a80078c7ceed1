#!/bin/bash
# quick matrix: config:ablate pairs; prints config, GB/s, matches, roofline frac, kernel ms
for spec in "$@"; do
  c=${spec%%:*}; a=${spec#*:}; [ "$a" = "$spec" ] && a=0
  UGPU_ABLATE=$a timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline 2>gpurun_out/bench_${c}_$a.err > gpurun_out/bench_${c}_$a.json || { echo "bench $spec failed"; tail -3 gpurun_out/bench_${c}_$a.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bench_${c}_$a.json')); print('$spec', j['value'], j['matches'], j['roofline']['frac'], j['roofline']['kernel_ms'])"
done
