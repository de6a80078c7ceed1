#!/bin/bash
# Quick benchmark matrix on the GPU box.  Each spec is config[:ablate[:filter_levels]]
# (UGPU_ABLATE / UGPU_FILTER_LEVELS are benchmarking knobs; results of ablated
# runs are not valid matches).  Prints: spec, GB/s, matches, roofline frac, kernel ms.
for spec in "$@"; do
  IFS=: read -r c a l <<< "$spec"
  a=${a:-0}
  tag="${c}_${a}_${l:-d}"
  env UGPU_ABLATE=$a ${l:+UGPU_FILTER_LEVELS=$l} timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 \
      --no-cpu-baseline 2>gpurun_out/bench_$tag.err > gpurun_out/bench_$tag.json \
    || { echo "bench $spec failed"; tail -3 gpurun_out/bench_$tag.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/bench_$tag.json')); print('$spec', j['value'], j['matches'], j['roofline']['frac'], j['roofline']['kernel_ms'])"
done
