#!/bin/bash
# round 6: end-of-word candidate filter (ScanParams::wend) for fixed-length word-boundary tables
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6l; rm -rf $out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_wordb.py tests/test_word.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -2
for rx in '\<(in|ut)\>' '\bfoo\b' '\b(in|ut)\b'; do
  for we in 1 0 1 0; do
    n=$(echo "$rx" | tr -dc 'a-z')
    UGPU_WEND=$we timeout -k 10 300 python3 bench.py --config c2 --regex "$rx" --no-cpu-baseline --pcie-sample-mib 0 > $out/b_${n}_$we.json 2> $out/b_${n}_$we.err || { tail -5 $out/b_${n}_$we.err; exit 1; }
    python3 -c "import json;j=json.load(open('$out/b_${n}_$we.json'));print('$rx wend=$we', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])" | tee -a $out/summary.txt
  done
done
