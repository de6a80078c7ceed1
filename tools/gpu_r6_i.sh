#!/bin/bash
# round 6: option W subset mode on xc_kernel: tests, then the C2 -w '[A-Za-z]+' bench line
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6i; rm -rf $out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_wsub.py tests/test_word.py tests/test_xc.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -2
for rx in '[A-Za-z]+' '[a-z]+'; do
  n=$(echo "$rx" | tr -dc 'a-zA-Z')
  timeout -k 10 300 python3 bench.py --config c2 --regex "$rx" --word --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_w_$n.json 2> $out/bench_w_$n.err || { tail -5 $out/bench_w_$n.err; exit 1; }
  python3 -c "import json;j=json.load(open('$out/bench_w_$n.json'));print('$rx -w', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'])"
done
