#!/bin/bash
# round 6: loop-needle lookback over needle sets (C+ (N1|N2|...)): GPU tests, then
# A/B bench lines on C2 (16 GiB) with the lookback on and off
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6w2; rm -rf $out; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lookback.py tests/test_dom.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for rx in '[a-z]+(ing|ed)' '[A-Za-z]+(tion|sion|ment|ness)' '[a-z]+ing'; do
  for lb in 1 0; do
    n=$(echo "$rx" | tr -c 'a-zA-Z0-9' '_')
    UGPU_LB=$lb timeout -k 10 300 python3 bench.py --config c2 --regex "$rx" --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/b_${n}_$lb.json 2> $out/b_${n}_$lb.err || { tail -5 $out/b_${n}_$lb.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['frac'], d.get('matches', d.get('count')))" $out/b_${n}_$lb.json "$rx" $lb
  done
done
timeout -k 10 300 python3 bench.py --config c2 --regex '[a-z]+(ing|ed)' --word --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/b_w_inged.json 2> $out/b_w_inged.err || { tail -5 $out/b_w_inged.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/b_w_inged.json')); print('-w inged', d['ms_per_step'], d['roofline']['frac'])"
