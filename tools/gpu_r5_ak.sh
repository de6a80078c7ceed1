# round 5: the word-start filter for word-boundary tables when only
# byte-reachable states count (default) against all states (UGPU_WSTART_REACH=0)
set -o pipefail
out=gpurun_out/r5ak; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_wordb.py tests/test_anchor.py tests/test_records.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rr in 1 0; do
for spec in 'bfoo:\bfoo\b' 'inut:\<(in|ut)\>' 'bthe:\b(the|and|of)\b' 'ing_e:ing\>'; do
  name=${spec%%:*}; rx=${spec#*:}
  UGPU_WSTART_REACH=$rr timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.$rr.json 2> $out/$name.$rr.err || { tail -5 $out/$name.$rr.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.$rr.json')); r=d['roofline']
print('reach=$rr', d['config']['pattern'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['matches'])"
done
done
