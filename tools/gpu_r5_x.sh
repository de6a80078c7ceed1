# round 5: loop-needle lookback (sparse_kernel lb_batch): parity tests, then
# bench A/B of -w '[a-z]+ing' and '[a-z]+ing' with UGPU_LB=1 / 0
set -o pipefail
out=gpurun_out/r5x; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_lookback.py tests/test_plan.py -x -v --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for lb in 1 0; do
for spec in 'tion:[A-Za-z]+tion:' 'hing:[a-z-]+ing:' 'wtion:[A-Za-z]+tion:--word'; do
  name=${spec%%:*}; rest=${spec#*:}; rx=${rest%:*}; flag=${rest##*:}
  UGPU_LB=$lb timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" $flag --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.$lb.json 2> $out/$name.$lb.err || { tail -5 $out/$name.$lb.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.$lb.json')); r=d['roofline']
print('lb=$lb', d['config']['pattern'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['matches'])"
done
done
echo done
