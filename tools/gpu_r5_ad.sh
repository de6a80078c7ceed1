# round 5: option W without a selective prefilter on sparse_kernel
# (default; UGPU_WSPARSE=0: wfind_kernel): GPU tests, then C2 bench lines
set -o pipefail
out=gpurun_out/r5ad; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests/test_word.py tests/test_multi.py tests/test_stream.py tests/test_records.py tests/test_plan.py tests/test_lookback.py tests/test_c5.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for ws in 1 0; do
for spec in 'azAZ:[A-Za-z]+' 'az09:[a-z]+[0-9]*'; do
  name=${spec%%:*}; rx=${spec#*:}
  UGPU_WSPARSE=$ws timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" --word --steps 3 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.$ws.json 2> $out/$name.$ws.err || { tail -5 $out/$name.$ws.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.$ws.json')); r=d['roofline']
print('wsparse=$ws', d['config']['pattern'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['matches'])"
done
done
echo done
