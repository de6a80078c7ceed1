# round 5: word-start candidate filter (P.wstart) -- W / word-boundary tests,
# then the three word bench lines (c2 corpus, 16 GiB) with it on and off
set -o pipefail
out=gpurun_out/r5j; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_word.py tests/test_wordb.py tests/test_stream.py tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for ws in 1 0; do
  i=0
  for spec in 'bfoo:\bfoo\b:' 'inut:\<(in|ut)\>:' 'wing:[a-z]+ing:--word'; do
    name=${spec%%:*}; rest=${spec#*:}; rx=${rest%:*}; flag=${rest##*:}
    UGPU_WSTART=$ws timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" $flag --steps 5 --warmup 2 --cpu-sample-mib 256 --pcie-sample-mib 0 > $out/wb_${name}_ws$ws.json 2> $out/wb_${name}_ws$ws.err || { tail -5 $out/wb_${name}_ws$ws.err; exit 1; }
    python -c "
import json; d=json.load(open('$out/wb_${name}_ws$ws.json')); r=d['roofline']
print('ws=$ws', d['config']['pattern'], d['config']['word'], d['ms_per_step'], r['kernel'], r['frac'], d['matches'], (d.get('parity_vs_reference') or {}).get('equal'), d['cpu_baseline']['value'])"
  done
done
echo done
