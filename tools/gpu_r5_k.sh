# round 5: the whole GPU suite, smoke, and the word bench lines
set -o pipefail
out=gpurun_out/r5k; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -10 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
for spec in 'bfoo:\bfoo\b:' 'inut:\<(in|ut)\>:' 'wing:[a-z]+ing:--word'; do
  name=${spec%%:*}; rest=${spec#*:}; rx=${rest%:*}; flag=${rest##*:}
  timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" $flag --steps 5 --warmup 2 --cpu-sample-mib 256 --pcie-sample-mib 0 > $out/wb_${name}.json 2> $out/wb_${name}.err || { tail -5 $out/wb_${name}.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/wb_${name}.json')); r=d['roofline']
print(d['config']['pattern'], d['config']['word'], d['ms_per_step'], r['kernel'], r['frac'], d['matches'], (d.get('parity_vs_reference') or {}).get('equal'), d['cpu_baseline']['value'])"
done
echo done
