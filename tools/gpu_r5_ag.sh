# round 5, closing: the C2 pattern lines on the final build (one more box)
set -o pipefail
out=gpurun_out/r5ag; mkdir -p $out
for spec in 'bfoo:\bfoo\b:' 'inut:\<(in|ut)\>:' 'wing:[a-z]+ing:--word' 'ing:[a-z]+ing:' 'tion:[A-Za-z]+tion:' 'wazAZ:[A-Za-z]+:--word'; do
  name=${spec%%:*}; rest=${spec#*:}; rx=${rest%:*}; flag=${rest##*:}
  timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" $flag --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.json 2> $out/$name.err || { tail -5 $out/$name.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.json')); r=d['roofline']
print('$name', d['config']['pattern'], '$flag', d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['matches'])"
done
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > $out/c4.json 2> $out/c4.err || { tail -5 $out/c4.err; exit 1; }
python -c "
import json; d=json.load(open('$out/c4.json')); r=d['roofline']; print('c4', d['ms_per_step'], r['kernel_ms'], r['frac'])"
