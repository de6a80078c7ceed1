# round 5: the plain sparse kernel at 6 (default, 3 spilled VGPRs) / 5 / 4
# blocks per CU (no spills): C2 and -w '[a-z]+ing'
set -o pipefail
out=gpurun_out/r5al; mkdir -p $out
for rep in 1 2; do
for lib in libugrep_amd.so libugrep_amd_p5.so libugrep_amd_p4.so; do
for spec in 'c2::' 'wing:[a-z]+ing:--word'; do
  name=${spec%%:*}; rest=${spec#*:}; rx=${rest%:*}; flag=${rest##*:}
  if [ -n "$rx" ]; then a="--regex $rx $flag"; else a=""; fi
  UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config c2 $a --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.$lib.$rep.json 2> $out/$name.$lib.$rep.err || { tail -5 $out/$name.$lib.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.$lib.$rep.json')); r=d['roofline']
print('$lib', d['config']['pattern'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
done
done
