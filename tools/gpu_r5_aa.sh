# round 5: context walks on sparse_kernel: 4 waves per SIMD without spills
# (o4), the candidate's LDS window (o4w), acap/amap in LDS (UGPU_SP_ACAP_LDS)
set -o pipefail
out=gpurun_out/r5aa; mkdir -p $out
UGPU_LIB=libugrep_amd_o4w.so timeout -k 10 600 python -u -m pytest tests/test_wordb.py tests/test_anchor.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for cfg in libugrep_amd.so:0 libugrep_amd.so:1 libugrep_amd_o4.so:1 libugrep_amd_o4w.so:0 libugrep_amd_o4w.so:1; do
lib=${cfg%%:*}; al=${cfg##*:}
for spec in 'bfoo:\bfoo\b' 'inut:\<(in|ut)\>'; do
  name=${spec%%:*}; rx=${spec#*:}
  UGPU_SP_ACAP_LDS=$al UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.$lib.$al.$rep.json 2> $out/$name.$lib.$al.$rep.err || { tail -5 $out/$name.$lib.$al.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.$lib.$al.$rep.json')); r=d['roofline']
print('$lib acap_lds=$al', d['config']['pattern'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['matches'])"
done
done
done
echo done
