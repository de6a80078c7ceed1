# round 5: W / context walks reading the candidate's LDS window (libugrep_amd.so)
# against global-memory walks (libugrep_amd_ool0.so); W / word-boundary tests
set -o pipefail
out=gpurun_out/r5w; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_word.py tests/test_wordb.py tests/test_anchor.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for lib in libugrep_amd.so libugrep_amd_ool0.so; do
for spec in 'bfoo:\bfoo\b:' 'inut:\<(in|ut)\>:'; do
  name=${spec%%:*}; rest=${spec#*:}; rx=${rest%:*}; flag=${rest##*:}
  UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config c2 --regex "$rx" $flag --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$name.$lib.$rep.json 2> $out/$name.$lib.$rep.err || { tail -5 $out/$name.$lib.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$name.$lib.$rep.json')); r=d['roofline']
print('$lib', d['config']['pattern'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['matches'])"
done
done
done
echo done
