# round 5: nib16 by shifts (libugrep_amd_nb.so) against the multiply, OFFSETS C4 / C3
set -o pipefail
out=gpurun_out/r5af; mkdir -p $out
UGPU_LIB=libugrep_amd_nb.so timeout -k 10 300 python -u -m pytest tests/test_xc.py tests/test_xu.py -x -q --timeout 200 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for lib in libugrep_amd.so libugrep_amd_nb.so; do
for c in c4 c3; do
  UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --offsets --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$c.$lib.$rep.json 2> $out/$c.$lib.$rep.err || { tail -5 $out/$c.$lib.$rep.err; exit 1; }
  python -c "import json;j=json.load(open('$out/$c.$lib.$rep.json'));print('$lib $c', j['ms_per_step'], j['roofline']['kernel_ms'], j['offsets']['digest_matches_totals'])"
done
done
done
