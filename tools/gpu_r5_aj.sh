# round 5: the COUNT pass's In bits stored per chunk (libugrep_amd_xd.so)
# against LDS staging + per-tile stores (libugrep_amd.so): OFFSETS C3 / C4
set -o pipefail
out=gpurun_out/r5aj; mkdir -p $out
UGPU_LIB=libugrep_amd_xd.so timeout -k 10 600 python -u -m pytest tests/test_xc.py tests/test_xu.py tests/test_c5.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for lib in libugrep_amd.so libugrep_amd_xd.so; do
for c in c3 c4; do
  UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --offsets --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$c.$lib.$rep.json 2> $out/$c.$lib.$rep.err || { tail -5 $out/$c.$lib.$rep.err; exit 1; }
  python -c "import json;j=json.load(open('$out/$c.$lib.$rep.json'));print('$lib $c', j['ms_per_step'], j['roofline']['kernel_ms'], j['offsets']['digest_matches_totals'])"
done
done
done
