# round 5: byte-major In bits (bm_pack / bm_unpack, libugrep_amd.so) against
# nib16's multiply gather (libugrep_amd_old.so): OFFSETS tests, then C4 / C3
set -o pipefail
out=gpurun_out/r5ai; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_xc.py tests/test_xu.py tests/test_c5.py tests/test_records.py tests/test_gpu.py tests/test_xc_host.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for lib in libugrep_amd_old.so libugrep_amd.so; do
for c in c4 c3; do
  UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --offsets --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$c.$lib.$rep.json 2> $out/$c.$lib.$rep.err || { tail -5 $out/$c.$lib.$rep.err; exit 1; }
  python -c "import json;j=json.load(open('$out/$c.$lib.$rep.json'));print('$lib $c', j['ms_per_step'], j['roofline']['kernel_ms'], j['offsets']['digest_matches_totals'])"
done
done
done
