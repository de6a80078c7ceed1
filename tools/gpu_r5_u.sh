# round 5: OFFSETS expansion variants (non-temporal stores, 8 waves/SIMD, 512-entry
# staging) against the default, and the store probe with non-temporal stores
set -o pipefail
out=gpurun_out/r5u; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_c5.py::test_offsets_record_by_record tests/test_xc.py tests/test_xu.py tests/test_redo.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
for lib in libugrep_amd_clamp.so; do
  UGPU_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_c5.py::test_offsets_record_by_record tests/test_xc.py tests/test_xu.py tests/test_redo.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests_$lib.log 2>&1 || { tail -30 $out/tests_$lib.log; exit 1; }
done
tail -1 $out/tests.log
for rep in 1 2; do
for cfg in c4 c3; do
for lib in libugrep_amd.so libugrep_amd_clamp.so; do
  UGPU_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --offsets --no-cpu-baseline --pcie-sample-mib 0 > $out/$cfg.$lib.$rep.json 2> $out/$cfg.$lib.$rep.err || { tail -5 $out/$cfg.$lib.$rep.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$cfg.$lib.$rep.json')); print('$cfg $lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['offsets']['digest_matches_totals'])"
done
done
done
echo done
