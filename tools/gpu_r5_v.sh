# round 5: C4 U-mode lookups into 16-bit register halves (ds_read_u8_d16/_hi,
# one v_lshl_or per dword) against the default; U-mode tests on the variant
set -o pipefail
out=gpurun_out/r5v; mkdir -p $out
UGPU_LIB=libugrep_amd_d16.so timeout -k 10 600 python -u -m pytest tests/test_xu.py tests/test_c5.py::test_offsets_record_by_record tests/test_word.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do
for lib in libugrep_amd.so libugrep_amd_d16.so; do
  UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 > $out/$lib.$rep.json 2> $out/$lib.$rep.err || { tail -5 $out/$lib.$rep.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$lib.$rep.json')); print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['digest'])"
done
done
echo done
