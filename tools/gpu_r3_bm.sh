# Round 3: OFFSETS from the COUNT pass's In bits (UGPU_XC_BITMAP=1) against
# the WRITE pass, C4 and C3, then the record tests with the bitmap on.
set -o pipefail
out=gpurun_out/${1:-r3bm}
mkdir -p $out
b="--steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0"
for c in c4 c3; do
  for bm in 1 0; do
    UGPU_XC_BITMAP=$bm timeout -k 10 200 python bench.py --config $c --offsets $b > $out/${c}_bm$bm.json 2> $out/${c}_bm$bm.err || { tail -8 $out/${c}_bm$bm.err; exit 1; }
    python -c "import json; j=json.loads(open('$out/${c}_bm$bm.json').read().strip().splitlines()[-1]); print('$c bm$bm', j['ms_per_step'], j['roofline']['kernel_ms'], j['matches'], j['digest'], j.get('offsets', {}).get('digest_matches_totals'))"
  done
done
UGPU_XC_BITMAP=1 timeout -k 10 600 python -u -m pytest tests/test_xc.py tests/test_xu.py tests/test_records.py tests/test_offsets_stage.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
