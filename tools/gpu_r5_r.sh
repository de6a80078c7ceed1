# round 5: C2 COUNT after the sparse kernel's spill fix (C3 beside it as the
# box's yardstick), then the word-boundary / W tests on the new build
set -o pipefail
out=gpurun_out/r5r; mkdir -p $out
for rep in 1 2; do
for c in c2 c3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --pcie-sample-mib 0 > $out/$c.$rep.json 2> $out/$c.$rep.err || { tail -5 $out/$c.$rep.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$c.$rep.json')); print('$c', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
done
timeout -k 10 600 python -u -m pytest tests/test_word.py tests/test_wordb.py tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
