# A/B of U-mode builds on C4 (UGPU_XU=1), then the U-mode GPU tests on the second library.
set -o pipefail
out=gpurun_out/${1:-ab2}; shift
mkdir -p $out
for lib in "$@"; do
  UGPU_XU=1 UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --verify > $out/$lib.json 2> $out/$lib.err || { tail -5 $out/$lib.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$lib.json')); print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['digest'], j['verified_whole_stream'])"
done
UGPU_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_xu.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
