# Round 3: C4 on U mode (UGPU_XU=1) and on xg_kernel, same box; then the given GPU test files.
# usage: tools/gpu_r3_c4.sh TAG [TESTFILE...]
set -o pipefail
out=gpurun_out/${1:-r3c4}; shift
mkdir -p $out
UGPU_XU=1 timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/u.json 2> $out/u.err || { tail -5 $out/u.err; exit 1; }
UGPU_XU=0 timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/xg.json 2> $out/xg.err || { tail -5 $out/xg.err; exit 1; }
for f in u xg; do python -c "import json; j=json.load(open('$out/$f.json')); print('$f', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])"; done
if [ $# -gt 0 ]; then
  timeout -k 10 1000 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
  grep -E "passed|failed" $out/tests.log | tail -2
fi
