# Round 3: A/B of builds on C4 (UGPU_XU=1 U mode), then the U-mode GPU tests (+ adapter) on the default library.
# usage: tools/gpu_r3_ab.sh TAG LIB...
set -o pipefail
out=gpurun_out/${1:-r3ab}; shift
mkdir -p $out
for lib in "$@"; do
  UGPU_XU=1 UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/u_$lib.json 2> $out/u_$lib.err || { tail -5 $out/u_$lib.err; exit 1; }
  python -c "import json; j=json.load(open('$out/u_$lib.json')); print('U $lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])"
done
UGPU_XU=1 timeout -k 10 400 python -u -m pytest tests/test_xu.py -x -q --timeout 150 --timeout-method thread > $out/tests_xu.log 2>&1 || { tail -20 $out/tests_xu.log; exit 1; }
tail -1 $out/tests_xu.log
timeout -k 10 600 python -u -m pytest tests/test_adapter.py -x -q --timeout 500 --timeout-method thread > $out/tests_adapter.log 2>&1 || { tail -20 $out/tests_adapter.log; exit 1; }
tail -1 $out/tests_adapter.log
