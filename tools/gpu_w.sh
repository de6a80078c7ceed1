# W fast path + xc LDS classifier: GPU tests and the C4 -w / C3 bench lines. Usage: tools/gpu_w.sh TAG
set -o pipefail
tag=${1:-w}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_word.py tests/test_xc.py -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python bench.py --config c4 --word --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_c4w.json 2> $out/bench_c4w.err || { tail -20 $out/bench_c4w.err; exit 1; }
cat $out/bench_c4w.json
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_c3.json 2> $out/bench_c3.err || { tail -20 $out/bench_c3.err; exit 1; }
cat $out/bench_c3.json
