set -o pipefail
mkdir -p gpurun_out/xg
timeout -k 10 500 python -u -m pytest tests/test_xg.py tests/test_gpu.py tests/test_compile.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/xg/t.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/xg/bench_c4.json 2> gpurun_out/xg/bench_c4.err || exit 1
bash tools/profile.sh xg_c4 c4 --pcie-sample-mib 0 > gpurun_out/xg/prof.log 2>&1
