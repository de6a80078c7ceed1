mkdir -p gpurun_out/v2
timeout -k 10 300 python -u -m pytest tests/test_compile.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/v2/gpu_compile.log 2>&1 && \
for c in c1 c2 c3 c4; do timeout -k 10 200 python bench.py --config $c --compile --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/v2/bench_$c.json 2> gpurun_out/v2/bench_$c.err || exit 1; done
