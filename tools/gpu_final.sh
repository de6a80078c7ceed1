# Round-end check on one GPU: full -m gpu suite, smoke, default bench, W benches, C2 profile.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/final/gpu_all.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
for c in c3 c4; do
  timeout -k 10 240 python bench.py --config $c --word --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/final/bench_${c}_word.json 2> gpurun_out/final/bench_${c}_word.err || exit 1
done
bash tools/profile.sh final_c2 c2 > gpurun_out/final/profile_c2.log 2>&1 || exit 1
