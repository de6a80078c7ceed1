# Closing check of a session: full -m gpu suite, smoke, default bench.
set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/final2/gpu_all.log 2>&1 || { tail -30 gpurun_out/final2/gpu_all.log; exit 1; }
tail -1 gpurun_out/final2/gpu_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final2/bench.json 2> gpurun_out/final2/bench.err || exit 1
cat gpurun_out/final2/bench.json
