#!/bin/bash
# round 4: long walks in sparse_kernel -- new tests, then the sparse-path suites, then the C2 bench
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_longrun.py > gpurun_out/r4_longrun.log 2>&1 || { echo "longrun failed"; tail -30 gpurun_out/r4_longrun.log; exit 1; }
tail -15 gpurun_out/r4_longrun.log
if [ "$1" = "all" ]; then
  timeout -k 10 600 $T tests/test_gpu.py tests/test_offsets_stage.py tests/test_c5.py tests/test_stream.py tests/test_multi.py > gpurun_out/r4_sparse_suites.log 2>&1 || { echo "suites failed"; tail -30 gpurun_out/r4_sparse_suites.log; exit 1; }
  tail -3 gpurun_out/r4_sparse_suites.log
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_bench_c2.json 2> gpurun_out/r4_bench_c2.err || { tail gpurun_out/r4_bench_c2.err; exit 1; }
  cat gpurun_out/r4_bench_c2.json
fi
