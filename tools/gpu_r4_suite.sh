#!/bin/bash
# round 4: the whole GPU suite, as the driver runs it
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 1100 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r4_gpu_all.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error|error" gpurun_out/r4_gpu_all.log | head -20; tail -30 gpurun_out/r4_gpu_all.log; exit 1; }
tail -2 gpurun_out/r4_gpu_all.log
grep -E "passed|failed" gpurun_out/r4_gpu_all.log | tail -1
