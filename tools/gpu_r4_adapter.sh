#!/bin/bash
# round 4: adapter (SCAN/MATCH from records, device queue), drop-in suite with the
# default queue, the a+ halo test, and ugrep -J16 CPU vs GPU
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 400 $T -m gpu tests/test_adapter.py tests/test_ugrep_dropin.py tests/test_plan.py "tests/test_c5.py::test_scan_shard_grows_the_halo" > gpurun_out/r4_adapter.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4_adapter.log | head -30; tail -40 gpurun_out/r4_adapter.log; exit 1; }
tail -3 gpurun_out/r4_adapter.log
timeout -k 10 600 python -u tools/bench_ugrep.py --files ${UG_FILES:-16} --mib ${UG_MIB:-64} --reps 2 > gpurun_out/r4_bench_ugrep.jsonl 2> gpurun_out/r4_bench_ugrep.err || { tail -20 gpurun_out/r4_bench_ugrep.err; exit 1; }
cat gpurun_out/r4_bench_ugrep.jsonl
