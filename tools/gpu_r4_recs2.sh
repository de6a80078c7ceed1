#!/bin/bash
# round 4: records defaults (32/16 MiB chunks, 2-byte dense pieces) -- tests, sweep, adapter bench
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 400 $T -m gpu tests/test_records.py tests/test_adapter.py > gpurun_out/r4_recs2_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4_recs2_tests.log | head -30; tail -30 gpurun_out/r4_recs2_tests.log; exit 1; }
tail -2 gpurun_out/r4_recs2_tests.log
timeout -k 10 400 python -u tools/bench_adapter.py --max-mib 256 --reps 3 > gpurun_out/r4_bench_adapter2.jsonl 2> gpurun_out/r4_bench_adapter2.err || { tail gpurun_out/r4_bench_adapter2.err; exit 1; }
tail -4 gpurun_out/r4_bench_adapter2.jsonl
