#!/bin/bash
# round 4: word boundaries on the GPU (fixtures, shards, streams), the adapter and drop-in suites
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests/test_wordb.py tests/test_anchor.py tests/test_plan.py tests/test_adapter.py tests/test_ugrep_dropin.py > gpurun_out/r4_wordb.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4_wordb.log | head -30; tail -40 gpurun_out/r4_wordb.log; exit 1; }
tail -3 gpurun_out/r4_wordb.log
