#!/bin/bash
# round 6: drop-in tests after the warm-up wait default
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6q; rm -rf $out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_ugrep_dropin.py tests/test_adapter.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
grep -E "PASS|FAIL" $out/tests.log | tail -12; tail -1 $out/tests.log
