#!/bin/bash
# round 6: dominated restarts (tests/test_dom.py) + the long-walk suites they touch
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6b; rm -rf $out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_dom.py tests/test_longrun.py tests/test_lookback.py -x -v -m gpu --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -3
