#!/bin/bash
# round 6: lookahead from the native compiler -- GPU parity of compiled tables and the ugrep drop-in commands
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6j; rm -rf $out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_lookahead_compile.py tests/test_lookahead.py tests/test_ugrep_dropin.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -2
cp gpurun_out/dropin_lookahead_ledger.json $out/ 2>/dev/null; true
