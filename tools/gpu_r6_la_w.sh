#!/bin/bash
# round 6: lookahead under option W -- lookahead / W GPU tests and the drop-in commands
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6lw; rm -rf $out; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lookahead_w.py tests/test_lookahead.py tests/test_lookahead_compile.py tests/test_word.py tests/test_redo_w.py tests/test_ugrep_dropin.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
cp gpurun_out/dropin_lookahead_w_ledger.json $out/ 2>/dev/null; true
