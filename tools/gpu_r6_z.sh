#!/bin/bash
# round 6: negative patterns under option W -- REDO/W/word-boundary/lookback GPU tests, the drop-in commands
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6z; rm -rf $out; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_redo_w.py tests/test_redo.py tests/test_word.py tests/test_wordb.py tests/test_lookback.py tests/test_ugrep_dropin.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
cp gpurun_out/dropin_redo_w_ledger.json $out/ 2>/dev/null; true
