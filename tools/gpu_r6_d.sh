#!/bin/bash
# round 6: dominated restarts: timings (tools/dbg_dom.py) then the suites they touch
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6d; rm -rf $out; mkdir -p $out
timeout -k 10 300 python3 -u tools/dbg_dom.py > $out/dbg.txt 2>&1 || { tail -30 $out/dbg.txt; exit 1; }
cat $out/dbg.txt
timeout -k 10 900 python -u -m pytest tests/test_dom.py tests/test_longrun.py tests/test_lookback.py tests/test_gpu.py tests/test_multi.py tests/test_offsets_stage.py tests/test_records.py -x -v -m gpu --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -3
