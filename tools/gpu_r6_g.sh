#!/bin/bash
# round 6: VALU rates (second pass) + lookahead on the GPU + the wfind suites
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6g; rm -rf $out; mkdir -p $out
timeout -k 10 120 ./tools/probe/valu_rate3 > $out/valu_rate3.txt 2>&1 || { cat $out/valu_rate3.txt; exit 1; }
cat $out/valu_rate3.txt
timeout -k 10 900 python -u -m pytest tests/test_lookahead.py tests/test_anchor.py tests/test_word.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -3
