#!/bin/bash
# round 6: the whole GPU test suite, one process
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6s; rm -rf $out; mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
