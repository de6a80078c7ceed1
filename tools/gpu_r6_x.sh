#!/bin/bash
# round 6: assertion groups distributed by the compiler: GPU tests (fixtures,
# anchors, word boundaries, compile) and the drop-in commands
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6x; rm -rf $out; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_asgroup.py tests/test_anchor.py tests/test_wordb.py tests/test_compile.py "tests/test_ugrep_dropin.py::test_dropin_assertion_groups" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
cp gpurun_out/dropin_asgroup_ledger.json $out/ 2>/dev/null; true
