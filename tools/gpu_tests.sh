# Run the given GPU test files (one pytest process), log under gpurun_out/TAG.
# usage: tools/gpu_tests.sh TAG TESTFILE...
set -o pipefail
out=gpurun_out/${1:-tests}; shift
mkdir -p $out
timeout -k 10 1000 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -3
grep -E "PASSED|FAILED" $out/tests.log | sed -E 's/ +\[.*//' | awk '{print $2, $1}' | sort | uniq -c | sort -rn | head -3
