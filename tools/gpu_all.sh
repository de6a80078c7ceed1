# The whole GPU suite in one pytest process, with per-test durations, logged
# under gpurun_out/TAG.   usage: tools/gpu_all.sh TAG
set -o pipefail
out=gpurun_out/${1:-all}
mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=30 > $out/tests.log 2>&1
rc=$?
grep -E "passed|failed" $out/tests.log | tail -3
exit $rc
