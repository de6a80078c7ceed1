# round 5, first GPU call: VALU issue-rate probe, then the GPU tests touched by
# the host/device split, the HALO-safe stitch and the records fixes
set -o pipefail
out=gpurun_out/r5a; mkdir -p $out
timeout -k 10 120 ./tools/probe/valu_rate > $out/valu_rate.txt 2>&1 || { cat $out/valu_rate.txt; exit 1; }
cat $out/valu_rate.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c5.py tests/test_records.py tests/test_ugrep_dropin.py -m gpu > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error|free .* s" $out/tests.log | tail -8
exit $rc
