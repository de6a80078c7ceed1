# round 5: the whole GPU suite with per-test durations, and smoke
set -o pipefail
out=gpurun_out/r5s; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu --durations=40 > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -A45 "slowest" $out/tests.log | head -50
tail -1 $out/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -10 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
