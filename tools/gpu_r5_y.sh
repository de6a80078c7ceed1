# round 5: loop-needle lookback debug run (progress per step)
set -o pipefail
out=gpurun_out/r5y; mkdir -p $out
timeout -k 10 300 python -u tools/lb_debug.py > $out/dbg.log 2>&1; rc=$?
tail -60 $out/dbg.log
exit $rc
