# round 5: loop-needle lookback, which kernels the slow inputs spend their time in
set -o pipefail
out=gpurun_out/r5z; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 -u tools/lb_prof.py tail > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1); head -12 "$f"
