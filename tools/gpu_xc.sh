# xc_kernel round-2 check: its GPU tests, a C3 bench line and a rocprofv3 kernel-trace summary.
# Usage: tools/gpu_xc.sh TAG
set -o pipefail
tag=${1:-xc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xc.py -x -v --timeout 150 --timeout-method thread > $out/test_xc.log 2>&1 || { tail -30 $out/test_xc.log; exit 1; }
tail -3 $out/test_xc.log
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_c3.json 2> $out/bench_c3.err || { tail -20 $out/bench_c3.err; exit 1; }
cat $out/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o c3 -- python bench.py --config c3 --no-cpu-baseline --pcie-sample-mib 0 --steps 5 > $out/prof_c3.log 2>&1 || { tail -20 $out/prof_c3.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3 | xargs -I{} sh -c 'head -5 {}'
