# xc_kernel U mode (code-point runs, C4): its GPU tests, the C4 bench line and a
# rocprofv3 kernel-trace summary.  Usage: tools/gpu_xu.sh TAG
set -o pipefail
tag=${1:-xu}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xu.py -x -v --timeout 150 --timeout-method thread > $out/test_xu.log 2>&1 || { tail -40 $out/test_xu.log; exit 1; }
tail -3 $out/test_xu.log
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --verify > $out/bench_c4.json 2> $out/bench_c4.err || { tail -20 $out/bench_c4.err; exit 1; }
cat $out/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o c4 -- python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --steps 5 > $out/prof_c4.log 2>&1 || { tail -20 $out/prof_c4.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3 | xargs -I{} sh -c 'head -6 {}'
