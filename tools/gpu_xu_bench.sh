# C4 bench line (U mode) with the reference-parity sample and a rocprofv3 kernel-trace summary.
# Usage: tools/gpu_xu_bench.sh TAG
set -o pipefail
tag=${1:-xub}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c4 --pcie-sample-mib 0 --verify > $out/bench_c4.json 2> $out/bench_c4.err || { tail -20 $out/bench_c4.err; exit 1; }
cat $out/bench_c4.json
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --word > $out/bench_c4w.json 2> $out/bench_c4w.err || { tail -20 $out/bench_c4w.err; exit 1; }
cat $out/bench_c4w.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o c4 -- python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --steps 5 > $out/prof_c4.log 2>&1 || { tail -20 $out/prof_c4.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3 | xargs -I{} sh -c 'head -6 {}'
