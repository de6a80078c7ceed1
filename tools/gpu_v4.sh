# option W throughput (wfind_kernel) on the BASELINE corpora
mkdir -p gpurun_out/v4
for c in c3 c4 c2; do
  timeout -k 10 240 python bench.py --config $c --word --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/v4/bench_${c}_word.json 2> gpurun_out/v4/bench_${c}_word.err || exit 1
done
