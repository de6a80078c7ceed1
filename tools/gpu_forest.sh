set -o pipefail
mkdir -p gpurun_out/forest
for m in 128 1024; do
timeout -k 10 120 python -u tools/bench_forest.py --mib $m --ref-mib 64 >> gpurun_out/forest/bench.json 2>> gpurun_out/forest/bench.err || exit 1
done
bash tools/gpu_check.sh r02b
