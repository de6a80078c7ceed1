# Round 3 end rehearsal on one MI355X: smoke(), the default bench line (as the
# driver runs it), and the torch.distributed (RCCL) launch path with one rank.
set -o pipefail
out=gpurun_out/${1:-r3end}
mkdir -p $out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cut -c1-300 $out/bench.json
# (UGPU_BENCH_PG=1: the process group, the stitch all_gather and the records
# all_gather run over RCCL also with one rank)
for extra in "" "--offsets"; do
  tag=nccl1$(echo "$extra" | tr -d ' -')
  UGPU_BENCH_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 $extra > $out/bench_$tag.json 2> $out/bench_$tag.err || { tail -20 $out/bench_$tag.err; exit 1; }
  cut -c1-300 $out/bench_$tag.json
done
