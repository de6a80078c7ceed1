# Multi-rank rehearsal on one GPU (gloo): 3 ranks of 1 GiB each, C2 and C3, offsets + whole-stream verify.
set -o pipefail
export UGPU_BENCH_BACKEND=gloo
for c in c2 c3; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 3 --config $c --bytes 1073741824 --steps 2 --warmup 1 --offsets --verify --no-cpu-baseline --pcie-sample-mib 0 \
    > gpurun_out/rehearsal_$c.json 2> gpurun_out/rehearsal_$c.err || { tail -20 gpurun_out/rehearsal_$c.err; exit 1; }
  grep -h "verify" gpurun_out/rehearsal_$c.err | tail -2
done
