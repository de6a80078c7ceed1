#!/bin/bash
# round 6: multi-rank rehearsal on one GPU (gloo, 2 ranks x 16 GiB):
#   C3 --offsets: dense-table records stay on their ranks (auto -> sharded; sums all-gathered)
#   C2 --offsets: small record sets are still gathered to rank 0 (auto -> gather)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6e; rm -rf $out; mkdir -p $out
export UGPU_BENCH_BACKEND=gloo
for c in c3 c2; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --config $c --steps 3 --warmup 1 --offsets --no-cpu-baseline --pcie-sample-mib 0 \
    > $out/rehearsal_$c.json 2> $out/rehearsal_$c.err || { tail -20 $out/rehearsal_$c.err; exit 1; }
  python3 -c "import json;j=[json.loads(l) for l in open('$out/rehearsal_$c.json') if l.startswith('{')][0];print('$c', j['n_gpus'], j['ms_per_step'], j['value'], j['offsets'])"
done
