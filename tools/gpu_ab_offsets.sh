#!/bin/bash
# A/B of two in-tree library builds on the OFFSETS lines, alternated on one box:
#   bash tools/gpu_ab_offsets.sh libugrep_amd_base.so [configs...]
set -o pipefail
cd "$(dirname "$0")/.."
B=$1; shift
CFGS=${@:-c4 c3}
for rep in 1 2; do
  for c in $CFGS; do
    for lib in libugrep_amd.so $B; do
      UGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --offsets --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/ab_$c.json 2> gpurun_out/ab_$c.err || { tail gpurun_out/ab_$c.err; exit 1; }
      python3 -c "import json;j=json.load(open('gpurun_out/ab_$c.json'));print('$rep $c $lib', j['ms_per_step'], j['offsets']['digest_matches_totals'], j.get('kernel_ms'))" | tee -a gpurun_out/ab_offsets.txt
    done
  done
done
