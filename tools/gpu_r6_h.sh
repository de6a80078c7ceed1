#!/bin/bash
# round 6: C4 U-mode A/B: VGPR mask constants (default) vs SGPR/literals (vk0) vs 7 waves/SIMD (vk7)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6h; rm -rf $out; mkdir -p $out
for rep in 1 2; do
for lib in ${LIBS:-libugrep_amd.so libugrep_amd_vk0.so libugrep_amd_vk7.so}; do
  UGPU_LIB=$lib timeout -k 10 200 python3 bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 > $out/$lib.$rep.json 2> $out/$lib.$rep.err || { tail -5 $out/$lib.$rep.err; exit 1; }
  python3 -c "import json; j=json.load(open('$out/$lib.$rep.json')); print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['digest'])"
done
done
