#!/bin/bash
# round 4: xc_expand_kernel ablations (UGPU_XE_ABL variants: 1 no stores, 2 no length stores, 3 no start stores)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in c4 c3; do
  for v in "" xe1; do
    lib=libugrep_amd${v:+_$v}.so
    UGPU_LIB=$lib UGPU_XC_BITMAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_xeabl_${c}_$v -o run --output-format csv -- python3 bench.py --config $c --offsets --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_xeabl_${c}_$v.log 2>&1 || { tail -5 gpurun_out/r4_xeabl_${c}_$v.log; exit 1; }
    f=$(ls gpurun_out/r4_xeabl_${c}_$v/*kernel_stats.csv | head -1)
    echo "$c ${v:-base}: $(grep -E 'expand|bm_kernel' $f | awk -F, '{printf "%s %.3f ms; ", $1, $4/1e6}')"
  done
done
