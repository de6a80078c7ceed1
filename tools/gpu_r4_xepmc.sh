#!/bin/bash
# round 4: PMC passes over the OFFSETS kernels (one counter group per run)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
C=${1:-c4}
i=0
for g in "WRITE_SIZE" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g -d gpurun_out/xepmc_${C}_$i -o run -- python3 -u bench.py --config $C --offsets --steps 2 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/xepmc_${C}_$i.json 2> gpurun_out/xepmc_${C}_$i.err || { tail -5 gpurun_out/xepmc_${C}_$i.err; exit 1; }
  echo "pass $i done"
done
