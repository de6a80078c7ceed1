#!/bin/bash
# Profile one bench config on the GPU box (run from the repo root under gpurun):
#   1. rocprofv3 --kernel-trace --stats   -> per-kernel durations
#   2. rocprofv3 --pmc passes (counters only, with --kernel-trace) -> HBM bytes, VALU/wave counters
# then tools/pmc_summary.py condenses them into gpurun_out/prof_TAG/summary.json.
# usage: tools/profile.sh TAG CONFIG [extra bench.py args]
set -e -o pipefail
tag=$1; cfg=$2; shift 2
root=$(pwd)
out=$root/gpurun_out/prof_$tag
rm -rf "$out"; mkdir -p "$out"
export TMPDIR=/tmp
# (no PCIe leg, no CPU baseline and its reference-parity sample: the scan
# kernel's dispatches are then the bench's own warmup + timed steps)
args=(--config "$cfg" --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 "$@")
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run -- \
    python3 "$root/bench.py" "${args[@]}" > "$out/bench.json" 2> "$out/trace.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/pmc1" -o run -- \
    python3 "$root/bench.py" "${args[@]}" > /dev/null 2> "$out/pmc1.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$out/pmc2" -o run -- \
    python3 "$root/bench.py" "${args[@]}" > /dev/null 2> "$out/pmc2.err"
if [ -n "$PMC3" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d "$out/pmc3" -o run -- \
      python3 "$root/bench.py" "${args[@]}" > /dev/null 2> "$out/pmc3.err"
fi
cd "$root"
python3 tools/pmc_summary.py "$out" > "$out/summary.json"
cat "$out/summary.json"
