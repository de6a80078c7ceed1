#!/bin/bash
# round 6, last: the C4 bench command under a trace-only rocprofv3 pass and one
# FETCH_SIZE pass (as tools/gpu_r6_end.sh), to sample the box-to-box spread
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
d=gpurun_out/r06c4; rm -rf $d; mkdir -p $d
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/trace -o run -- python3 -u bench.py --config c4 > $d/bench.json 2> $d/bench.err || { tail $d/bench.err; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $d/pmc1 -o run -- python3 -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $d/pmc1.json 2> $d/pmc1.err || { tail $d/pmc1.err; exit 1; }
python3 tools/pmc_summary.py $d > $d/summary.json
python3 -c "import json;s=json.load(open('$d/summary.json'));b=s['bench'];print('c4', b['ms_per_step'], b['value'], s.get('kernel_ms'), s.get('kernel_ms_bench'), s.get('traffic_over_algorithmic'))"
