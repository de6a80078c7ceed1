#!/bin/bash
# round 4: trace-only profile of the default C2 bench (kernel times incl. the
# resume launch and fix_kernel), and the long-run rates printed
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_c2prof -o c2 -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_c2prof_bench.json 2> gpurun_out/r4_c2prof_bench.err || { tail gpurun_out/r4_c2prof_bench.err; exit 1; }
cat gpurun_out/r4_c2prof_bench.json
find gpurun_out/r4_c2prof -name "*kernel_stats.csv" | head -3
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_longrun.py -k rate > gpurun_out/r4_rate.log 2>&1 || { tail -20 gpurun_out/r4_rate.log; exit 1; }
grep "MiB: COUNT" gpurun_out/r4_rate.log
