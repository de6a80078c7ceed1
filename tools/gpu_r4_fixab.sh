#!/bin/bash
# round 4: long-walk tests, then fix_kernel / resume-launch time with and
# without walk truncation (rocprofv3 trace), then the default C2 line
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread tests/test_longrun.py tests/test_offsets_stage.py tests/test_records.py > gpurun_out/r4_longrun2.log 2>&1 || { tail -30 gpurun_out/r4_longrun2.log; exit 1; }
grep -E "passed|MiB: COUNT" gpurun_out/r4_longrun2.log
for t in 0 1; do
  UGPU_TRUNC=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_fixab2_$t -o f -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 --bytes 4294967296 > gpurun_out/r4_fixab2_$t.json 2>/dev/null || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_bench_c2b.json 2> gpurun_out/r4_bench_c2b.err || exit 1
python3 -c "import json;j=json.load(open('gpurun_out/r4_bench_c2b.json'));print('c2', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
