#!/bin/bash
# round 4: expansion with untracked prefetch loads -- record tests and the OFFSETS lines
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests/test_xc.py tests/test_xu.py tests/test_c5.py tests/test_records.py > gpurun_out/r4_xe_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4_xe_tests.log | head -30; tail -30 gpurun_out/r4_xe_tests.log; exit 1; }
tail -2 gpurun_out/r4_xe_tests.log
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --offsets --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_xe_offsets_$c.json 2> gpurun_out/r4_xe_offsets_$c.err || { tail gpurun_out/r4_xe_offsets_$c.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/r4_xe_offsets_$c.json'));print('$c', j['ms_per_step'], j['offsets'])"
done
bash tools/gpu_r4_xeprof.sh
