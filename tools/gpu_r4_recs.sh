#!/bin/bash
# round 4: records / offsets tests with the In-bits expansion as the default, and the OFFSETS lines
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/test_records.py tests/test_c5.py tests/test_xc.py tests/test_xu.py tests/test_adapter.py tests/test_wordb.py tests/test_plan.py tests/test_gpu.py > gpurun_out/r4_recs_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4_recs_tests.log | head -30; tail -30 gpurun_out/r4_recs_tests.log; exit 1; }
tail -2 gpurun_out/r4_recs_tests.log
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --offsets --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_offsets_$c.json 2> gpurun_out/r4_offsets_$c.err || { tail gpurun_out/r4_offsets_$c.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/r4_offsets_$c.json'));print('$c', j['ms_per_step'], j['offsets'])"
done
timeout -k 10 400 python -u tools/bench_adapter.py --max-mib 256 --reps 3 > gpurun_out/r4_bench_adapter.jsonl 2> gpurun_out/r4_bench_adapter.err || { tail gpurun_out/r4_bench_adapter.err; exit 1; }
tail -4 gpurun_out/r4_bench_adapter.jsonl
