#!/bin/bash
# round 4: word boundaries + 12-byte OFFSETS records (bitmap expansion A/B)
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests/test_wordb.py tests/test_anchor.py tests/test_plan.py tests/test_adapter.py tests/test_ugrep_dropin.py tests/test_records.py "tests/test_c5.py::test_offsets_record_by_record" > gpurun_out/r4_off_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4_off_tests.log | head -30; tail -30 gpurun_out/r4_off_tests.log; exit 1; }
tail -2 gpurun_out/r4_off_tests.log
for c in c4 c3; do
  for bm in 0 1; do
    UGPU_XC_BITMAP=$bm timeout -k 10 300 python -u bench.py --config $c --offsets --steps 5 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_off_${c}_bm$bm.json 2> gpurun_out/r4_off_${c}_bm$bm.err || { tail gpurun_out/r4_off_${c}_bm$bm.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/r4_off_${c}_bm$bm.json'));print('$c bm=$bm', j['ms_per_step'], j['offsets'])"
  done
done
