#!/bin/bash
# round 4: the whole GPU suite, the long-run rates, and quick C2/C3/C4 bench lines
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests > gpurun_out/r4_gpu_all.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error|error" gpurun_out/r4_gpu_all.log | head -20; tail -30 gpurun_out/r4_gpu_all.log; exit 1; }
tail -2 gpurun_out/r4_gpu_all.log
timeout -k 10 300 $T -s tests/test_longrun.py -k rate > gpurun_out/r4_rate.log 2>&1 || { tail -20 gpurun_out/r4_rate.log; exit 1; }
grep "MiB: COUNT" gpurun_out/r4_rate.log
for c in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --pcie-sample-mib 0 > gpurun_out/r4_bench_$c.json 2> gpurun_out/r4_bench_$c.err || { tail gpurun_out/r4_bench_$c.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/r4_bench_$c.json'));print('$c', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'])"
done
