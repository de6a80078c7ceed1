#!/bin/bash
# round 6: C4/C3 main loops with 32-bit lane sums (UGPU_XC_ACC32) on top of the swizzle / fill change: parity, A/B
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6n; rm -rf $out; mkdir -p $out
UGPU_LIB=libugrep_amd_sfa.so timeout -k 10 900 python -u -m pytest tests/test_xu.py tests/test_xc.py tests/test_wsub.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -2
for run in 1 2; do
for cfg in c4 c3; do
  for lib in default sf sfa a; do
    if [ $cfg = c3 ] && [ $lib = sf ]; then continue; fi
    if [ $lib = default ]; then L=libugrep_amd.so; else L=libugrep_amd_$lib.so; fi
    UGPU_LIB=$L timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --pcie-sample-mib 0 --steps 20 > $out/b_${cfg}_$lib.json 2> $out/b_${cfg}_$lib.err || { tail -5 $out/b_${cfg}_$lib.err; exit 1; }
    python3 -c "import json;j=json.load(open('$out/b_${cfg}_$lib.json'));print('$cfg $lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])" | tee -a $out/summary.txt
  done
done
done
