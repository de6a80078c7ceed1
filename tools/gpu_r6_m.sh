#!/bin/bash
# round 6: C4 U mode with fewer half-rate VALU (swizzle y ^ x; a one-shift 3-byte fill): parity, then A/B
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6m; rm -rf $out; mkdir -p $out
UGPU_LIB=libugrep_amd_sf.so timeout -k 10 600 python -u -m pytest tests/test_xu.py tests/test_xu_host.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -2
for lib in default sf swz2 fix7 default sf; do
  if [ $lib = default ]; then L=libugrep_amd.so; else L=libugrep_amd_$lib.so; fi
  UGPU_LIB=$L timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --steps 20 > $out/b_$lib.json 2> $out/b_$lib.err || { tail -5 $out/b_$lib.err; exit 1; }
  python3 -c "import json;j=json.load(open('$out/b_$lib.json'));print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])" | tee -a $out/summary.txt
done
