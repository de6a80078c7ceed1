#!/bin/bash
# round 6: the exit abort after the exit guard (engine.hip exit_guard_arm): 40-120 runs per variant
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd); out=$root/gpurun_out/r6v; rm -rf $out; mkdir -p $out
cd $out
python3 - <<'PY'
import numpy as np, sys
sys.path.insert(0, "../../tests")
from oracle_lib import gen
lorem = open("../../tests/golden/verify/lorem.utf8.txt", "rb").read()
open("lorem1m.txt", "wb").write((lorem * (1 + (1 << 20) // len(lorem)))[:1 << 20])
open("words.txt", "wb").write(np.asarray(gen(4, 5, 0, 3 << 20)).tobytes())
PY
export UGPU_ADAPTER_STATS=1 UGPU_ADAPTER_WARM=0
run() {  # name env... -- args (N runs)
  local name=$1; shift
  local bad=0
  for i in $(seq 1 $N); do
    env "$@" > out.txt 2> err.txt
    rc=$?
    if [ $rc -ne 0 ]; then bad=$((bad+1)); cp err.txt err_${name}_$i.txt; fi
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "$name run $i: rc $rc: stop"; exit 1; fi
  done
  echo "$name: $bad of $N non-zero exits"
}
G=$root/oracle/_ref/ugrep_gpu
N=120 run lorem_gpu    UGPU_ADAPTER_MIN_BYTES=0 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt
N=60  run both_gpu     UGPU_ADAPTER_MIN_BYTES=0 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt words.txt
N=60  run both_cpu     UGPU_ADAPTER_MIN_BYTES=99999999999 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt words.txt
N=40  run j16_wait     UGPU_ADAPTER_WARM=wait timeout -k 5 60 $G --sort -J16 -co '\w+' lorem1m.txt words.txt
cd $root && timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ugrep_dropin.py > $out/dropin_tests.log 2>&1; rc=$?; tail -3 $out/dropin_tests.log; exit $rc
