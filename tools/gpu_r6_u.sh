#!/bin/bash
# round 6: bisect the rare ugrep_gpu exit abort: 40 runs per variant (files, chunk size, CPU-only)
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd); out=$root/gpurun_out/r6u; rm -rf $out; mkdir -p $out
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
run() {  # name env... -- args
  local name=$1; shift
  local bad=0
  for i in $(seq 1 40); do
    env "$@" > out.txt 2> err.txt
    rc=$?
    if [ $rc -ne 0 ]; then bad=$((bad+1)); cp err.txt err_${name}_$i.txt; fi
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timeout: stop"; exit 1; fi
  done
  echo "$name: $bad of 40 non-zero exits"
}
G=$root/oracle/_ref/ugrep_gpu
run both_gpu     UGPU_ADAPTER_MIN_BYTES=0 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt words.txt
run words_gpu    UGPU_ADAPTER_MIN_BYTES=0 timeout -k 5 60 $G --sort -J1 -o '\w+' words.txt
run lorem_gpu    UGPU_ADAPTER_MIN_BYTES=0 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt
run both_chunk8  UGPU_ADAPTER_MIN_BYTES=0 UGPU_ADAPTER_CHUNK=8388608 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt words.txt
run both_count   UGPU_ADAPTER_MIN_BYTES=0 timeout -k 5 60 $G --sort -J1 -co '\w+' lorem1m.txt words.txt
run both_cpu     UGPU_ADAPTER_MIN_BYTES=99999999999 timeout -k 5 60 $G --sort -J1 -o '\w+' lorem1m.txt words.txt
