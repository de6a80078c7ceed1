#!/bin/bash
# round 6: the intermittent exit abort of ugrep_gpu ("corrupted double-linked list"): 40 runs of the plain
# build, then 40 under AddressSanitizer (host code only: ugrep and the adapter instrumented,
# tools/asan/build_ugrep_gpu_asan.sh), two commands alternating
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd); out=$root/gpurun_out/r6s2; rm -rf $out; mkdir -p $out
cd $out
python3 - <<'PY'
import numpy as np, sys
sys.path.insert(0, "../../tests")
from oracle_lib import gen
lorem = open("../../tests/golden/verify/lorem.utf8.txt", "rb").read()
open("lorem1m.txt", "wb").write((lorem * (1 + (1 << 20) // len(lorem)))[:1 << 20])
open("words.txt", "wb").write(np.asarray(gen(4, 5, 0, 3 << 20)).tobytes())
PY
export UGPU_ADAPTER_MIN_BYTES=0 UGPU_ADAPTER_STATS=1 UGPU_ADAPTER_WARM=0
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=0
for exe in ugrep_gpu asan/ugrep_gpu_asan; do
  bad=0
  for i in $(seq 1 40); do
    if [ $((i % 2)) = 0 ]; then rx='\w+'; else rx='\w+(?=\.)'; fi
    timeout -k 5 120 $root/oracle/_ref/$exe --sort -J1 -o "$rx" lorem1m.txt words.txt > got.txt 2> err.txt
    rc=$?
    if [ $rc -ne 0 ]; then
      bad=$((bad+1)); echo "$exe run $i rc=$rc"; cp err.txt err_$(basename $exe)_$i.txt
      grep -m1 -A 30 "ERROR: AddressSanitizer" err.txt | head -40
    fi
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timeout: stop"; exit 1; fi
  done
  echo "$exe: $bad of 40 non-zero exits"
done
