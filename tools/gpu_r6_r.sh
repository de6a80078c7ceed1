#!/bin/bash
# round 6: an intermittent abort at ugrep_gpu's exit ("corrupted double-linked list") after a lookahead
# command: how often, for which commands (host-side heap check; each run bounded, outputs compared)
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd); out=$root/gpurun_out/r6r; rm -rf $out; mkdir -p $out
cd $out
python3 - <<'PY'
import numpy as np, sys
sys.path.insert(0, "../../tests")
from oracle_lib import gen
lorem = open("../../tests/golden/verify/lorem.utf8.txt", "rb").read()
open("lorem1m.txt", "wb").write((lorem * (1 + (1 << 20) // len(lorem)))[:1 << 20])
open("words.txt", "wb").write(np.asarray(gen(4, 5, 0, 3 << 20)).tobytes())
PY
export UGPU_ADAPTER_MIN_BYTES=0 UGPU_ADAPTER_STATS=1 UGPU_ADAPTER_WARM=0 MALLOC_CHECK_=3
$root/oracle/_ref/ugrep --sort -J1 -o '\w+(?=\.)' lorem1m.txt words.txt > ref_look.txt
$root/oracle/_ref/ugrep --sort -J1 -o '\w+' lorem1m.txt words.txt > ref_w.txt
for cmd in look w; do
  if [ $cmd = look ]; then rx='\w+(?=\.)'; else rx='\w+'; fi
  bad=0; diff=0
  for i in $(seq 1 15); do
    timeout -k 5 60 $root/oracle/_ref/ugrep_gpu --sort -J1 -o "$rx" lorem1m.txt words.txt > got.txt 2> err_${cmd}_$i.txt
    rc=$?
    if [ $rc -ne 0 ]; then bad=$((bad+1)); echo "$cmd run $i rc=$rc"; tail -3 err_${cmd}_$i.txt; fi
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timeout: stop"; exit 1; fi
    cmp -s got.txt ref_$cmd.txt || diff=$((diff+1))
  done
  echo "$cmd: $bad of 15 non-zero exits, $diff outputs differ"
done
