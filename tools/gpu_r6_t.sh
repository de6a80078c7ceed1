#!/bin/bash
# round 6: does the rare exit abort come from the engine + HIP runtime alone? 60 runs of
# tools/probe/exit_probe (stream feeds through the C ABI, no ugrep, no adapter)
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd); out=$root/gpurun_out/r6t; rm -rf $out; mkdir -p $out
cd $out
python3 - <<'PY'
import numpy as np, sys
sys.path.insert(0, "../../tests")
from oracle_lib import gen
open("words.txt", "wb").write(np.asarray(gen(4, 5, 0, 3 << 20)).tobytes())
PY
bad=0
for i in $(seq 1 60); do
  timeout -k 5 60 $root/tools/probe/exit_probe words.txt '(?m)[A-Za-z]+' > out.txt 2> err.txt
  rc=$?
  if [ $rc -ne 0 ]; then bad=$((bad+1)); echo "run $i rc=$rc"; cat err.txt | head -5; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "timeout: stop"; exit 1; fi
done
echo "exit_probe: $bad of 60 non-zero exits ($(cat out.txt))"
