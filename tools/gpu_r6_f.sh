#!/bin/bash
# round 6: VALU issue rates, second pass (tools/probe/valu_rate3.hip)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6f; rm -rf $out; mkdir -p $out
timeout -k 10 120 ./tools/probe/valu_rate3 > $out/valu_rate3.txt 2>&1 || { cat $out/valu_rate3.txt; exit 1; }
cat $out/valu_rate3.txt
