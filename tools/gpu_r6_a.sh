#!/bin/bash
# round 6 probe: VALU issue rates of SDWA / bitop3 / shift forms (valu_rate2),
# then the C4 COUNT line on this box as the baseline for the U-mode rewrite
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6a; rm -rf $out; mkdir -p $out
timeout -k 10 120 ./tools/probe/valu_rate2 > $out/valu_rate2.txt 2>&1 || { cat $out/valu_rate2.txt; exit 1; }
cat $out/valu_rate2.txt
timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
python3 -c "import json;j=json.load(open('$out/c4.json'));print('c4', j['ms_per_step'], j['roofline'])"
