#!/bin/bash
# round 6: ugrep end to end (ugrep -co -J16, 16 x 256 MiB), default policy and with the warm-up awaited
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6p; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/bench_ugrep.py --files 16 --mib 256 --reps 3 --configs c3,c4 > $out/default.jsonl 2> $out/default.err || { tail -5 $out/default.err; exit 1; }
UGPU_ADAPTER_WARM=wait timeout -k 10 500 python3 -u tools/bench_ugrep.py --files 16 --mib 256 --reps 3 --configs c3,c4 > $out/wait.jsonl 2> $out/wait.err || { tail -5 $out/wait.err; exit 1; }
for f in default wait; do python3 -c "
import json
for l in open('$out/$f.jsonl'):
    j=json.loads(l); a=j['adapter']
    print('$f', j['config'], j.get('cpu_s'), j.get('gpu_s'), j.get('speedup'), j.get('outputs_equal'), a['gpu_finds'], a['cpu_finds'], a['cpu_why'])
"; done
