# round 5: ugrep end to end (reference build vs drop-in): option W without a prefilter, and C3
set -o pipefail
out=gpurun_out/r5ab; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_ugrep.py --files 16 --mib 256 --reps 2 --configs c3_wazAZ,c3 > $out/e2e_w.jsonl 2> $out/e2e_w.err || { tail -20 $out/e2e_w.err; cat $out/e2e_w.jsonl; exit 1; }
python -c "
import json
for l in open('$out/e2e_w.jsonl'):
    d=json.loads(l); print(d['config'], d.get('pattern'), d.get('flags'), d['cpu_s'], d['gpu_s'], d.get('speedup'), d['outputs_equal'], d['adapter'].get('gpu_finds'), d['adapter'].get('cpu_finds'), d['adapter'].get('cpu_why'))"
