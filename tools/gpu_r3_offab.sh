# Round 3: OFFSETS A/B over library variants (C4 and C3 --offsets).
# usage: tools/gpu_r3_offab.sh TAG LIB...
set -o pipefail
out=gpurun_out/${1:-r3offab}; shift
mkdir -p $out
b="--steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0"
for lib in "$@"; do
  for c in c4 c3; do
    UGPU_LIB=$lib timeout -k 10 200 python bench.py --config $c --offsets $b > $out/${c}_$lib.json 2> $out/${c}_$lib.err || { tail -5 $out/${c}_$lib.err; exit 1; }
    python -c "import json; j=json.loads(open('$out/${c}_$lib.json').read().strip().splitlines()[-1]); print('$c $lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['matches'], j.get('offsets', {}).get('digest_matches_totals'))"
  done
done
