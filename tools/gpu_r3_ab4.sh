# Round 3: C4 / C3 COUNT, C4 -w and C4 OFFSETS over library variants, one box.
# usage: tools/gpu_r3_ab4.sh TAG LIB...
set -o pipefail
out=gpurun_out/${1:-r3ab4}; shift
mkdir -p $out
b="--steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0"
for lib in "$@"; do
  for v in "c4" "c3" "c4 --word" "c4 --offsets"; do
    tag=$(echo "$v" | tr -d ' -')_$lib
    UGPU_LIB=$lib timeout -k 10 200 python bench.py --config $v $b > $out/$tag.json 2> $out/$tag.err || { tail -5 $out/$tag.err; exit 1; }
    python -c "import json; j=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('%-28s' % '$tag', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['matches'], j['digest'])"
  done
done
