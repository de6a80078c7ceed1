# round 5: C3 / C4 OFFSETS step, kernel breakdown (trace only)
set -o pipefail
out=gpurun_out/r5ae; mkdir -p $out
export TMPDIR=/tmp
for c in c3 c4; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --offsets --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $GRAFT_REPO_ROOT/$out/$c.json 2> $GRAFT_REPO_ROOT/$out/$c.err) || { tail -5 $out/$c.err; exit 1; }
  f=$(find $out/$c -name '*kernel_stats.csv' | head -1); head -10 "$f" | cut -c1-160
  python3 -c "import json;j=json.load(open('$out/$c.json'));print('$c', j['ms_per_step'])"
done
