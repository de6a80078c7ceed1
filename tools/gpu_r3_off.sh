# Round 3: OFFSETS lines (C3, C4) and C4 -w on the default library and the
# given variants, then the given GPU test files.
# usage: tools/gpu_r3_off.sh TAG "LIB..." [TESTFILE...]
set -o pipefail
out=gpurun_out/${1:-r3off}; libs=$2; shift 2
mkdir -p $out
b="--steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0"
for c in c4 c3; do
  timeout -k 10 200 python bench.py --config $c --offsets $b > $out/off_$c.json 2> $out/off_$c.err || { tail -5 $out/off_$c.err; exit 1; }
done
for lib in libugrep_amd.so $libs; do
  UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --word $b > $out/w_$lib.json 2> $out/w_$lib.err || { tail -5 $out/w_$lib.err; exit 1; }
done
for f in $out/*.json; do python -c "import json; j=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['matches'], j['digest'], j.get('offsets', {}).get('digest_matches_totals'))"; done
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -q -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
fi
