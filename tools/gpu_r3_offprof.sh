# rocprofv3 kernel trace of the C3 and C4 --offsets bench commands
set -o pipefail
out=$(pwd)/gpurun_out/r3off
mkdir -p $out
root=$(pwd)
cd /tmp
export TMPDIR=/tmp
for c in c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$c -o run -- python3 $root/bench.py --config $c --offsets --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_$c.json 2> $out/trace_$c.err || exit 1
done
cd $root
for c in c3 c4; do python3 tools/pmc_summary.py $out/trace_$c xc_kernel xg_kernel > $out/summary_$c.json; done
python3 - <<'PY'
import json
for c in ("c3", "c4"):
    s = json.load(open("gpurun_out/r3off/summary_%s.json" % c))
    for k in s["kernels"][:8]:
        print(c, k["name"][:60], k["calls"], k["avg_us"], k["pct"])
PY
