# Round 3: kernel trace (--stats) of the OFFSETS bench steps, per config.
# usage: tools/gpu_r3_offprof2.sh TAG CONFIG...
set -o pipefail
tag=$1; shift
root=$(pwd)
export TMPDIR=/tmp
for c in "$@"; do
  out=$root/gpurun_out/$tag/$c
  mkdir -p $out
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 $root/bench.py --config $c --offsets --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/bench.json 2> $out/trace.err) || { tail -5 $out/trace.err; exit 1; }
  python3 tools/pmc_summary.py $out > $out/summary.json
  python3 -c "
import json; s=json.load(open('$out/summary.json'))
for k in s['kernels'][:8]: print('$c', k['name'][:60], k['calls'], k['avg_us'], k['total_us'])"
done
