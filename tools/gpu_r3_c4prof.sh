# Round 3: the C4 bench line (CPU baseline + reference parity) and the
# rocprofv3 summary of the same command on the same box.
set -o pipefail
tag=${1:-r3c4p}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u bench.py --config c4 > $out/bench_c4.json 2> $out/bench_c4.err || exit 1
PMC3=1 bash tools/profile.sh ${tag}_c4 c4 > /dev/null 2> $out/prof_c4.err || exit 1
cp gpurun_out/prof_${tag}_c4/summary.json $out/summary_c4.json
python3 -c "
import json
b=json.loads(open('$out/bench_c4.json').read().strip().splitlines()[-1]); s=json.load(open('$out/summary_c4.json'))
print('bench', b['ms_per_step'], b['roofline']['kernel_ms'], b['roofline']['frac'], b.get('cpu_baseline',{}).get('value'), b.get('parity_vs_reference'))
print('trace', s.get('kernel_ms'), s.get('kernel_ms_bench'), s.get('traffic_over_algorithmic'), s.get('effective_clock_ghz'))"
