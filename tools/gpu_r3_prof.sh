# Round-3 measurement pass (one MI355X): default bench line, C3/C4 lines with
# cpu_baseline + parity, C4 with offsets, and rocprofv3 summaries (trace +
# FETCH_SIZE + wave counters) of the same commands, per config.
# usage: tools/gpu_r3_prof.sh TAG
set -o pipefail
tag=${1:-r3p}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --config c3 > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
timeout -k 10 300 python -u bench.py --config c4 > $out/bench_c4.json 2> $out/bench_c4.err || exit 1
timeout -k 10 300 python -u bench.py --config c4 --offsets --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_c4_offsets.json 2> $out/bench_c4_offsets.err || exit 1
timeout -k 10 300 python -u bench.py --config c3 --offsets --no-cpu-baseline --pcie-sample-mib 0 > $out/bench_c3_offsets.json 2> $out/bench_c3_offsets.err || exit 1
for c in c2 c3 c4; do
  PMC3=1 bash tools/profile.sh ${tag}_$c $c > /dev/null 2> $out/prof_$c.err || exit 1
  cp gpurun_out/prof_${tag}_$c/summary.json $out/summary_$c.json
done
for f in $out/bench_*.json; do echo "$f: $(cut -c1-400 $f)"; done
