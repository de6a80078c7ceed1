#!/bin/bash
# round 6 closing measurement (one MI355X):
#   per config (c2 = the default command, c3, c4): the exact bench command under a
#   trace-only rocprofv3 pass (the line and its kernel times come from the same
#   run), then one FETCH_SIZE pass (HBM bytes per launch); the OFFSETS lines;
#   tools/pmc_summary.py condenses each config into gpurun_out/r06e/<c>/summary.json
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r06e
rm -rf $out; mkdir -p $out
for c in c2 c3 c4; do
  d=$out/$c; mkdir -p $d
  if [ $c = c2 ]; then a=""; else a="--config $c"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/trace -o run -- python3 -u bench.py $a > $d/bench.json 2> $d/bench.err || { tail $d/bench.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $d/pmc1 -o run -- python3 -u bench.py $a --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $d/pmc1.json 2> $d/pmc1.err || { tail $d/pmc1.err; exit 1; }
  python3 tools/pmc_summary.py $d > $d/summary.json
  python3 -c "import json;s=json.load(open('$d/summary.json'));b=s['bench'];print('$c', b['ms_per_step'], b['value'], s.get('kernel_ms'), s.get('kernel_ms_bench'), s.get('traffic_over_algorithmic'))"
done
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --offsets --no-cpu-baseline --pcie-sample-mib 0 > $out/offsets_$c.json 2> $out/offsets_$c.err || { tail $out/offsets_$c.err; exit 1; }
  python3 -c "import json;j=json.load(open('$out/offsets_$c.json'));print('$c offsets', j['ms_per_step'], j['offsets'])"
done
# W subset mode, lookahead (compiled), dominated restarts: one line each on the C2 corpus
timeout -k 10 300 python3 bench.py --config c2 --regex '[A-Za-z]+' --word --no-cpu-baseline --pcie-sample-mib 0 > $out/w_azAZ.json 2> $out/w_azAZ.err || { tail $out/w_azAZ.err; exit 1; }
timeout -k 10 300 python3 bench.py --config c2 --regex '[a-z]+(ing|ed)' --no-cpu-baseline --pcie-sample-mib 0 > $out/dom_inged.json 2> $out/dom_inged.err || { tail $out/dom_inged.err; exit 1; }
for f in w_azAZ dom_inged; do
  python3 -c "import json;j=json.load(open('$out/$f.json'));print('$f', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'])"
done
# (last: a lookahead table runs wfind_kernel over all 16 GiB; bounded steps, and nothing runs after it)
timeout -k 10 180 python3 bench.py --config c2 --regex 'foo(?=bar)' --steps 3 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/look_foobar.json 2> $out/look_foobar.err || { tail $out/look_foobar.err; exit 1; }
python3 -c "import json;j=json.load(open('$out/look_foobar.json'));print('look_foobar', j['ms_per_step'], j['roofline']['kernel'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'])"
