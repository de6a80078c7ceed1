# C5's 128 GiB stream on ONE MI355X (the baseline the 8-GPU run's speed-up is measured against),
# after a 40 GiB rehearsal of the same path.  Usage: tools/gpu_c5_one.sh TAG
set -o pipefail
out=gpurun_out/${1:-c5one}
mkdir -p $out
timeout -k 10 180 python bench.py --config c5 --bytes 42949672960 --no-cpu-baseline --pcie-sample-mib 0 --verify --steps 5 --warmup 2 > $out/bench_c5_40g.json 2> $out/bench_c5_40g.err || { tail -5 $out/bench_c5_40g.err; exit 1; }
python -c "import json; j=json.load(open('$out/bench_c5_40g.json')); print('40G', j['value'], j['ms_per_step'], j['roofline']['frac'], j['matches'], j.get('verified_whole_stream'))"
timeout -k 10 400 python bench.py --config c5 --cpu-sample-mib 2048 --pcie-sample-mib 0 --verify --steps 5 --warmup 2 > $out/bench_c5.json 2> $out/bench_c5.err || { tail -5 $out/bench_c5.err; exit 1; }
python -c "import json; j=json.load(open('$out/bench_c5.json')); print('128G', j['value'], j['ms_per_step'], j['roofline']['frac'], j['matches'], j.get('verified_whole_stream'), j.get('parity_vs_reference', {}).get('equal'))"
