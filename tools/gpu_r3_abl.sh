# Round 3: U-mode ablations on C4 (LDS conflicts / LDS / loads only) and the xg baseline.
# usage: tools/gpu_r3_abl.sh TAG LIB...
set -o pipefail
out=gpurun_out/${1:-r3abl}; shift
mkdir -p $out
for lib in "$@"; do
  UGPU_XU=1 UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/u_$lib.json 2> $out/u_$lib.err || { tail -5 $out/u_$lib.err; exit 1; }
  python -c "import json; j=json.load(open('$out/u_$lib.json')); print('U $lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])"
done
timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/xg.json 2> $out/xg.err || { tail -5 $out/xg.err; exit 1; }
python -c "import json; j=json.load(open('$out/xg.json')); print('xg', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'])"
