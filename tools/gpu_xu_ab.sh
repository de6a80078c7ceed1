# A/B of U-mode builds on C4 (UGPU_XU=1): kernel time and digest check per library.
# Usage: tools/gpu_xu_ab.sh TAG LIB...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for lib in "$@"; do
  UGPU_XU=1 UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --verify > $out/$lib.json 2> $out/$lib.err || { tail -5 $out/$lib.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$lib.json')); print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['digest'], j['verified_whole_stream'])"
done
