# usage: tools/gpu_abl.sh TAG CONFIG ENV LIB... : bench lines (HIP-event kernel times) per
# library variant, ENV (e.g. UGPU_XU=1) applied to every run; ablation builds give wrong counts
set -o pipefail
tag=$1; cfg=$2; envs=$3; shift 3
out=$GRAFT_REPO_ROOT/gpurun_out/abl_$tag
mkdir -p $out
for lib in "$@"; do
  env $envs UGPU_LIB=$lib timeout -k 10 200 python $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --pcie-sample-mib 0 > $out/$lib.json 2> $out/$lib.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else d.get('kernel_ms'), d['roofline']['frac'])" $out/$lib.json $lib
done
