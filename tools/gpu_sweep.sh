# usage: tools/gpu_sweep.sh TAG CONFIG LIB... : bench + FETCH_SIZE per library variant
set -o pipefail
tag=$1; cfg=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out/sweep_$tag
mkdir -p $out
export TMPDIR=/tmp
for lib in "$@"; do
  UGPU_LIB=$lib timeout -k 10 200 python $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/$lib.json 2> $out/$lib.err || exit 1
  (cd /tmp && UGPU_LIB=$lib timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc_$lib -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 2 --warmup 0 --no-cpu-baseline --pcie-sample-mib 0 > /dev/null 2> $out/pmc_$lib.err) || exit 1
done
