# usage: tools/pmc_issue.sh TAG CONFIG [LIB]: one rocprofv3 --pmc pass of issue/wait counters over a short bench
set -o pipefail
tag=$1; cfg=$2; lib=${3:-libugrep_amd.so}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp && UGPU_LIB=$lib timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $out/p -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 2 --warmup 0 --no-cpu-baseline --pcie-sample-mib 0 > /dev/null 2> $out/err
