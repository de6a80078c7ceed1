# round 5: OFFSETS expansion A/B (one wave per COUNT wave, no counting pass,
# against the four-quarter kernel), record tests, WRITE/FETCH PMC passes
set -o pipefail
out=gpurun_out/r5c; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_c5.py::test_offsets_record_by_record tests/test_xc.py tests/test_xu.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for cfg in c4 c3; do
for nw in 4 1; do
  UGPU_XE_WAVES=$nw timeout -k 10 300 python bench.py --config $cfg --offsets --no-cpu-baseline --pcie-sample-mib 0 > $out/$cfg.$nw.$rep.json 2> $out/$cfg.$nw.$rep.err || { tail -5 $out/$cfg.$nw.$rep.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$cfg.$nw.$rep.json')); print('$cfg nw=$nw', j['ms_per_step'], j['roofline']['kernel_ms'], j['offsets'])"
done
done
done
export TMPDIR=/tmp
for cfg in c4 c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $GRAFT_REPO_ROOT/$out/pmc_${cfg}_$ctr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --offsets --steps 2 --warmup 0 --no-cpu-baseline --pcie-sample-mib 0 > /dev/null 2> $GRAFT_REPO_ROOT/$out/pmc_${cfg}_$ctr.err) || { echo "pmc $cfg $ctr failed"; tail -3 $out/pmc_${cfg}_$ctr.err; exit 1; }
  done
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace_$cfg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --offsets --steps 5 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $GRAFT_REPO_ROOT/$out/trace_$cfg.json 2> $GRAFT_REPO_ROOT/$out/trace_$cfg.err) || { echo "trace $cfg failed"; exit 1; }
done
echo done
