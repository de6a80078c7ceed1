# round 5: what the C3 bits pass (xc_bm_kernel) pays for: bits stored into
# 32 KiB (xa1, L2-resident) and not stored (xa2) against the real pass
# (benchmarking builds; their records are wrong, so only the bits pass's time
# is read from the trace)
set -o pipefail
out=gpurun_out/r5ah; mkdir -p $out
export TMPDIR=/tmp
for lib in libugrep_amd.so libugrep_amd_xa1.so libugrep_amd_xa2.so; do
  (cd /tmp && UGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/$lib -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --offsets --steps 3 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $GRAFT_REPO_ROOT/$out/$lib.json 2> $GRAFT_REPO_ROOT/$out/$lib.err); echo "rc $?"
  f=$(find $out/$lib -name '*kernel_stats.csv' | head -1); grep -E "xc_bm|xc_kernel|xc_expand" "$f" | cut -d, -f1-4
done
