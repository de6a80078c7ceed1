# round 5: C4 COUNT ablations on the current kernel: LDS lookups made
# broadcasts (no bank conflicts) and no LDS lookups (benchmarking; wrong counts)
set -o pipefail
out=gpurun_out/r5o; mkdir -p $out
for rep in 1 2; do
for lib in libugrep_amd.so libugrep_amd_abl1.so libugrep_amd_abl2.so; do
  UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 > $out/$lib.$rep.json 2> $out/$lib.$rep.err || { tail -5 $out/$lib.$rep.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$lib.$rep.json')); print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
done
echo done
