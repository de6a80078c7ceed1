# round 5: C4 U-mode A/B (byte-wise counts vs v_bcnt/v_dot4), U-mode and word-boundary
# GPU tests, word-boundary bench lines on sparse_kernel, LDS/issue PMC, VALU probe
set -o pipefail
out=gpurun_out/r5b; mkdir -p $out
timeout -k 10 120 ./tools/probe/valu_rate > $out/valu_rate.txt 2>&1 || { cat $out/valu_rate.txt; exit 1; }
cat $out/valu_rate.txt
timeout -k 10 600 python -u -m pytest tests/test_xu.py tests/test_wordb.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for lib in libugrep_amd_cnt0.so libugrep_amd.so libugrep_amd_pk.so; do
  UGPU_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 > $out/$lib.$rep.json 2> $out/$lib.$rep.err || { tail -5 $out/$lib.$rep.err; exit 1; }
  python -c "import json; j=json.load(open('$out/$lib.$rep.json')); print('$lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['digest'])"
done
done
for rx in '\bfoo\b' '\<(in|ut)\>'; do
  tag=$(echo "$rx" | tr -c 'a-z' '_')
  timeout -k 10 300 python bench.py --config c2 --regex "$rx" --cpu-sample-mib 1024 --pcie-sample-mib 0 > $out/wb_$tag.json 2> $out/wb_$tag.err || { tail -5 $out/wb_$tag.err; exit 1; }
  python -c "import json; j=json.load(open('$out/wb_$tag.json')); print(j['config']['pattern'], j['ms_per_step'], j['roofline'], j.get('parity_vs_reference',{}).get('equal'), j['cpu_baseline']['value'])"
done
timeout -k 10 600 python bench.py --config c2 --regex '[a-z]+ing' --word --steps 3 --warmup 1 --cpu-sample-mib 256 --pcie-sample-mib 0 > $out/wb_w_ing.json 2> $out/wb_w_ing.err || { tail -5 $out/wb_w_ing.err; exit 1; }
python -c "import json; j=json.load(open('$out/wb_w_ing.json')); print(j['config']['pattern'], j['ms_per_step'], j['roofline'], j.get('parity_vs_reference',{}).get('equal'), j['cpu_baseline']['value'])"
bash tools/pmc_lds.sh r5b_c4 c4 && python3 tools/pmc_summary.py gpurun_out/pmc_r5b_c4 > $out/pmc_lds.json 2>&1; tail -30 $out/pmc_lds.json
timeout -k 10 600 python -u -m pytest tests/test_redo.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/redo_tests.log 2>&1 || { tail -30 $out/redo_tests.log; exit 1; }
tail -1 $out/redo_tests.log
