# U mode and neighbours: GPU tests of xc/xg/xu/word, then C4 (U forced) and C4 -w bench lines.
set -o pipefail
out=gpurun_out/${1:-xut}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_xu.py tests/test_xg.py tests/test_word.py tests/test_xc.py -x -v --timeout 150 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
UGPU_XU=1 timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --verify > $out/bench_c4_xu.json 2> $out/bench_c4_xu.err || { tail -5 $out/bench_c4_xu.err; exit 1; }
UGPU_XU=1 timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --word > $out/bench_c4w_xu.json 2> $out/bench_c4w_xu.err || { tail -5 $out/bench_c4w_xu.err; exit 1; }
for f in bench_c4_xu bench_c4w_xu; do python -c "import json; j=json.load(open('$out/$f.json')); print('$f', j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['digest'])"; done
