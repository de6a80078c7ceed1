# U mode quick check: GPU tests then the C4 bench line.  Usage: tools/gpu_xu_quick.sh TAG
set -o pipefail
tag=${1:-xuq}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xu.py -x -v --timeout 150 --timeout-method thread > $out/test_xu.log 2>&1 || { tail -40 $out/test_xu.log; exit 1; }
tail -2 $out/test_xu.log
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --pcie-sample-mib 0 --verify > $out/bench_c4.json 2> $out/bench_c4.err || { tail -20 $out/bench_c4.err; exit 1; }
python -c "import json; j=json.load(open('$out/bench_c4.json')); print(j['ms_per_step'], j['roofline'])"
