# One-GPU check: full -m gpu suite, smoke, default bench (C2). Usage: tools/gpu_check.sh TAG
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $out/gpu_all.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || exit 1
