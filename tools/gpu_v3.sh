# GPU check after the W path: word tests first, then the whole -m gpu suite.
mkdir -p gpurun_out/v3
timeout -k 10 300 python -u -m pytest tests/test_word.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v3/gpu_word.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/v3/gpu_all.log 2>&1 || exit 1
