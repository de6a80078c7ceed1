set -o pipefail
mkdir -p gpurun_out/dropin
timeout -k 10 600 python -u -m pytest tests/test_adapter.py tests/test_ugrep_dropin.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/dropin/t.log 2>&1
