# round 5: loop-needle lookback fuzz against the oracle
set -o pipefail
out=gpurun_out/r5ac; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_lookback.py -x -v --timeout 300 --timeout-method thread -m gpu -k "fuzz or word" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
