#!/bin/bash
# round 6: option-W walks through an 8-byte register word (UGPU_WREG): word
# tests, then the long-run A/B against the byte-load build
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r6y; rm -rf $out; mkdir -p $out
timeout -k 10 300 python3 -u tools/bench_wlong.py > $out/wlong_new.jsonl 2> $out/wlong_new.err || { tail -5 $out/wlong_new.err; exit 1; }
UGPU_LIB=libugrep_amd_wr0.so timeout -k 10 600 python3 -u tools/bench_wlong.py > $out/wlong_wr0.jsonl 2> $out/wlong_wr0.err || { tail -5 $out/wlong_wr0.err; exit 1; }
cat $out/wlong_new.jsonl $out/wlong_wr0.jsonl
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_word.py tests/test_wordb.py tests/test_lookback.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
