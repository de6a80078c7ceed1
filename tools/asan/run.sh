#!/bin/bash
# tools/asan/run.sh -- the host half under AddressSanitizer + UBSan (CPU only):
#   1. the fuzz harness (tools/asan/fuzz_host.cpp), 4 x N/4 patterns in parallel;
#   2. the host-side CPU tests (compiler, plan, tables) with the instrumented
#      libugpu_host.so loaded in place of the plain one (LD_LIBRARY_PATH wins
#      over libugrep_amd.so's RUNPATH) and the sanitizer runtimes preloaded.
# usage: tools/asan/run.sh [N]     (default 10000)
set -o pipefail
cd "$(dirname "$0")/../.."
N=${1:-10000}
make -C tools/asan -j4 >/dev/null || exit 1
OUT=ugrep_amd/build/asan
export ASAN_OPTIONS=halt_on_error=1:detect_leaks=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
pids=()
for s in 1 2 3 4; do
  ./$OUT/fuzz_host $((N / 4)) $s > $OUT/fuzz_$s.log 2>&1 &
  pids+=($!)
done
rc=0
for i in 0 1 2 3; do wait ${pids[$i]} || { echo "fuzz seed $((i + 1)) failed:"; tail -n 30 $OUT/fuzz_$((i + 1)).log; rc=1; }; done
[ $rc = 0 ] || exit 1
tail -q -n 1 $OUT/fuzz_*.log
# Python's own allocations are not instrumented: leak checks off for pytest
ASAN_OPTIONS=halt_on_error=1:detect_leaks=0 UGPU_NO_TORCH=1 LD_LIBRARY_PATH=$PWD/$OUT \
  LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so) \
  python3 -m pytest tests/test_compile.py tests/test_plan.py tests/test_host.py tests/test_dom.py -q -m "not gpu" -p no:cacheprovider \
  > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
grep -c "ERROR: AddressSanitizer\|runtime error:" $OUT/pytest.log $OUT/fuzz_*.log | grep -v ":0$" && exit 1
echo "asan/ubsan: clean"
