# Round 3: records path with the pack kernel storing straight into pinned
# memory (UGPU_REC_ZC=1) against the D2H copy, C4/C3/C2 at 256 MiB, then the
# record tests with zero copy on.
set -o pipefail
out=gpurun_out/${1:-r3zc}
mkdir -p $out
for c in c4 c3 c2; do
  for zc in 1 0; do
    UGPU_REC_ZC=$zc UGPU_REC_TRACE=1 timeout -k 10 120 python tools/rec_trace.py $c 256 2> $out/${c}_zc$zc.txt || { tail -5 $out/${c}_zc$zc.txt; exit 1; }
  done
done
grep "rep 2" $out/*.txt
UGPU_REC_ZC=1 timeout -k 10 600 python -u -m pytest tests/test_records.py tests/test_adapter.py tests/test_ugrep_dropin.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
