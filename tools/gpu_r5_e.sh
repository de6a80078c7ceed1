# round 5: stream feeds on pooled resources -- stream/drop-in tests, ugrep end
# to end (default feed size and 32 MiB feeds), one kernel + HIP API trace of C3
set -o pipefail
out=${OUT:-gpurun_out/r5e}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stream.py tests/test_ugrep_dropin.py tests/test_redo.py -x -v --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 600 python -u tools/bench_ugrep.py --files 16 --mib 256 --reps 2 --configs c2,c3,c4 > $out/bench_ugrep.jsonl 2> $out/bench_ugrep.err || { tail -20 $out/bench_ugrep.err; exit 1; }
cat $out/bench_ugrep.jsonl
UGPU_ADAPTER_CHUNK=33554432 timeout -k 10 600 python -u tools/bench_ugrep.py --files 16 --mib 256 --reps 2 --configs c3,c4 > $out/bench_ugrep_32m.jsonl 2> $out/bench_ugrep_32m.err || { tail -20 $out/bench_ugrep_32m.err; exit 1; }
cat $out/bench_ugrep_32m.jsonl
d=/tmp/ug_c3; mkdir -p $d
python -c "
import sys; sys.path.insert(0,'tests')
from oracle_lib import gen
for k in range(16): gen(3, 1, k * (256 << 20), 256 << 20).tofile('$d/f%02d.txt' % k)
"
(cd /tmp && UGPU_ADAPTER_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_c3 -o run -- $GRAFT_REPO_ROOT/oracle/_ref/ugrep_gpu -co -J16 '[A-Za-z_][A-Za-z0-9_]*' $d/f00.txt $d/f01.txt $d/f02.txt $d/f03.txt $d/f04.txt $d/f05.txt $d/f06.txt $d/f07.txt $d/f08.txt $d/f09.txt $d/f10.txt $d/f11.txt $d/f12.txt $d/f13.txt $d/f14.txt $d/f15.txt > $GRAFT_REPO_ROOT/$out/prof_c3.out 2> $GRAFT_REPO_ROOT/$out/prof_c3.err) || { echo "prof failed"; tail -5 $out/prof_c3.err; exit 1; }
rm -rf $d
echo done
