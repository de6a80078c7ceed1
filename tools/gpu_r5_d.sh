# round 5: ugrep end to end (reference build against the drop-in build), and
# one rocprofv3 kernel + HIP API trace of ugrep_gpu -co -J16 on C3 / C4 files
set -o pipefail
out=gpurun_out/r5d; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_ugrep.py --files 16 --mib 256 --reps 2 > $out/bench_ugrep.jsonl 2> $out/bench_ugrep.err || { tail -20 $out/bench_ugrep.err; exit 1; }
cat $out/bench_ugrep.jsonl
for cfg in c3:3 c4:4; do
  name=${cfg%%:*}; kind=${cfg##*:}
  d=/tmp/ug_$name; mkdir -p $d
  python -c "
import sys; sys.path.insert(0,'tests')
from oracle_lib import gen
for k in range(16): gen($kind, 1, k * (256 << 20), 256 << 20).tofile('$d/f%02d.txt' % k)
"
  rx='[A-Za-z_][A-Za-z0-9_]*'; [ $name = c4 ] && rx='\w+'
  # the program itself right after --
  (cd /tmp && UGPU_ADAPTER_STATS=1 UGPU_REC_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_$name -o run -- $GRAFT_REPO_ROOT/oracle/_ref/ugrep_gpu -co -J16 "$rx" $d/f00.txt $d/f01.txt $d/f02.txt $d/f03.txt $d/f04.txt $d/f05.txt $d/f06.txt $d/f07.txt $d/f08.txt $d/f09.txt $d/f10.txt $d/f11.txt $d/f12.txt $d/f13.txt $d/f14.txt $d/f15.txt > $GRAFT_REPO_ROOT/$out/prof_$name.out 2> $GRAFT_REPO_ROOT/$out/prof_$name.err) || { echo "prof $name failed"; tail -5 $out/prof_$name.err; exit 1; }
  rm -rf $d
done
echo done
