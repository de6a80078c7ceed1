# round 5: ugrep end to end, stream feeds: reservation on/off, feed size 4/8 MiB
set -o pipefail
out=${OUT:-gpurun_out/r5g}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stream.py tests/test_ugrep_dropin.py -x -v --timeout 300 --timeout-method thread -m gpu > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in ${VARIANTS:-"R1C8:1:8388608" "R0C8:0:8388608" "R1C4:1:4194304" "R0C4:0:4194304"}; do
  name=${v%%:*}; rest=${v#*:}; r=${rest%%:*}; ch=${rest#*:}
  UGPU_ADAPTER_RESERVE=$r UGPU_ADAPTER_CHUNK=$ch timeout -k 10 400 python -u tools/bench_ugrep.py --files 16 --mib 256 --reps ${REPS:-2} --configs c3,c4 > $out/bench_$name.jsonl 2> $out/bench_$name.err || { tail -20 $out/bench_$name.err; exit 1; }
  echo "== $name"; grep -v startup $out/bench_$name.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); a = d['adapter']
    print(d['config'], d['cpu_s'], d['gpu_s'], d['speedup'], d['outputs_equal'], 'cpu_finds', a['cpu_finds'], 'read_max', a['read_ms_max'], 'feed_max', a['feed_ms_max'])
"
done
echo done
