#!/bin/bash
# kernel averages (rocprofv3 trace only) of one bench command under several in-tree library builds:
#   bash tools/gpu_prof_variants.sh "<bench args>" lib1.so lib2.so ...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ARGS=$1; shift
n=0
for lib in "$@"; do
  n=$((n+1))
  d=gpurun_out/pv_$n
  rm -rf $d
  UGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 -u bench.py $ARGS > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
  python3 - $d $lib <<'PY'
import sqlite3, glob, sys, json
d, lib = sys.argv[1], sys.argv[2]
con = sqlite3.connect(glob.glob(d + "/*.db")[0])
j = json.load(open(d + ".json"))
print(lib, "ms_per_step", j["ms_per_step"])
for name, calls, avg in con.execute("select name, total_calls, average from top_kernels limit 6"):
    if "ugpu" in name and "gen_kernel" not in name:
        print("   %-60s %4d %9.4f ms" % (name.split("(")[0][-60:], calls, avg / 1e3))
PY
done
