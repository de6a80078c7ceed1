#!/bin/bash
# One PMC pass (VALU/SALU/LDS instruction counts, LDS conflicts, wave cycles)
# over a short bench run: tools/pmc_quick.sh TAG CONFIG [ablate]
set -e -o pipefail
tag=$1; cfg=$2; ab=${3:-0}
root=$(pwd); out=$root/gpurun_out/pmcq_$tag
rm -rf "$out"; mkdir -p "$out"
export TMPDIR=/tmp UGPU_ABLATE=$ab
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d "$out/pmc1" -o run -- \
    python3 "$root/bench.py" --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline > "$out/bench.json" 2> "$out/err"
cd "$root"
python3 - "$out" <<'PY'
import glob, json, sqlite3, sys
d = sys.argv[1]
c = sqlite3.connect(glob.glob(d + "/pmc1/**/*.db", recursive=True)[0])
k = c.execute("select kernel_name, max(dispatch_id) from counters_collection where kernel_name like '%dense_kernel%' or kernel_name like '%sparse_kernel%' group by kernel_name").fetchall()
for name, disp in k:
    rows = dict(c.execute("select counter_name, sum(value) from counters_collection where kernel_name=? and dispatch_id=? group by counter_name", (name, disp)).fetchall())
    print(name, json.dumps({a: round(b) for a, b in rows.items()}))
PY
