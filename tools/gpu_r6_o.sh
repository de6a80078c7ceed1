#!/bin/bash
# round 6: C4 U mode / C3 carry chain with the new defaults (swizzle y ^ x, one-shift fill, 32-bit lane sums):
# parity suites, A/B against the round-5 settings (libugrep_amd_r5.so), one VALU PMC pass on C4
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd); out=$root/gpurun_out/r6o; rm -rf $out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_xu.py tests/test_xc.py tests/test_wsub.py tests/test_gpu.py "tests/test_c5.py::test_offsets_record_by_record" -x -v -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
grep -E "passed|failed" $out/tests.log | tail -2
for run in 1 2; do
for cfg in c4 c3; do
  for lib in default r5; do
    if [ $lib = default ]; then L=libugrep_amd.so; else L=libugrep_amd_$lib.so; fi
    UGPU_LIB=$L timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --pcie-sample-mib 0 --steps 20 > $out/b_${cfg}_$lib.json 2> $out/b_${cfg}_$lib.err || { tail -5 $out/b_${cfg}_$lib.err; exit 1; }
    python3 -c "import json;j=json.load(open('$out/b_${cfg}_$lib.json'));print('$cfg $lib', j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['matches'], j['digest'])" | tee -a $out/summary.txt
  done
done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/pmc1 -o run -- python3 $root/bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --pcie-sample-mib 0 > $out/pmc1.json 2> $out/pmc1.err || { tail -5 $out/pmc1.err; exit 1; }
cd $root
python3 - $out <<'PY' | tee $out/pmc_summary.txt
import glob, json, sqlite3, sys, csv
d = sys.argv[1]
dbs = glob.glob(d + "/pmc1/**/*.db", recursive=True)
if dbs:
    c = sqlite3.connect(dbs[0])
    k = c.execute("select kernel_name, max(dispatch_id) from counters_collection where kernel_name like '%xu_kernel%' group by kernel_name").fetchall()
    for name, disp in k:
        rows = dict(c.execute("select counter_name, sum(value) from counters_collection where kernel_name=? and dispatch_id=? group by counter_name", (name, disp)).fetchall())
        print(name, json.dumps({a: round(b) for a, b in rows.items()}))
else:
    for f in glob.glob(d + "/pmc1/**/*counter_collection*.csv", recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if "xu_kernel" in r.get("Kernel_Name", ""):
                key = (r["Kernel_Name"][:60], r["Dispatch_Id"])
                agg.setdefault(key, {})[r["Counter_Name"]] = agg.setdefault(key, {}).get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        for key, v in list(agg.items())[-2:]:
            print(key, json.dumps({a: round(b) for a, b in v.items()}))
PY
