# records path: pipeline time vs native decode time (per config, 256 MiB host buffer)
import sys, os, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import ugrep_amd as U
from oracle_lib import gen
for name, rx, kind in [("c3", "[A-Za-z_][A-Za-z0-9_]*", 3), ("c4", r"\w+", 4)]:
    pat = U.Pattern(U.compile_regex(rx))
    buf = gen(kind, 1, 0, 256 << 20)
    for chunk in (16 << 20, 64 << 20):
        os.environ["UGPU_REC_CHUNK"] = str(chunk)
        U.Records(pat, buf).drain()
        tc = td = 1e9
        for _ in range(3):
            t0 = time.perf_counter(); r = U.Records(pat, buf); t1 = time.perf_counter(); r.drain(); t2 = time.perf_counter()
            tc = min(tc, t1 - t0); td = min(td, t2 - t1); r.close()
        print(json.dumps(dict(cfg=name, chunk=chunk, create_ms=round(tc * 1e3, 2), drain_ms=round(td * 1e3, 2))), flush=True)
