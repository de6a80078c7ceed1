# debug: option-W stream with flushed feeds vs the oracle (one pattern)
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch
import ugrep_amd as U
from oracle_lib import OracleDfa
from test_multi import _w_corpus
rx = sys.argv[1] if len(sys.argv) > 1 else "de|dei|é"
data = _w_corpus(1 << 20)
rng = np.random.default_rng(5)
opc = U.compile_regex(rx)
pat = U.Pattern(opc, word=True)
want = OracleDfa(opc).find_w(data, want_list=True)[3]
for rep in range(2):
    cuts = sorted(set(int(x) for x in rng.integers(1, data.size, 60)))
    for flush in (False, True):
        st = U.Stream(pat, keep=4096)
        trip, i, log = [], 0, []
        for c in cuts + [data.size]:
            r = st.feed(data[i:c].tobytes(), final=c == data.size, flush=flush and c < data.size)
            t = r.triples()
            log.append((i, c, st.settled(), len(t), t[0] if t else None, t[-1] if t else None))
            trip += t
            i = c
        ok = trip == want
        print("rep", rep, "flush", flush, "ok", ok, len(trip), len(want))
        if not ok:
            k = next(j for j in range(min(len(trip), len(want))) if trip[j] != want[j])
            print("first diff", k, trip[k - 2:k + 2], want[k - 2:k + 2])
            for e in log:
                print(e)
            p = want[k][0]
            print(bytes(data[p - 12:p + 8]))
            sys.exit(1)
