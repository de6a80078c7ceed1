"""Debug: \\w+ under option W, fast path vs wfind vs oracle (GPU)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import ugrep_amd as U
from oracle_lib import OracleDfa, gen

for kind, rx in ((3, "[A-Za-z_][A-Za-z0-9_]*"), (4, r"\w+")):
    host = gen(kind, 9, 0, 24 << 20)
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    opc = U.compile_regex(rx)
    pat = U.Pattern(opc, word=True)
    print(rx, pat.info(), flush=True)
    want = OracleDfa(opc).find_w(host)[:3]
    sc = U.Scanner(pat)
    sc.scan(dev.data_ptr(), 0, host.size, host.size, True, 0, torch.cuda.current_stream().cuda_stream)
    t = sc.totals()
    print(" scanner", (t.count, t.digest, t.dcap), t.flags, "want", want, flush=True)
    r = U.find_all(pat, dev, offsets=False)
    print(" find_all count", (r.count, r.digest, r.dcap), flush=True)
    try:
        r = U.find_all(pat, dev, offsets=True)
        print(" find_all offsets", (r.count, r.digest, r.dcap), flush=True)
    except Exception as e:
        print(" offsets failed", e, flush=True)
    plain = OracleDfa(opc).find(host)[:3]
    print(" plain FIND", plain, flush=True)
