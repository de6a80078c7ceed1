"""Debug: fix_kernel rounds and wall time of a non-resynchronising dense scan."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import ugrep_amd as U  # noqa: E402
from oracle_lib import OracleDfa, gen  # noqa: E402

rx = sys.argv[1] if len(sys.argv) > 1 else r"\D\D"
opc = U.compile_regex(rx)
pat = U.Pattern(opc)
o = OracleDfa(opc)
print(rx, pat.info(), flush=True)
for kib in (64, 256, 1024):
    n = kib << 10
    host = gen(4, 11, 0, n)
    dev = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    dev[:n].copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    sc = U.Scanner(pat)
    t = time.time()
    sc.scan(dev.data_ptr(), 0, n, n, True, 0)
    tt = sc.totals()
    dt = time.time() - t
    want = o.find(host)[:3]
    print("  %d KiB: %.3f s rounds %d kernel_ms %.3f count %d ok %s" % (
        kib, dt, tt.fix_rounds, sc.kernel_ms(), tt.count, (tt.count, tt.digest, tt.dcap) == want), flush=True)
