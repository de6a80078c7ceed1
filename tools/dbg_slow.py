"""Debug: time find_all for patterns over growing sizes (prints as it goes)."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import ugrep_amd as U  # noqa: E402
from oracle_lib import gen  # noqa: E402

for rx in sys.argv[1:]:
    opc = U.compile_regex(rx)
    pat = U.Pattern(opc)
    print(rx, pat.info(), flush=True)
    for mib in (1, 4, 16):
        host = gen(4, 11, 0, mib << 20)
        dev = torch.from_numpy(host).to("cuda")
        torch.cuda.synchronize()
        t = time.time()
        r = U.find_all(pat, dev)
        print("  %d MiB: %.3f s count %d" % (mib, time.time() - t, r.count), flush=True)
