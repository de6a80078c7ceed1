import sys, time, numpy as np, torch
sys.path.insert(0, "/root/repo")
import ugrep_amd as U
out = open(sys.argv[1], "w")
for run in [1 << 16, 1 << 18, 1 << 20]:
    n = 8 << 20
    host = np.frombuffer(b"xy " * (n // 3 + 1), np.uint8)[:n].copy()
    host[3 << 20:(3 << 20) + run] = ord("a")
    whole = torch.from_numpy(host).to("cuda")
    pat = U.Pattern(U.compile_regex("a+"))
    for off in (False, True):
        t0 = time.time()
        r = U.find_all(pat, whole, offsets=off)
        torch.cuda.synchronize()
        print("run %d offsets %d: %.3f s count %d info %s" % (run, off, time.time() - t0, r.count, pat.info()), file=out, flush=True)
