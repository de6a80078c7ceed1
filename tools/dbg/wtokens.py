"""Token sets of \\w (2- and 3-byte) from the oracle, and the Boolean structure
of the 2-byte matrix (distinct lead rows, distinct continuation columns)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle_lib as O
from ugrep_amd.matcher import compile_regex
d = O.OracleDfa(compile_regex(r"\w+"))
# 2-byte: lead C0-DF x c1 80-BF, each as " L C "
seqs = [(l, c) for l in range(0xC0, 0xE0) for c in range(0x80, 0xC0)]
buf = np.frombuffer(b"".join(bytes([0x20, l, c, 0x20]) for l, c in seqs), np.uint8)
n, _, _, lst = d.find(buf, want_list=True)
ok2 = np.zeros((32, 64), bool)
for s, ln, cap in lst:
    if ln == 2 and s % 4 == 1:
        k = s // 4; ok2[seqs[k][0] - 0xC0, seqs[k][1] - 0x80] = True
rows = {tuple(r) for r in ok2}
cols = {tuple(c) for c in ok2.T}
print("2-byte tokens", ok2.sum(), "distinct lead rows", len(rows), "distinct cont cols", len(cols))
ok3 = np.zeros((16, 64, 64), bool)
buf = bytearray()
for l in range(0xE0, 0xF0):
    for c1 in range(0x80, 0xC0):
        for c2 in range(0x80, 0xC0):
            buf += bytes([0x20, l, c1, c2, 0x20])
buf = np.frombuffer(bytes(buf), np.uint8)
n, _, _, lst = d.find(buf, want_list=True)
for s, ln, cap in lst:
    if ln == 3 and s % 5 == 1:
        k = s // 5; ok3[k // 4096, (k // 64) % 64, k % 64] = True
blk = ok3.reshape(1024, 64)
full = blk.all(axis=1).sum(); empty = (~blk).all(axis=1).sum()
print("3-byte tokens", ok3.sum(), "(lead,c1) blocks: full", full, "empty", empty, "mixed", 1024 - full - empty,
      "distinct mixed masks", len({tuple(r) for r in blk if r.any() and not r.all()}))
np.savez("/tmp/wtok.npz", ok2=ok2, ok3=ok3)
