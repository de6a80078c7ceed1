"""LDS cycles of byte-lookup layouts on the C4 corpus (simulated banking:
32 banks of dwords per 32-lane group, cycles = max distinct dwords per bank).
Lane l holds bytes [16 l, 16 l + 16) of a 1 KiB chunk; instruction k reads
the entry for byte k of every lane."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle_lib as O

N = 1 << 22
b = O.gen(4, 1, 0, N + 8).astype(np.int64)
x = b[:N]
y = b[1:N + 1]


def cycles(addr_bytes, active=None):
    """addr_bytes: byte address per position (N,), u8 reads.  Returns mean LDS
    cycles per wave-instruction (two 32-lane groups)."""
    d = (addr_bytes >> 2).reshape(-1, 64, 16)           # chunk, lane, k
    d = d.transpose(0, 2, 1).reshape(-1, 2, 32)          # instr, group, lane
    if active is not None:
        a = active.reshape(-1, 64, 16).transpose(0, 2, 1).reshape(-1, 2, 32)
        d = np.where(a, d, -1)
    tot = 0
    bank = np.where(d >= 0, d & 31, 32)
    # distinct dwords per (instr, group, bank)
    key = (bank << 40) | np.where(d >= 0, d, (1 << 40) - 1)
    key = np.sort(key, axis=2)
    new = np.ones_like(key, dtype=bool)
    new[:, :, 1:] = key[:, :, 1:] != key[:, :, :-1]
    bk = key >> 40
    cnt = np.zeros(bk.shape[:2] + (33,), np.int64)
    for j in range(32):
        np.add.at(cnt, (np.arange(bk.shape[0])[:, None], np.arange(2)[None, :], bk[:, :, j]), new[:, :, j])
    cnt[:, :, 32] = 0
    per = np.maximum(cnt.max(axis=2), 1)
    return per.sum(axis=1).mean()


sw = x << 8 | (y ^ ((x << 2) & 0xfc))
print("U swizzled pair table      %.2f" % cycles(sw))
print("plain pair x<<8|y          %.2f" % cycles(x << 8 | y))
print("byte table (256 B)         %.2f" % cycles(x))
lead = x >= 0xC0
asc = x < 0x80
coll = np.where(lead, sw, np.where(asc, (x << 8) | ((x << 2) & 0xfc), 0xFF00 | y))
print("collapsed rows             %.2f" % cycles(coll))
print("leads only (others masked) %.2f" % cycles(sw, lead))
print("fraction lead %.3f ascii %.3f cont %.3f" % (lead.mean(), asc.mean(), ((x >= 0x80) & (x < 0xC0)).mean()))
l3 = (x >= 0xE0) & (x < 0xF0)
print("3-byte leads %.3f" % l3.mean())
z = b[2:N + 2]
bm3 = 4096 + (((x & 15) << 12 | (y & 63) << 6 | (z & 63)) >> 3)
print("3-byte bitmap, 3-leads only %.2f" % cycles(bm3, l3))
# 2-byte lead (lead & 0x1F) qword bitmaps via ds_read_b64: conflict-free

print("--- variants")
asc = x < 0x80
c2 = (x << 2) & 0xfc
def sw_of(lo_fn):
    return lo_fn
v2 = np.where(asc, x << 8 | c2, sw)
print("ASCII rows collapsed (bank x&31)          %.2f" % cycles(v2))
f = ((x ^ ((x >> 5) & 1) * 0x10) << 2) & 0xfc
v3 = np.where(asc, x << 8 | f, sw)
print("ASCII collapsed, upper/lower split        %.2f" % cycles(v3))
cont = (x >= 0x80) & (x < 0xC0)
v4 = np.where(cont, x << 8 | ((x << 2) & 0xfc), v3)
print("+ cont rows collapsed (no y class: ideal) %.2f" % cycles(v4))
print("ASCII lanes only (current)                %.2f" % cycles(sw, asc))
print("cont lanes only (current)                 %.2f" % cycles(sw, cont))
print("lead lanes only (current)                 %.2f" % cycles(sw, x >= 0xC0))
