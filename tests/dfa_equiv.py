"""Language equivalence of two opcode tables, per accept index (test helper).

Two FIND tables give identical FIND results on every input iff, for every
byte string w, the accept index reached after w agrees (0 = not accepting),
counting states that can no longer reach an accept as dead: FIND
 only records the last accepting position of each walk.
`counterexample(a, b)` returns None when the tables are equivalent, else the
shortest byte string on which they differ.
"""
from collections import deque

import numpy as np



def _parse_opc(opc):
    """Opcode words -> (next[S][256], caps[S], start=1); state 0 is dead.
    Follows include/reflex/pattern.h:1155-1247, with no
    size limit, so large tables can be compared too."""
    opc = [int(w) for w in opc]
    ids = {0: 1}
    order = [0]
    rows, caps = [[0] * 256], [0]
    for pc in order:
        k, cap = pc, 0
        while (opc[k] >> 24) == 0xFE:
            cap = opc[k] & 0xFFFFFF
            k += 1
        row = [None] * 256
        left = 256
        while left:
            w = opc[k]
            lo, hi, idx = w >> 24, (w >> 16) & 0xFF, w & 0xFFFF
            assert lo < 0xFB, "unsupported opcode word %08x" % w
            if idx == 0xFFFE:
                tgt = opc[k + 1] & 0xFFFFFF
                k += 2
            else:
                tgt = None if idx == 0xFFFF else idx
                k += 1
            if tgt is not None and tgt not in ids:
                ids[tgt] = len(order) + 1
                order.append(tgt)
            for c in range(lo, hi + 1):
                if row[c] is None:
                    row[c] = 0 if tgt is None else ids[tgt]
                    left -= 1
        rows.append(row)
        caps.append(cap)
    return np.array(rows, np.int64), np.array(caps, np.int64)


class _Table:
    def __init__(self, opc):
        self.next, self.caps = _parse_opc(opc)
        self.start = 1
        # live = can reach an accepting state (reverse reachability)
        live = self.caps != 0
        changed = True
        while changed:
            nl = live | live[self.next].any(axis=1)
            nl[0] = False
            changed = bool((nl != live).any())
            live = nl
        self.live = live

    def norm(self, s):
        return s if self.live[s] else 0


def counterexample(opc_a, opc_b):
    a, b = _Table(opc_a), _Table(opc_b)
    s0 = (a.norm(a.start), b.norm(b.start))
    seen = {s0: None}
    q = deque([s0])
    while q:
        p = q.popleft()
        x, y = p
        if a.caps[x] != b.caps[y]:
            w = []
            while seen[p] is not None:
                p, byte = seen[p]
                w.append(byte)
            return bytes(reversed(w))
        if x == 0 and y == 0:
            continue
        nx, ny = a.next[x], b.next[y]
        for byte in range(256):
            r = (a.norm(nx[byte]), b.norm(ny[byte]))
            if r not in seen:
                seen[r] = (p, byte)
                q.append(r)
    return None
