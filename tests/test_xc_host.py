"""CPU: the two-state carry-chain FIND of xc_kernel (ugrep_amd/csrc/xc_kernel.hip).

1. The byte classes tables.cpp derives from a table (ugpu_tables_xc_host: the
   LDS class table, and the SWAR range program of the UGPU_XC_SWAR build)
   reproduce the table's G (start -> A) and X (A -> A) byte sets exactly, the
   range program evaluated with the kernel's SWAR arithmetic on all 256 bytes.
2. The kernel's arithmetic -- one big addition S = X' + G' over the byte
   encoding X' = 0x7f | X << 7, G' = G << 7, carry-in bytes S ^ X' ^ G', starts
   G & !carry, the exit rule past hi -- restated here with Python integers over
   whole buffers, equals the oracle's FIND chain (counts, digests, exit) on
   seeded corpora and edge cases, from arbitrary [lo, hi).
"""
import numpy as np
import pytest

from oracle_lib import OracleDfa, gen

M = (1 << 64) - 1
TWO_STATE = ("c3_ident", "digits")


def _xc(opc):
    from ugrep_amd.matcher import host_xc
    return host_xc(opc)


def _sets(opc):
    """G and X of a two-state table from its dense form."""
    from ugrep_amd import host_tables
    t = host_tables(opc)
    row, fmt = t["info"]["row"], t["info"]["format"]
    cls = t["cls"]

    def nxt(s, b):
        return int(t["trans"][s + (b if fmt == 0 else cls[b])])
    st = t["start"]
    A = next(nxt(st, b) for b in range(256) if nxt(st, b))
    G = np.array([nxt(st, b) == A for b in range(256)])
    X = np.array([nxt(A, b) == A for b in range(256)])
    return G, X, row


def _swar(shape, k, x):
    """The kernel's class program (CProg) on uint32 words x: (G80, X')."""
    nf, ng, np_ = shape & 15, (shape >> 4) & 15, (shape >> 8) & 15
    x = x.astype(np.uint64)
    m32 = np.uint64(0xFFFFFFFF)
    x7 = x & np.uint64(0x7F7F7F7F)
    g = np.zeros_like(x)
    h = x7 | np.uint64(0x20202020)
    for i in range(nf):
        g |= ((h + np.uint64(k[2 * i])) & m32) & ~((h + np.uint64(k[2 * i + 1])) & m32)
    for i in range(ng):
        g |= ((x7 + np.uint64(k[4 + 2 * i])) & m32) & ~((x7 + np.uint64(k[5 + 2 * i])) & m32)
    G = g & ~x & np.uint64(0x80808080)
    p = np.zeros_like(x)
    for i in range(np_):
        p |= ((x7 + np.uint64(k[10 + 2 * i])) & m32) & ~((x7 + np.uint64(k[11 + 2 * i])) & m32)
    X = ((p & ~x) | G | np.uint64(0x7F7F7F7F)) & m32
    return G & m32, X


def _classify(shape, k, data):
    """Per byte (G, X) booleans through the SWAR program."""
    n = data.size
    pad = np.zeros((n + 3) // 4 * 4, np.uint8)
    pad[:n] = data
    G, X = _swar(shape, k, pad.view("<u4"))
    gb = np.frombuffer(G.astype("<u4").tobytes(), np.uint8)[:n] & 0x80
    xb = np.frombuffer(X.astype("<u4").tobytes(), np.uint8)[:n] & 0x80
    return gb != 0, xb != 0


@pytest.mark.parametrize("pname", TWO_STATE)
def test_two_state_tables_qualify(patterns, pname):
    assert _xc(patterns[pname]["opc"]) is not None


def test_range_program_reproduces_byte_sets(patterns):
    seen = 0
    for name, p in patterns.items():
        if p.get("unsupported"):
            continue
        try:
            xc = _xc(p["opc"])
        except Exception:
            continue
        if xc is None:
            continue
        seen += 1
        G, X, _ = _sets(p["opc"])
        cls, shape, k = xc
        assert np.array_equal((cls & 0x80) != 0, G), name  # the LDS class table
        assert np.array_equal((cls & 0x40) != 0, X), name
        if shape:
            g, x = _classify(shape, k, np.arange(256, dtype=np.uint8))
            assert np.array_equal(g, G), name
            assert np.array_equal(x, X), name
    assert seen >= 2


def test_range_program_on_synthetic_sets():
    """Random ASCII sets through tables.cpp's program builder via the compiler:
    every compiled two-state bracket pattern must classify exactly."""
    import ugrep_amd
    rng = np.random.default_rng(7)
    done = 0
    for _ in range(60):
        lo1, lo2 = sorted(rng.integers(0x21, 0x7F, 2))
        hi_extra = int(rng.integers(0x21, 0x7F))
        rx = "[\\x%02x-\\x%02x\\x%02x][\\x%02x-\\x%02x\\x%02x0-9]*" % (lo1, lo2, hi_extra, lo1, lo2, hi_extra)
        try:
            opc = ugrep_amd.compile_regex(rx)
        except Exception:
            continue
        xc = _xc(opc)
        if xc is None:
            continue
        G, X, _ = _sets(opc)
        assert np.array_equal((xc[0] & 0x80) != 0, G) and np.array_equal((xc[0] & 0x40) != 0, X), rx
        if not xc[1]:
            continue  # more ranges than the SWAR shapes hold: the LDS classes only
        g, x = _classify(xc[1], xc[2], np.arange(256, dtype=np.uint8))
        assert np.array_equal(g, G), rx
        assert np.array_equal(x, X), rx
        done += 1
    assert done >= 20


def xc_restated(shape, k, cap, data, lo, hi, rend, at_eof):
    """The kernel's chain arithmetic over the whole buffer as one integer.
    Returns (count, digest, dcap, exit, halo)."""
    g, x = _classify(shape, k, data[:rend])
    pos = np.arange(rend)
    g &= (pos >= lo) & (pos < hi)
    x &= pos >= lo
    xb = np.where(x, 0xFF, 0x7F).astype(np.uint8)
    gb = np.where(g, 0x80, 0x00).astype(np.uint8)
    Xi = int.from_bytes(xb.tobytes(), "little")
    Gi = int.from_bytes(gb.tobytes(), "little")
    S = Xi + Gi
    cbytes = np.frombuffer(((S ^ Xi ^ Gi) & ((1 << (8 * rend)) - 1)).to_bytes(rend, "little"), np.uint8)
    carry = np.zeros(rend + 1, bool)  # carry INTO position q (In_{q-1})
    carry[:rend] = cbytes != 0
    carry[rend] = (S >> (8 * rend)) & 1 == 1
    starts = np.nonzero(g & ~carry[:rend])[0]
    inb = carry[1:]  # In_q
    after = np.nonzero(~carry[hi + 1:rend + 1])[0]  # exit: the first q >= hi with In_q clear
    ex = min(hi + int(after[0]), rend) if after.size else rend
    halo = bool(carry[rend]) and not at_eof
    cnt = int(starts.size)
    sst = int(starts.sum()) if cnt else 0
    ln = int(inb[lo:ex].sum())
    return cnt, (31 * sst + ln) & M, (cap * (sst + cnt)) & M, ex, halo


def _oracle_range(opc, host, lo, hi):
    _, _, _, lst = OracleDfa(opc).find(host, start=lo, want_list=True)
    cnt = dg = dc = 0
    ex = hi
    for s, ln, cap in lst:
        if s >= hi:
            break
        cnt += 1
        dg = (dg + 31 * s + ln) & M
        dc = (dc + (s + 1) * cap) & M
        if s + ln > hi:
            ex = s + ln
    return cnt, dg, dc, ex


def _inputs():
    n = 96 << 10
    out = {"code": gen(3, 41, 0, n), "words": gen(1, 42, 0, n), "utf8": gen(4, 43, 0, n)}
    rng = np.random.default_rng(3)
    d = rng.integers(0, 256, n, dtype=np.uint8)
    d[rng.random(n) < 0.4] = ord("7")
    out["digits_noise"] = d
    out["all_ident"] = np.full(20000, ord("x"), np.uint8)
    out["digit_run"] = np.frombuffer(b"ab" + b"1" * 5000 + b" z9 " + b"9" * 3000, np.uint8).copy()
    return out


@pytest.mark.parametrize("pname", TWO_STATE)
def test_restated_arithmetic_equals_oracle(patterns, pname):
    opc = patterns[pname]["opc"]
    _, shape, k = _xc(opc)
    rng = np.random.default_rng(11)
    for name, host in _inputs().items():
        n = host.size
        ranges = [(0, n), (0, 1), (1, 2), (5, n - 3), (n - 1, n)]
        for _ in range(8):
            lo = int(rng.integers(0, n))
            ranges.append((lo, int(rng.integers(lo, n + 1))))
        for lo, hi in ranges:
            want = _oracle_range(opc, host, lo, hi)
            got = xc_restated(shape, k, 1, host, lo, hi, n, True)
            # the table's accept index: every two-state pattern here has cap 1
            assert got[:4] == want, (pname, name, lo, hi, got, want)
            assert not got[4]


def test_restated_halo_at_readable_end(patterns):
    opc = patterns["c3_ident"]["opc"]
    _, shape, k = _xc(opc)
    data = np.frombuffer(b"abc def ghij", np.uint8)
    # readable end inside "ghij", not EOF: the match may go on
    assert xc_restated(shape, k, 1, data, 0, 9, 10, False)[4]
    assert not xc_restated(shape, k, 1, data, 0, 9, 10, True)[4]
    # the match ending before the readable end's byte: no halo
    assert not xc_restated(shape, k, 1, data, 0, 5, 8, False)[4]
