"""CPU: the two-state carry-chain FIND of xc_kernel (ugrep_amd/csrc/xc_kernel.hip).

1. The byte classes tables.cpp derives from a table (ugpu_tables_xc_host)
   reproduce the table's G (start -> A) and X (A -> A) byte sets exactly.
2. The kernel's arithmetic -- one big addition S = e + 0x0101..01 over the
   byte codes e = 0xFF (G), 0xFE (P), 0x00 (K), carry-in bits bit 0 of
   S ^ e ^ 0x01, starts G & !carry, the exit rule past hi -- restated here with
   Python integers over whole buffers, equals the oracle's FIND chain (counts,
   digests, exit) on seeded corpora and edge cases, from arbitrary [lo, hi).
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


def _codes(cls, data):
    """The kernel's byte codes: 0xFF (G), 0xFE (P), 0x00 (K)."""
    c = cls[data]
    return np.where(c & 0x80, 0xFF, np.where(c & 0x40, 0xFE, 0)).astype(np.uint8)


@pytest.mark.parametrize("pname", TWO_STATE)
def test_two_state_tables_qualify(patterns, pname):
    assert _xc(patterns[pname]["opc"]) is not None


def test_byte_classes_reproduce_byte_sets(patterns):
    seen = 0
    for name, p in patterns.items():
        try:
            cls = _xc(p["opc"])
        except Exception:
            continue  # (unsupported tables)
        if cls is None:
            continue
        seen += 1
        G, X, _ = _sets(p["opc"])
        assert np.array_equal((cls & 0x80) != 0, G), name
        assert np.array_equal((cls & 0x40) != 0, X), name
    assert seen >= 2


def test_byte_classes_of_compiled_brackets():
    """Random byte-class patterns through the native compiler: every two-state
    table's classes equal its G/X sets."""
    import ugrep_amd
    rng = np.random.default_rng(7)
    done = 0
    for _ in range(60):
        lo1, lo2 = sorted(rng.integers(0x21, 0x7F, 2))
        extra = int(rng.integers(0x21, 0x7F))
        rx = "[\\x%02x-\\x%02x\\x%02x][\\x%02x-\\x%02x\\x%02x0-9]*" % (lo1, lo2, extra, lo1, lo2, extra)
        try:
            opc = ugrep_amd.compile_regex(rx)
        except Exception:
            continue
        cls = _xc(opc)
        if cls is None:
            continue
        G, X, _ = _sets(opc)
        assert np.array_equal((cls & 0x80) != 0, G) and np.array_equal((cls & 0x40) != 0, X), rx
        done += 1
    assert done >= 20


def xc_restated(cls, cap, data, lo, hi, rend, at_eof):
    """The kernel's chain arithmetic over the whole buffer as one integer:
    codes e (0xFF G, 0xFE P, 0x00 K; K outside [lo, rend), G -> P past hi),
    S = e + 0x0101..01, carry into byte i = bit 0 of (S ^ e ^ 0x01).
    Returns (count, digest, dcap, exit, halo)."""
    e = _codes(cls, data[:rend]).copy()
    pos = np.arange(rend)
    e[pos < lo] = 0
    e[(pos >= hi) & (e == 0xFF)] = 0xFE
    Ei = int.from_bytes(e.tobytes(), "little")
    Oi = int.from_bytes(b"\x01" * rend, "little")
    S = Ei + Oi
    x = np.frombuffer(((S ^ Ei ^ Oi) & ((1 << (8 * rend)) - 1)).to_bytes(rend, "little"), np.uint8)
    carry = np.zeros(rend + 1, bool)  # carry INTO position q (In_{q-1})
    carry[:rend] = (x & 1) != 0
    carry[rend] = (S >> (8 * rend)) & 1 == 1
    starts = np.nonzero((e & 1).astype(bool) & ~carry[:rend])[0]
    inb = carry[1:]  # In_q
    after = np.nonzero(~carry[hi + 1:rend + 1])[0]  # exit: the first q >= hi with In_q clear
    ex = min(hi + int(after[0]), rend) if after.size else rend
    halo = bool(carry[rend]) and not at_eof
    cnt = int(starts.size)
    sst = int(starts.sum()) if cnt else 0
    ln = int(inb[lo:ex].sum())
    return cnt, (31 * sst + ln) & M, (cap * (sst + cnt)) & M, ex, halo


def _oracle_range(opc, host, lo, hi):
    """(count, digest, dcap, exit) of the chain entering at lo, matches starting before hi."""
    from oracle_lib import range_totals
    return range_totals(opc, host, lo, hi)


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
    cls = _xc(opc)
    rng = np.random.default_rng(11)
    for name, host in _inputs().items():
        n = host.size
        ranges = [(0, n), (0, 1), (1, 2), (5, n - 3), (n - 1, n)]
        for _ in range(8):
            lo = int(rng.integers(0, n))
            ranges.append((lo, int(rng.integers(lo, n + 1))))
        for lo, hi in ranges:
            want = _oracle_range(opc, host, lo, hi)
            got = xc_restated(cls, 1, host, lo, hi, n, True)
            # the table's accept index: every two-state pattern here has cap 1
            assert got[:4] == want, (pname, name, lo, hi, got, want)
            assert not got[4]


def test_restated_halo_at_readable_end(patterns):
    cls = _xc(patterns["c3_ident"]["opc"])
    data = np.frombuffer(b"abc def ghij", np.uint8)
    # readable end inside "ghij", not EOF: the match may go on
    assert xc_restated(cls, 1, data, 0, 9, 10, False)[4]
    assert not xc_restated(cls, 1, data, 0, 9, 10, True)[4]
    # the match ending before the readable end's byte: no halo
    assert not xc_restated(cls, 1, data, 0, 5, 8, False)[4]
