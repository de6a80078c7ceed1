"""CPU: the code-point run FIND of xc_kernel's U mode (ugrep_amd/csrc/xc_kernel.hip).

For a table whose language is S+ (S = single-code-point tokens, tables.hpp
xu_*), the FIND matches are the maximal runs of bytes lying inside a token.
The kernel codes every byte x (next bytes y, z) from the host tables
(ugpu_tables_xu_host): a thermometer of the token starting at x, resolved by
the third byte for 3-byte tokens; M_i = OR_k bit k of code_{i-k}; a run starts
at M_i & !M_{i-1}; past hi a run only continues.  This file restates that
arithmetic with numpy over whole buffers and pins it to the oracle's FIND chain
(lib/matcher.cpp:42-750 restated in oracle/restate.c) on seeded corpora, random
bytes (invalid UTF-8), cut-off sequences and arbitrary [lo, hi).
"""
import numpy as np
import pytest

from oracle_lib import OracleDfa, gen

M = (1 << 64) - 1
# patterns (native compiler, ugrep's default ERE in Unicode mode) expected to qualify
XU_RX = ["\\w+", "\\S+", "[[:alpha:]]+", "\\p{L}+", "[a-z\\x{e9}\\x{20ac}]+", "\\p{Greek}+", "[^ \\n]+",
         "[\\x{10000}-\\x{10fff}a-c]+"]


def _xu(opc):
    from ugrep_amd.matcher import host_xu
    return host_xu(opc)


KXU_CLS = 256 + 64 * 256  # tables.hpp kXuCls


def xu_codes(tab, bm3, b):
    """Per-byte token codes of the padded stream b (the kernel's lookups and
    its 3-byte resolution: the classes of the byte after, else the bitmap)."""
    n = b.size - 3
    x, y, z = b[:n + 1].astype(np.int64), b[1:n + 2].astype(np.int64), b[2:n + 3].astype(np.int64)
    code = np.where(x < 0x80, tab[np.minimum(x, 127)],
                    np.where(x < 0xC0, tab[KXU_CLS + y], tab[256 + (x & 63) * 256 + y])).astype(np.int64)
    cy = np.concatenate([code[1:], [0]])
    l3 = (code & 0x80) != 0
    ok = l3 & ((code & cy & 0x70) != 0)
    idx = ((x & 15) << 12) | ((y & 63) << 6) | (z & 63)
    bit = (bm3[idx >> 5].astype(np.int64) >> (idx & 31)) & 1
    mix = l3 & ((code & 0x70) == 0) & (bit == 1) & ((z & 0xC0) == 0x80)
    code = np.where(ok | mix, code | 7, code)
    return code[:n]


def xu_restated(tab, bm3, cap, data, lo, hi, rend, at_eof):
    """Returns (count, digest, dcap, exit, halo, slow)."""
    null = int(tab[129])
    b = np.full(rend + 3, null, np.uint8)
    b[lo:rend] = data[lo:rend]
    code = xu_codes(tab, bm3, b)
    slow = bool((code[lo:rend] & 0x08).any())  # (XU_SLOW = 0x0F: only 4-byte leads have bit 3)
    m = np.zeros(rend, bool)
    for k in range(4):
        m[k:] |= ((code[:rend - k] >> k) & 1) != 0
    prev = np.concatenate([[False], m[:-1]])
    pos = np.arange(rend)
    starts = np.nonzero(m & ~prev & (pos >= lo) & (pos < hi))[0]
    if hi > 0 and hi - 1 >= lo and m[hi - 1]:
        after = np.nonzero(~m[hi:])[0]
        ex = hi + int(after[0]) if after.size else rend
    else:
        ex = hi
    ex = min(ex, rend)
    halo = (not at_eof) and ex + 3 >= rend
    ln = int(m[lo:ex].sum())
    cnt = int(starts.size)
    sst = int(starts.sum()) if cnt else 0
    return cnt, (31 * sst + ln) & M, (cap * (sst + cnt)) & M, ex, halo, slow


def _oracle_range(opc, host, lo, hi):
    """(count, digest, dcap, exit) of the chain entering at lo, matches starting before hi."""
    from oracle_lib import range_totals
    return range_totals(opc, host, lo, hi)


def _inputs():
    n = 48 << 10
    rng = np.random.default_rng(5)
    out = {"utf8": gen(4, 43, 0, n), "words": gen(1, 42, 0, 8192)}
    out["random"] = rng.integers(0, 256, 8192, dtype=np.uint8)
    # UTF-8 fragments: cut-off, extra and stray continuation bytes, 4-byte code points
    frags = [b"\xc3\xa9", b"\xc3", b"\xa9", b"\xe2\x82\xac", b"\xe2\x82", b"\xe2\x82\x81", b"\xe2\x82\x90",
             b"\xce\xb1", b"\xcd\xbe", b"\xf0\x90\x80\x80", b"\xf0\x90\x80", b"\xf0\x9f\x98\x80", b"a", b"Z", b"_",
             b"7", b" ", b"\n", b"\x00", b"\xff", b"\xc0\x80", b"\xe4\xb8\xad", b"\xed\xa0\x80", b"\xd7\x90"]
    out["fragments"] = np.frombuffer(b"".join(frags[i] for i in rng.integers(0, len(frags), 3000)), np.uint8).copy()
    f3 = [f for f in frags if not f.startswith(b"\xf0")]  # (no 4-byte tokens: never handed off)
    out["fragments3"] = np.frombuffer(b"".join(f3[i] for i in rng.integers(0, len(f3), 3000)), np.uint8).copy()
    return out


def _qualifying():
    import ugrep_amd
    out = []
    for rx in XU_RX:
        opc = ugrep_amd.compile_regex(rx)
        t = _xu(opc)
        assert t is not None, rx
        out.append((rx, opc, t))
    return out


def test_word_plus_qualifies(patterns):
    """The reference's own \\w+ table (C4) qualifies; two-state and literal tables do not."""
    assert _xu(patterns["c4_word"]["opc"]) is not None
    assert _xu(patterns["c2_foobarbaz"]["opc"]) is None
    assert _xu(patterns["c3_ident"]["opc"]) is None   # (two-state: xc proper)


def test_non_token_languages_rejected():
    import ugrep_amd
    for rx in ["\\w+x", "ab+", "\\w\\w+", "[a-z]+[0-9]", "(\\w\\s)+", "\\w*"]:
        try:
            opc = ugrep_amd.compile_regex(rx)
            t = _xu(opc)
        except Exception:
            continue  # (tables the engine does not take at all)
        assert t is None, rx


@pytest.mark.parametrize("which", ["reference_c4", "compiled"])
def test_restated_runs_equal_oracle(patterns, which):
    if which == "reference_c4":
        opc = patterns["c4_word"]["opc"]
        cases = [("c4_word", opc, _xu(opc))]
    else:
        cases = _qualifying()
    rng = np.random.default_rng(13)
    checked = 0
    for rx, opc, (tab, bm3) in cases:
        for name, host in _inputs().items():
            n = host.size
            ranges = [(0, n), (0, 1), (1, 2), (5, n - 3), (n - 1, n), (n, n)]
            for _ in range(4):
                lo = int(rng.integers(0, n))
                ranges.append((lo, int(rng.integers(lo, n + 1))))
            for lo, hi in ranges:
                want = _oracle_range(opc, host, lo, hi)
                got = xu_restated(tab, bm3, 1, host, lo, hi, n, True)
                if got[5]:
                    continue  # 4-byte token: the kernel hands the range to another kernel
                assert got[:4] == want, (rx, name, lo, hi, got, want)
                checked += name in ("utf8", "fragments3")
    assert checked >= 10 * len(cases)


def test_restated_halo_rule(patterns):
    tab, bm3 = _xu(patterns["c4_word"]["opc"])
    d = np.frombuffer("ab cd é".encode(), np.uint8)
    # a run reaching the readable end of a non-EOF shard may go on
    assert xu_restated(tab, bm3, 1, d, 0, 7, 8, False)[4]
    assert not xu_restated(tab, bm3, 1, d, 0, 7, 8, True)[4]
    assert not xu_restated(tab, bm3, 1, d, 0, 1, 8, False)[4]
