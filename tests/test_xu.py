"""GPU: xc_kernel's U mode, the FIND of code-point run tables (\\w+ = BASELINE
C4, \\S+, [^ \\t]+, Unicode classes +; ugrep_amd/csrc/xc_kernel.hip, tables.hpp
xu_*), against the oracle restatement of the reference's FIND
(lib/matcher.cpp:42-750) on ranges [lo, hi) of the chain (counts, digests,
exit), grids that move the wave borders, unaligned buffers, OFFSETS records,
the hand-off of ranges with 4-byte code points, and the halo rule at a non-EOF
readable end.  tests/test_xu_host.py pins the same arithmetic on the CPU."""
import os

import numpy as np
import pytest

from test_xc import _scan  # noqa: F401  (with ptr_off)
from test_xi import U, _dev, _oracle_range  # noqa: F401  (fixtures and helpers)

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

RUNS = ("c4_word", "s_plus", "nonspace")  # (wide_class qualifies too, but is prefiltered: sparse_kernel)


@pytest.fixture(scope="module", autouse=True)
def _prefer_xu():
    """These tables also have a gap transducer (xg_kernel, the default for them);
    UGPU_XU=1 runs U mode."""
    os.environ["UGPU_XU"] = "1"
    yield
    os.environ.pop("UGPU_XU", None)


@pytest.fixture(scope="module")
def upats(U, patterns, _prefer_xu):  # noqa: F811
    return {k: U.Pattern(patterns[k]["opc"]) for k in RUNS}


def _inputs():
    from oracle_lib import gen
    n = 3 << 20
    out = {"utf8": gen(4, 51, 0, n), "code": gen(3, 52, 0, n), "words": gen(1, 53, 0, 1 << 20)}
    b = gen(4, 54, 0, n)
    for pos, ln in ((5000, 3000), (1 << 20, 70000), ((2 << 20) - 7, 1500)):
        b[pos:pos + ln] = np.frombuffer(("é" * (ln // 2) + "x" * (ln % 2)).encode(), np.uint8)[:ln]
    out["long_words"] = b
    out["all_word"] = np.frombuffer(("Ωx" * (1 << 19)).encode(), np.uint8)[:1 << 20].copy()
    c = np.frombuffer(("€ab₀ₐ" * 200000).encode(), np.uint8)[:1 << 20].copy()  # 3-byte chars, mixed blocks
    c[1023::1024] = ord(" ")
    out["euro_border"] = c
    rng = np.random.default_rng(9)
    # UTF-8 fragments without 4-byte sequences: cut-off, stray, overlong, surrogates
    frags = [b"\xc3\xa9", b"\xc3", b"\xa9", b"\xe2\x82\xac", b"\xe2\x82", b"\xe2\x82\x81", b"\xe2\x82\x90",
             b"\xce\xb1", b"\xcd\xbe", b"a", b"Z", b"_", b"7", b" ", b"\n", b"\x00", b"\xff", b"\xc0\x80",
             b"\xe4\xb8\xad", b"\xed\xa0\x80", b"\xd7\x90", b"\xe0\x80\x80"]
    idx = rng.integers(0, len(frags), 700000)
    out["fragments"] = np.frombuffer(b"".join(frags[i] for i in idx), np.uint8)[:1 << 20].copy()
    return out


@pytest.fixture(scope="module")
def uinputs():
    return _inputs()


@pytest.mark.parametrize("pname", RUNS)
def test_kernel_choice(U, upats, pname):  # noqa: F811
    assert upats[pname].info()["kernel"] == 6


@pytest.mark.parametrize("pname", RUNS)
def test_ranges_against_oracle(U, upats, patterns, uinputs, pname):  # noqa: F811
    rng = np.random.default_rng(sum(pname.encode()) + 1)
    opc = patterns[pname]["opc"]
    for name, host in uinputs.items():
        n = host.size
        t = _dev(host)
        ranges = [(0, n), (0, 1), (1, 2), (0, 4096), (4095, 8193), (1000, 4096 * 3 + 5), (n - 70000, n), (n, n)]
        for _ in range(3):
            lo = int(rng.integers(0, n))
            hi = int(rng.integers(lo, min(n, lo + int(rng.choice([100, 5000, 200000, 2 << 20]))) + 1))
            ranges.append((lo, hi))
        for lo, hi in ranges:
            got = _scan(U, upats[pname], t, lo, hi, n)
            assert got == _oracle_range(opc, host, lo, hi), (pname, name, lo, hi)


def test_grids_and_alignment(U, patterns, uinputs):  # noqa: F811
    """Grids of 1..many waves move every wave border (look-back, carried codes);
    unaligned buffers shift the 16-byte lanes against the bytes."""
    opc = patterns["c4_word"]["opc"]
    host = uinputs["utf8"]
    n = host.size
    t = _dev(host)
    want = _oracle_range(opc, host, 0, n)
    for g in ("1", "3", "17", "250"):
        os.environ["UGPU_MAX_GRID"] = g
        try:
            pat = U.Pattern(opc)
            assert _scan(U, pat, t, 0, n, n) == want, g
            assert _scan(U, pat, t, 777, n - 5, n) == _oracle_range(opc, host, 777, n - 5), g
        finally:
            os.environ.pop("UGPU_MAX_GRID", None)
    pat = U.Pattern(opc)
    for off in (1, 3, 7, 13):
        m = n - 16
        sub = host[off:off + m]
        assert _scan(U, pat, t, 0, m, m, ptr_off=off) == _oracle_range(opc, sub, 0, m), off


@pytest.mark.parametrize("pname", ("c4_word", "nonspace"))
def test_offsets_records(U, upats, patterns, uinputs, pname):  # noqa: F811
    from oracle_lib import OracleDfa
    opc = patterns[pname]["opc"]
    for name in ("utf8", "fragments", "euro_border"):
        host = uinputs[name]
        dev = _dev(host)[:host.size]
        res = U.find_all(upats[pname], dev, offsets=True)
        cnt, dg, dc, lst = OracleDfa(opc).find(host, want_list=True)
        assert (res.count, res.digest, res.dcap) == (cnt, dg, dc), (pname, name)
        assert res.triples() == lst, (pname, name)


def test_four_byte_tokens_hand_off(U, upats, patterns):  # noqa: F811
    """A 4-byte lead makes the range flag UGPU_FLAG_USLOW; the host then scans
    it with the next kernel: results still equal the oracle's."""
    from oracle_lib import OracleDfa, gen
    opc = patterns["c4_word"]["opc"]
    host = gen(4, 61, 0, 1 << 20)
    host[300000:300004] = np.frombuffer("𝐀".encode(), np.uint8)   # U+1D400, a Word letter
    host[700001:700005] = np.frombuffer("😀".encode(), np.uint8)   # not a Word character
    t = _dev(host)
    n = host.size
    for lo, hi in ((0, n), (299990, 300010), (500000, n)):
        assert _scan(U, upats["c4_word"], t, lo, hi, n) == _oracle_range(opc, host, lo, hi), (lo, hi)
    res = U.find_all(upats["c4_word"], t[:n], offsets=True)
    assert res.triples() == OracleDfa(opc).find(host, want_list=True)[3]


def test_halo_at_readable_end(U, upats, patterns):  # noqa: F811
    """A run reaching the last 3 bytes before a non-EOF readable end raises
    UGPU_HALO (their codes depend on bytes not read yet), unless it ends at an
    ASCII byte."""
    host = np.frombuffer("ab cd éé".encode() + b" " * 100, np.uint8).copy()
    t = _dev(host)
    sc = U.Scanner(upats["c4_word"])
    sc.scan(t.data_ptr(), 0, 7, 9, False, 0, torch.cuda.current_stream().cuda_stream)
    with pytest.raises(Exception):
        sc.totals()
    sc.scan(t.data_ptr(), 0, 7, 9, True, 0, torch.cuda.current_stream().cuda_stream)
    tot = sc.totals()
    assert tot.count == 3
    # an exit at an ASCII byte is decided: no halo ("cd" ends at the space 5)
    sc.scan(t.data_ptr(), 0, 4, 6, False, 0, torch.cuda.current_stream().cuda_stream)
    tot = sc.totals()
    assert (tot.count, tot.exit) == (2, 5)


def test_agrees_with_xg_at_scale(U, patterns):  # noqa: F811
    """256 MiB of the C4 corpus: U mode and xg_kernel (UGPU_XU=0) agree."""
    opc = patterns["c4_word"]["opc"]
    n = 256 << 20
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    U.gen(U.GEN_UTF8, 1, 0, buf.data_ptr(), n)
    torch.cuda.synchronize()
    a = U.find_all(U.Pattern(opc), buf[:n])
    os.environ["UGPU_XU"] = "0"
    try:
        pat = U.Pattern(opc)
        assert pat.info()["kernel"] == 3
        b = U.find_all(pat, buf[:n])
    finally:
        os.environ["UGPU_XU"] = "1"
    assert (a.count, a.digest, a.dcap) == (b.count, b.digest, b.dcap)
