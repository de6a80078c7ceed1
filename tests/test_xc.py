"""GPU: xc_kernel, the carry-chain FIND of two-state tables (identifiers, digit
runs; ugrep_amd/csrc/xc_kernel.hip), against the oracle restatement on ranges
[lo, hi) of the chain (counts, digests and the exit = first chain position >= hi).

Its waves take their carry-in from a look-back over the chunk before them, so
the cases include long identifiers and digit runs across chunks, tiles and
waves, a run of digits longer than the look-back (the scan hands the range to
the forest FIND), ranges cut inside matches, readable ends before EOF (halo),
and grids that move the wave borders.  xi_kernel (UGPU_XC=0) must agree on
256 MiB."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

M = (1 << 64) - 1
TWO_STATE = ("c3_ident", "digits")


@pytest.fixture(scope="module")
def U():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


@pytest.fixture(scope="module")
def pats(U, patterns):
    return {k: U.Pattern(patterns[k]["opc"]) for k in TWO_STATE}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dev(arr):
    t = torch.zeros(arr.size + 64, dtype=torch.uint8, device="cuda")
    t[:arr.size].copy_(torch.from_numpy(np.ascontiguousarray(arr)))
    torch.cuda.synchronize()
    return t


def _oracle_range(opc, host, lo, hi):
    """(count, digest, dcap, exit) of the chain entering at lo, matches starting before hi."""
    from oracle_lib import range_totals
    return range_totals(opc, host, lo, hi)


def _scan(U, pat, t, lo, hi, n, eof=True, ptr_off=0):
    sc = U.Scanner(pat)
    sc.scan(t.data_ptr() + ptr_off, lo, hi, n, eof, 0, _stream())
    tot = sc.totals()
    return tot.count, tot.digest, tot.dcap, tot.exit


def _inputs():
    from oracle_lib import gen
    n = 3 << 20
    out = {"code": gen(3, 21, 0, n), "words": gen(1, 22, 0, n), "utf8": gen(4, 23, 0, n)}
    rng = np.random.default_rng(1)
    b = gen(3, 24, 0, n)
    for pos, ln in ((5000, 3000), (1 << 20, 70000), ((2 << 20) - 7, 1500)):
        b[pos:pos + ln] = ord("a")
    out["long_words"] = b
    out["all_ident"] = np.full(1 << 20, ord("x"), np.uint8)
    c = np.full(1 << 20, ord("k"), np.uint8)
    c[1023::1024] = ord(" ")
    c[1024::1024] = ord(" ")
    out["border_sync"] = c
    out["all_space"] = np.full(1 << 20, ord(" "), np.uint8)
    d = rng.integers(0, 256, n, dtype=np.uint8)
    d[rng.random(n) < 0.5] = ord("7")
    out["digits_noise"] = d
    # digit runs just under and over the 8 KiB look-back, after and before letters
    e = gen(3, 25, 0, 1 << 20)
    e[10000:10000 + 8000] = ord("5")
    e[9999] = ord("q")
    e[300000:300000 + 30000] = ord("5")
    e[299999] = ord("q")
    out["digit_runs"] = e
    return out


@pytest.fixture(scope="module")
def inputs():
    return _inputs()


def test_kernel_choice(pats):
    assert pats["c3_ident"].info()["kernel"] == 5
    # prefiltered: sparse_kernel, or with UGPU_SPARSE=0 (this module's
    # default, _no_sparse) the dense kernel (xc_kernel takes no prefiltered table)
    assert pats["digits"].info()["kernel"] == 1
    os.environ.pop("UGPU_SPARSE", None)
    assert pats["digits"].info()["kernel"] == 0


@pytest.fixture(autouse=True)
def _no_sparse():
    """[0-9]+ has a selective prefilter; these tests run it on xc_kernel."""
    os.environ["UGPU_SPARSE"] = "0"
    yield
    os.environ.pop("UGPU_SPARSE", None)


@pytest.mark.parametrize("pname", TWO_STATE)
def test_ranges_against_oracle(U, pats, patterns, inputs, pname):
    rng = np.random.default_rng(sum(pname.encode()))
    opc = patterns[pname]["opc"]
    for name, host in inputs.items():
        n = host.size
        t = _dev(host)
        ranges = [(0, n), (0, 1), (1, 2), (0, 4096), (4096, 8192), (1000, 4096 * 3 + 5), (n - 70000, n), (n, n)]
        for _ in range(4):
            lo = int(rng.integers(0, n))
            hi = int(rng.integers(lo, min(n, lo + int(rng.choice([100, 5000, 200000, 2 << 20]))) + 1))
            ranges.append((lo, hi))
        for lo, hi in ranges:
            got = _scan(U, pats[pname], t, lo, hi, n)
            want = _oracle_range(opc, host, lo, hi)
            assert got == want, (pname, name, lo, hi, got, want)


def test_unaligned_buffers(U, pats, patterns, inputs):
    host = inputs["code"][: 1 << 20]
    t = _dev(np.concatenate([np.zeros(16, np.uint8), host]))
    for off in (1, 5, 15):
        tt = torch.zeros(host.size + 64, dtype=torch.uint8, device="cuda")
        tt[off:off + host.size].copy_(torch.from_numpy(host))
        torch.cuda.synchronize()
        got = _scan(U, pats["c3_ident"], tt, 0, host.size, host.size, ptr_off=off)
        assert got == _oracle_range(patterns["c3_ident"]["opc"], host, 0, host.size), off
    del t


def test_grid_moves_wave_borders(U, pats, patterns, inputs):
    """Every wave border is a carry look-back; several grids must agree with the oracle."""
    for name in ("code", "long_words", "border_sync", "all_ident", "digit_runs"):
        host = inputs[name]
        t = _dev(host)
        want = _oracle_range(patterns["c3_ident"]["opc"], host, 0, host.size)
        for g in ("1", "2", "5", "37", "300", ""):
            if g:
                os.environ["UGPU_MAX_GRID"] = g
            else:
                os.environ.pop("UGPU_MAX_GRID", None)
            try:
                got = _scan(U, pats["c3_ident"], t, 0, host.size, host.size)
            finally:
                os.environ.pop("UGPU_MAX_GRID", None)
            assert got == want, (name, g)


def test_long_digit_run_goes_to_forest(U, pats, patterns):
    """A digit run longer than the look-back leaves a wave's carry unknown for
    identifiers: the scan flags it and the forest FIND resolves the range."""
    host = np.full(1 << 20, ord(" "), np.uint8)
    host[4000] = ord("z")
    host[4001:4001 + 40000] = ord("3")
    t = _dev(host)
    sc = U.Scanner(pats["c3_ident"])
    sc.scan(t.data_ptr(), 0, host.size, host.size, True, 0, _stream())
    tot = sc.totals()
    assert tot.flags & 8  # UGPU_TOT_FOREST
    assert (tot.count, tot.digest, tot.dcap, tot.exit) == _oracle_range(patterns["c3_ident"]["opc"], host, 0,
                                                                        host.size)


def test_halo_at_readable_end(U, pats):
    host = np.frombuffer(b"abc def ghij   " * 4, np.uint8).copy()
    t = _dev(host)
    with pytest.raises(U.UgpuError) as e:
        _scan(U, pats["c3_ident"], t, 0, 9, 10, eof=False)
    assert e.value.code == 5
    assert _scan(U, pats["c3_ident"], t, 0, 9, 10, eof=True) == (3, (31 * (0 + 4 + 8) + 3 + 3 + 2) & M, 1 + 5 + 9, 10)
    assert _scan(U, pats["c3_ident"], t, 0, 5, 8, eof=False)[3] == 7


def test_no_separator_for_4mib(U, pats):
    """One identifier across 4 MiB (a single carry chain through every lane)."""
    n = 4 << 20
    t = torch.full((n + 16,), ord("x"), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert _scan(U, pats["c3_ident"], t, 0, n, n) == (1, n, 1, n)
    assert _scan(U, pats["c3_ident"], t, 5, n - 3, n) == (1, 31 * 5 + n - 5, 6, n)


def test_offsets_after_xc_count(U, pats, patterns, inputs):
    """OFFSETS mode after an xc COUNT scan (records rebuilt on the dense kernel)."""
    from oracle_lib import OracleDfa
    host = inputs["long_words"]
    r = U.find_all(pats["c3_ident"], host.tobytes(), offsets=True)
    cnt, dg, dc, lst = OracleDfa(patterns["c3_ident"]["opc"]).find(host, want_list=True)
    assert (r.count, r.digest, r.dcap) == (cnt, dg, dc)
    assert r.triples() == lst


def test_agrees_with_xi_kernel_256mib(U, pats):
    n = 256 << 20
    t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    U.gen(3, 31, 0, t.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    res = []
    for xc in ("1", "0"):
        os.environ["UGPU_XC"] = xc
        try:
            for pn in TWO_STATE:
                res.append(_scan(U, pats[pn], t, 0, n, n))
                res.append(_scan(U, pats[pn], t, 12345, n - 777, n))
        finally:
            os.environ.pop("UGPU_XC", None)
    assert res[:4] == res[4:], res


def test_offsets_written_by_xc(U, pats, patterns, inputs):
    """OFFSETS from xc_kernel's own WRITE pass (starts at exact indices, ends
    paired by index, lengths by the subtraction pass): records of ranges
    [lo, hi) equal the oracle's, over several grids."""
    from oracle_lib import OracleDfa
    opc = patterns["c3_ident"]["opc"]
    st = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(5)
    for name in ("code", "long_words", "border_sync", "all_ident", "digits_noise"):
        host = inputs[name]
        n = host.size
        t = _dev(host)
        _, _, _, lst = OracleDfa(opc).find(host, want_list=True)
        for lo, hi, g in ((0, n, ""), (0, n, "5"), (int(rng.integers(0, n // 2)), n - 3, "37"), (1, 5000, "")):
            if g:
                os.environ["UGPU_MAX_GRID"] = g
            try:
                sc = U.Scanner(pats["c3_ident"])
            finally:
                os.environ.pop("UGPU_MAX_GRID", None)
            sc.scan(t.data_ptr(), lo, hi, n, True, 0, st)
            cnt = sc.totals().count
            s = torch.empty(cnt + 1, dtype=torch.int64, device="cuda")
            ln = torch.empty(cnt + 1, dtype=torch.int32, device="cuda")
            cp = torch.empty(cnt + 1, dtype=torch.int32, device="cuda")
            sc.offsets(s.data_ptr(), ln.data_ptr(), cp.data_ptr(), cnt, st)
            torch.cuda.synchronize()
            got = list(zip(s[:cnt].cpu().tolist(), ln[:cnt].cpu().tolist(), cp[:cnt].cpu().tolist()))
            want = [tuple(r) for r in OracleDfa(opc).find(host, start=lo, want_list=True)[3] if r[0] < hi]
            assert got == want, (name, lo, hi, g)
