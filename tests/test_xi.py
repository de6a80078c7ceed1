"""GPU: xi_kernel, the FIND kernel of "immediate" restart-local tables
(identifiers, digit runs, '.'; ugrep_amd/csrc/xi_kernel.hip), against the
oracle restatement on ranges [lo, hi) of the chain (counts, digests and the
exit = first chain position >= hi).

Its lanes rely on sync bytes (bytes that kill every walk and start none), so
the cases include inputs where sync bytes are missing for more than a lane
segment (1 KiB), a wave tile (64 KiB) or the whole buffer, sync bytes exactly
on segment borders, ranges cut inside matches, and grids that move the wave
borders.  The dense kernel (UGPU_XI=0) must agree on 256 MiB."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

M = (1 << 64) - 1
IMMEDIATE = ("c3_ident", "digits", "dot")


@pytest.fixture(scope="module")
def U():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


@pytest.fixture(scope="module")
def pats(U, patterns):
    return {k: U.Pattern(patterns[k]["opc"]) for k in IMMEDIATE}


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


def _scan(U, pat, t, lo, hi, n):
    sc = U.Scanner(pat)
    sc.scan(t.data_ptr(), lo, hi, n, True, 0, _stream())
    tot = sc.totals()
    return tot.count, tot.digest, tot.dcap, tot.exit


def _inputs():
    from oracle_lib import gen
    n = 3 << 20
    out = {"code": gen(3, 21, 0, n), "words": gen(1, 22, 0, n), "utf8": gen(4, 23, 0, n)}
    rng = np.random.default_rng(1)
    # long identifiers: 3000 B (several lanes), 70000 B (more than a tile)
    b = gen(3, 24, 0, n)
    for pos, ln in ((5000, 3000), (1 << 20, 70000), ((2 << 20) - 7, 1500)):
        b[pos:pos + ln] = ord("a")
    out["long_words"] = b
    # no sync byte at all
    out["all_ident"] = np.full(1 << 20, ord("x"), np.uint8)
    # sync bytes exactly on lane segment borders, identifiers in between
    c = np.full(1 << 20, ord("k"), np.uint8)
    c[1023::1024] = ord(" ")
    c[1024::1024] = ord(" ")
    out["border_sync"] = c
    # only sync bytes
    out["all_space"] = np.full(1 << 20, ord(" "), np.uint8)
    # random bytes with many digits
    d = rng.integers(0, 256, n, dtype=np.uint8)
    d[rng.random(n) < 0.5] = ord("7")
    out["digits_noise"] = d
    return out


@pytest.fixture(scope="module")
def inputs():
    return _inputs()


@pytest.mark.parametrize("pname", IMMEDIATE)
def test_ranges_against_oracle(U, pats, patterns, inputs, pname):
    rng = np.random.default_rng(sum(pname.encode()))
    opc = patterns[pname]["opc"]
    for name, host in inputs.items():
        if pname == "dot":
            # (every byte a match: the lane walks are slow, 64 KiB of all_ident
            # is one lane's walk at about 1 MB/s)
            host = host[:64 << 10] if name == "all_ident" else host[:512 << 10]
        n = host.size
        t = _dev(host)
        ranges = [(0, n), (0, 1), (1, 2), (0, 65536), (65536, 131072), (1000, 65536 * 3 + 5), (n - 70000, n)]
        for _ in range(2 if pname == "dot" else 4):
            lo = int(rng.integers(0, n))
            hi = int(rng.integers(lo, min(n, lo + int(rng.choice([100, 5000, 200000, 2 << 20]))) + 1))
            ranges.append((lo, hi))
        for lo, hi in ranges:
            if not 0 <= lo <= hi <= n:
                continue  # (the fixed ranges of a shortened input)
            got = _scan(U, pats[pname], t, lo, hi, n)
            want = _oracle_range(opc, host, lo, hi)
            assert got == want, (pname, name, lo, hi, got, want)


def test_grid_moves_wave_borders(U, pats, patterns, inputs):
    """Every wave border is a chain stitch; several grids must agree with the oracle."""
    for name in ("code", "long_words", "border_sync", "all_ident"):
        host = inputs[name]
        t = _dev(host)
        want = _oracle_range(patterns["c3_ident"]["opc"], host, 0, host.size)
        for g in ("1", "2", "5", "37", ""):
            if g:
                os.environ["UGPU_MAX_GRID"] = g
            else:
                os.environ.pop("UGPU_MAX_GRID", None)
            try:
                got = _scan(U, pats["c3_ident"], t, 0, host.size, host.size)
            finally:
                os.environ.pop("UGPU_MAX_GRID", None)
            assert got == want, (name, g)


def test_offsets_after_xi_count(U, pats, patterns, inputs):
    """OFFSETS mode after an xi COUNT scan (records rebuilt on the dense kernel)."""
    from oracle_lib import OracleDfa
    host = inputs["long_words"]
    r = U.find_all(pats["c3_ident"], host.tobytes(), offsets=True)
    cnt, dg, dc, lst = OracleDfa(patterns["c3_ident"]["opc"]).find(host, want_list=True)
    assert (r.count, r.digest, r.dcap) == (cnt, dg, dc)
    assert r.triples() == lst


def test_agrees_with_dense_kernel_256mib(U, pats):
    n = 256 << 20
    t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    U.gen(3, 31, 0, t.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    res = []
    for xi in ("1", "0"):
        os.environ["UGPU_XI"] = xi
        try:
            res.append(_scan(U, pats["c3_ident"], t, 0, n, n))
            res.append(_scan(U, pats["c3_ident"], t, 12345, n - 777, n))
        finally:
            os.environ.pop("UGPU_XI", None)
    assert res[0] == res[2] and res[1] == res[3], res

def test_no_sync_byte_for_4mib(U, pats):
    """One identifier across 4 MiB: a single lane's tail covers it (64-bit tail
    sums, buffer resource moving with the tail).  Such stretches are walked by
    one lane at latency speed, about 1 MB/s: pathological for this kernel."""
    n = 4 << 20
    t = torch.full((n + 16,), ord("x"), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert _scan(U, pats["c3_ident"], t, 0, n, n) == (1, n, 1, n)
    assert _scan(U, pats["c3_ident"], t, 5, n - 3, n) == (1, 31 * 5 + n - 5, 6, n)
