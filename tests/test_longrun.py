"""GPU: long walks in the prefiltered kernel (sparse_kernel).

A prefiltered pattern whose walk runs far -- `a+` over a run of `a`, `fo+`
over a run of `o`, `(ab)+` over `abab...`, `a[^\\n]*b` over a long line --
used to cost one dependent byte load per byte of the walk, in every lane and
every wave the run crossed (round 3: 4.7 s for 1 MiB of `a`).  Now a walk
that outgrows its 32-byte window is continued by the whole wave (coop_walk),
stops at its wave's range end (an open walk), and fix_kernel resolves open
walks from the next waves' records; waves a match covers are skipped in one
step.  Parity against the oracle (record by record where the lists are
small), the forest fallback when an open walk cannot be resolved, OFFSETS,
and wall-time bounds on the runs of the round-3 verdict (1, 16 and 64 MiB
runs of `a` in a 256 MiB buffer, >= 100 GB/s)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def U():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _filler(n, unit=b"xy "):
    return np.frombuffer(unit * (n // len(unit) + 1), np.uint8)[:n].copy()


def _check(U, rx, host, lists=True):
    from oracle_lib import OracleDfa
    opc = U.compile_regex(rx)
    pat = U.Pattern(opc)
    assert pat.info()["kernel"] == 0, "expected the prefiltered kernel for %r" % rx
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    want = OracleDfa(opc).find(host, want_list=lists)
    got = U.find_all(pat, dev, offsets=lists)
    assert (got.count, got.digest, got.dcap) == tuple(want[:3]), rx
    if lists:
        assert got.triples() == want[3], rx
    cnt = U.find_all(pat, dev, offsets=False)
    assert (cnt.count, cnt.digest, cnt.dcap) == tuple(want[:3]), rx
    return got


@pytest.mark.parametrize("run", [1 << 10, 40000, 1 << 20, 5 << 20])
def test_a_plus_runs(U, run):
    """`a+` over one run of `a` planted at an odd offset of 24 MiB of filler
    (the run crosses many wave ranges), and a second run at the end (EOF)."""
    n = 24 << 20
    host = _filler(n)
    at = (7 << 20) + 12345
    host[at:at + run] = ord("a")
    host[n - 1000:] = ord("a")
    _check(U, "a+", host)


@pytest.mark.parametrize("rx,fill,run", [
    ("fo+", b"o", 3 << 20),            # one candidate, its walk crosses ~250 waves
    ("(ab)+", b"ab", 2 << 20),         # two-state cycle: the coop_walk guesses from 4 bytes
    ("a[^\n]*b", b"ab xyz ", 3 << 20),  # a long line with accepts all along
    ("x[a-z]*y", b"qrs", 1 << 20),     # a walk through a region without candidates
])
def test_long_walk_patterns(U, rx, fill, run):
    n = 16 << 20
    host = _filler(n, b"12 \n")
    at = (5 << 20) + 777
    seg = np.frombuffer(fill * (run // len(fill) + 1), np.uint8)[:run]
    head = {"fo+": b"f", "x[a-z]*y": b"x"}.get(rx, b"")
    tail = {"x[a-z]*y": b"y"}.get(rx, b"")
    blob = np.concatenate([np.frombuffer(head, np.uint8), seg, np.frombuffer(tail, np.uint8)])
    host[at:at + blob.size] = blob
    _check(U, rx, host)


def test_open_walk_ends_early(U):
    """`a[^\\n]*b` over long lines whose last `b` comes early: walks alive at
    a wave's range end whose last accept lies before it (fix_kernel re-walks
    the rest of the wave's chain from there), and lines without any `b`."""
    rng = np.random.default_rng(5)
    n = 8 << 20
    host = _filler(n, b"cd ")
    pos = 4096
    while pos < n - 200000:
        ln = int(rng.integers(20000, 150000))
        host[pos] = ord("a")
        if rng.integers(0, 3):
            host[pos + int(rng.integers(1, 200))] = ord("b")
        host[pos + ln] = ord("\n")
        pos += ln + int(rng.integers(1, 5000))
    _check(U, "a[^\n]*b", host)


def test_unresolved_open_walk_goes_to_the_forest(U):
    """An open walk that neither dies nor meets a later walk within the
    convergence budget (`x[a-z]*y` over 2 MiB of letters without candidates
    and without `y`): the scan falls back to the forest FIND, still exact."""
    n = 8 << 20
    host = _filler(n, b"12 ")
    host[1 << 20] = ord("x")
    host[(1 << 20) + 1:(3 << 20)] = ord("q")
    host[5 << 20] = ord("x")
    host[(5 << 20) + 1:(5 << 20) + 9] = ord("z")
    host[(5 << 20) + 9] = ord("y")
    _check(U, "x[a-z]*y", host)


def test_runs_across_shards_and_streams(U):
    """A long match across scanner ranges (nonzero starts, a readable end
    that is not EOF) and across stream chunks."""
    from oracle_lib import OracleDfa
    n = 12 << 20
    host = _filler(n)
    host[(3 << 20) + 5:(9 << 20) + 3] = ord("a")
    opc = U.compile_regex("a+")
    pat = U.Pattern(opc)
    o = OracleDfa(opc)
    dev = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    dev[:n].copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    sc = U.Scanner(pat)
    for lo in (0, (3 << 20) + 100, 6 << 20):
        sc.scan(dev.data_ptr(), lo, n, n, True, 0, _stream())
        t = sc.totals()
        want = o.find(host, start=lo)
        assert (t.count, t.digest, t.dcap) == tuple(want[:3]), lo
    st = U.Stream(pat)
    recs = []
    for k in range(0, n, 1 << 20):
        r = st.feed(host[k:k + (1 << 20)], final=k + (1 << 20) >= n)
        recs += r.triples()
    assert recs == o.find(host, want_list=True)[3]


@pytest.mark.parametrize("run", [1 << 20, 16 << 20, 64 << 20])
def test_a_plus_run_rate(U, run):
    """The round-3 verdict's bar: `a+` over a run of 1, 16 and 64 MiB of `a`
    inside a 256 MiB buffer scans at >= 100 GB/s, COUNT and OFFSETS, with the
    oracle's results.  (Round 3: 4.7 s COUNT for a 1 MiB run.)"""
    from oracle_lib import OracleDfa
    n = 256 << 20
    host = _filler(n)
    at = (100 << 20) + 4321
    host[at:at + run] = ord("a")
    opc = U.compile_regex("a+")
    pat = U.Pattern(opc)
    want = OracleDfa(opc).find(host)
    dev = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    dev[:n].copy_(torch.from_numpy(host))
    cap = want[0] + 16
    st = torch.empty(cap, dtype=torch.int64, device="cuda")
    ln = torch.empty(cap, dtype=torch.int32, device="cuda")
    ac = torch.empty(cap, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    sc = U.Scanner(pat)
    best_c = best_o = 1e9
    for _ in range(4):
        t0 = time.perf_counter()
        sc.scan(dev.data_ptr(), 0, n, n, True, 0, _stream())
        t = sc.totals()
        t1 = time.perf_counter()
        sc.offsets(st.data_ptr(), ln.data_ptr(), ac.data_ptr(), cap, _stream())
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        best_c = min(best_c, t1 - t0)
        best_o = min(best_o, t2 - t0)
        assert (t.count, t.digest, t.dcap) == tuple(want[:3])
    k = want[0]
    dg = int((st[:k] * 31 + ln[:k].to(torch.int64)).sum().item()) & ((1 << 64) - 1)
    assert dg == want[1]
    print("run %d MiB: COUNT %.3f ms (%.0f GB/s), COUNT+OFFSETS %.3f ms (%.0f GB/s)"
          % (run >> 20, best_c * 1e3, n / best_c / 1e9, best_o * 1e3, n / best_o / 1e9))
    assert n / best_c >= 100e9, best_c
    assert n / best_o >= 100e9, best_o


@pytest.mark.parametrize("offsets", [False, True])
def test_multi_true_entry_walks_past_the_halo(U, offsets):
    """ugpu_find_all_multi: shard 1's speculative chain (from its cut) is short
    (`xa` at the cut), but its true entry -- after shard 0's `qx` match across
    the cut -- starts `ab+` over a 6 MiB run of `b` that walks past the 1 MiB
    halo: the stitch and the re-scan grow the halo instead of failing with
    UGPU_HALO (the round-3 advisor's case)."""
    from oracle_lib import OracleDfa
    n = 12 << 20
    host = _filler(n, b"12 ")
    cut = 4 << 20
    host[cut - 1] = ord("q")
    host[cut] = ord("x")
    host[cut + 1] = ord("a")
    host[cut + 2:cut + 2 + (6 << 20)] = ord("b")
    opc = U.compile_regex("xa|ab+|qx")
    pat = U.Pattern(opc)
    want = OracleDfa(opc).find(host, want_list=offsets)
    for data in (host, torch.from_numpy(host).to("cuda")):
        got = U.find_all_multi(pat, data, ndev=3, offsets=offsets)
        assert (got.count, got.digest, got.dcap) == tuple(want[:3])
        if offsets:
            assert got.triples() == want[3]
