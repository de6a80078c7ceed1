"""GPU: the host records path ugpu_find_records (include/ugpu.h) -- chunked
H2D on a copy thread, per-chunk scans from the true chain entry, records
packed to 6/8 B and copied back into pinned memory while the next chunk
scans.  Record by record it must equal ugpu_find_all (itself pinned to the
reference's match lists) and the oracle restatement: many chunks (1 MiB),
nonzero starts, matches across chunk borders, lengths >= 0xFFFF and several
accept indices (the escape lists), device buffers, option W and anchors."""
import os

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


@pytest.fixture()
def small_chunks():
    os.environ["UGPU_REC_CHUNK"] = str(1 << 20)
    yield
    os.environ.pop("UGPU_REC_CHUNK", None)


def _check(U, pat, data, start=0, nul=False, word=False):
    from oracle_lib import OracleDfa
    o = OracleDfa(pat.opc)
    want = (o.find_w(data, start=start, want_list=True) if word else
            o.find(data, start=start, want_list=True, nul=nul))
    r = U.Records(pat, data, start=start)
    assert r.totals() == tuple(want[:3])
    assert r.triples() == want[3]
    r2 = U.Records(pat, data, start=start)
    assert r2.drain() == tuple(want[:3])
    # a borrowed buffer (UGPU_REC_BORROW): records popped while the input is
    # still crossing; a few records by next(), then the parallel drain
    r3 = U.Records(pat, data, start=start, borrow=True)
    assert r3.triples() == want[3]
    r4 = U.Records(pat, data, start=start, borrow=True)
    head = [r4.next() for _ in range(min(3, len(want[3])))]
    assert [list(t) for t in head] == want[3][:len(head)]
    k, dg, dc = r4.drain()
    m64 = (1 << 64) - 1
    hk, hdg, hdc = len(head), sum(s * 31 + ln for s, ln, _ in head), sum((s + 1) * c for s, _, c in head)
    assert (k + hk, (dg + hdg) & m64, (dc + hdc) & m64) == tuple(want[:3])


@pytest.mark.parametrize("rx,kind", [("foo|bar|baz", 1), ("[A-Za-z_][A-Za-z0-9_]*", 3), (r"\w+", 4)])
def test_records_equal_oracle(U, small_chunks, rx, kind):
    from oracle_lib import gen
    pat = U.Pattern(U.compile_regex(rx))
    data = gen(kind, 3, 0, (5 << 20) + 12345)
    for start in (0, 1, 777777):
        _check(U, pat, data, start)
    # a device buffer: no input copy
    dev = torch.from_numpy(data).cuda()
    torch.cuda.synchronize()
    r = U.Records(pat, dev)
    f = U.find_all(pat, dev, offsets=False)
    assert r.drain() == (f.count, f.digest, f.dcap)


def test_records_drain_one_thread(U, small_chunks, monkeypatch):
    """ugpu_records_drain with UGPU_REC_DRAIN_THREADS=1 (pieces decoded in
    order on the calling thread) and with 3 (in flight at once)."""
    from oracle_lib import gen
    pat = U.Pattern(U.compile_regex(r"\w+"))
    data = gen(4, 9, 0, (6 << 20) + 77)
    f = U.find_all(pat, data, offsets=False)
    for t in ("1", "3"):
        monkeypatch.setenv("UGPU_REC_DRAIN_THREADS", t)
        assert U.Records(pat, data).drain() == (f.count, f.digest, f.dcap)
        assert U.Records(pat, data, borrow=True).drain() == (f.count, f.digest, f.dcap)


def test_records_escapes_and_borders(U, small_chunks):
    """Matches longer than 0xFFFF bytes, across chunk borders, and accept
    indices of several alternatives."""
    from oracle_lib import gen
    data = gen(1, 4, 0, 3 << 20).copy()
    data[1000:1000 + 200000] = ord("a")            # one 200 000-byte match of a+
    data[(1 << 20) - 5:(1 << 20) + 70000] = ord("a")  # across the first chunk border
    data[(2 << 20) - 2:(2 << 20) + 2] = np.frombuffer(b"abab", np.uint8)
    for rx in ("a+|foo|bar", "(ab)+|a+|o"):
        _check(U, U.Pattern(U.compile_regex(rx)), data)


@pytest.mark.parametrize("dense", ["0", "1"])
def test_records_dense_pieces(U, small_chunks, monkeypatch, dense):
    """2-byte pieces (u8 gap + u8 len; chunks of one accept index with a record
    per < 32 bytes, the default) against the 6-byte form: gaps and lengths of
    255 bytes and more (escapes), a 70 000-byte match across a chunk border."""
    monkeypatch.setenv("UGPU_REC_DENSE", dense)
    rng = np.random.default_rng(8)
    data = np.where(rng.random(3 << 20) < 0.4, ord("a"), ord("-")).astype(np.uint8)
    for off, ln, ch in ((5000, 254, "-"), (9000, 255, "-"), (12000, 300, "-"), (20000, 254, "a"), (30000, 255, "a"),
                        (40000, 1000, "a"), ((1 << 20) - 30000, 70000, "a"), ((2 << 20) + 5, 256, "-")):
        data[off:off + ln] = ord(ch)
    _check(U, U.Pattern(U.compile_regex("a+")), data)
    _check(U, U.Pattern(U.compile_regex("a+")), data, start=12345)


def test_records_word_and_anchors(U, small_chunks):
    from test_multi import _w_corpus
    data = _w_corpus(3 << 20)
    _check(U, U.Pattern(U.compile_regex(r"\w+"), word=True), data, word=True)
    _check(U, U.Pattern(U.compile_regex(r"de|dei|é"), word=True), data, start=5, word=True)
    _check(U, U.Pattern(U.compile_regex(r"^\w+"), empty=True), data, nul=True)
    _check(U, U.Pattern(U.compile_regex(r"^(?:[^\n]*)$"), empty=True), data, nul=True)


@pytest.mark.gpu
def test_records_early_free_and_bounded_pieces(U, patterns, monkeypatch):
    """An early stop (ugrep -m1 / -l / -q): free() after a few pops cancels the
    pipeline instead of scanning and pinning the rest (the pipeline runs at
    most UGPU_REC_AHEAD pieces ahead of the consumer); totals() before any pop
    lifts that limit instead of waiting for pops (no deadlock); a later
    Records on the same table is exact."""
    import time
    from oracle_lib import OracleDfa, gen
    monkeypatch.setenv("UGPU_REC_CHUNK", str(1 << 20))
    monkeypatch.setenv("UGPU_REC_AHEAD", "2")
    opc = patterns["c3_ident"]["opc"]
    pat = U.Pattern(opc)
    host = gen(3, 9, 0, 64 << 20)
    r = U.Records(pat, host)
    first = [r.next() for _ in range(10)]
    t0 = time.perf_counter()
    r.close()
    assert time.perf_counter() - t0 < 5.0
    want = OracleDfa(opc).find(host[:1 << 20], want_list=True)[3][:10]
    assert [list(x) for x in first] == [list(x) for x in want]
    r2 = U.Records(pat, host)
    assert r2.totals() == tuple(OracleDfa(opc).find(host)[:3])
    r2.close()


def test_records_free_stops_the_upload(U):
    """free() on a BORROWED 4 GiB host buffer after the first pop
    stops the input copy too (the uploader checks the cancel flag between
    chunks) instead of copying the whole buffer to the device first.  The
    whole copy alone takes longer than the bound (4 GiB of pageable H2D)."""
    import time
    host = np.frombuffer(b"abc de_f9 12+3 " * 16, np.uint8)
    host = np.tile(host, (4 << 30) // host.size + 1)[:4 << 30]
    pat = U.Pattern(U.compile_regex("[A-Za-z_][A-Za-z0-9_]*"))
    r = U.Records(pat, host, borrow=True)
    assert r.next() == (0, 3, 1)
    t0 = time.perf_counter()
    r.close()
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    d = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    copy = time.perf_counter() - t1
    del d
    print("free %.3f s, whole H2D %.3f s" % (dt, copy))
    assert dt < 0.5 * copy
