"""GPU: line-level consumers (ugpu_lines): newline count,
the 1-based line of every match start, and the number of lines holding a
match (ugrep -c).  Pinned to the reference's own goldens (line numbers of
tests/out/Hello_*-ounkbT.out, the count of tests/out/Hello_Hello-c.out) and
to numpy on seeded corpora and edge cases (newlines on tile borders, '\\n'
next to 0x0b / 0x09 bytes, empty and newline-only buffers)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def U():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _run(U, data, starts):
    import torch
    n = len(data)
    buf = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    if n:
        buf[:n].copy_(torch.from_numpy(np.ascontiguousarray(data)))
    st = torch.from_numpy(np.asarray(starts, dtype=np.int64)).to("cuda")
    ln = torch.zeros(max(len(starts), 1), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    nl, ml = U.lines(buf.data_ptr(), n, st.data_ptr(), len(starts), ln.data_ptr())
    torch.cuda.synchronize()
    return nl, ml, ln[:len(starts)].cpu().numpy().astype(np.uint64)


def _np(data, starts):
    nlpos = np.flatnonzero(data == 10)
    lines = 1 + np.searchsorted(nlpos, np.asarray(starts, dtype=np.int64), side="left")
    return len(nlpos), len(np.unique(lines)), lines.astype(np.uint64)


def test_reference_goldens(U, patterns, refgold):
    import os
    data = np.frombuffer(open(os.path.join(os.path.dirname(__file__), "golden", "Hello.java"), "rb").read(),
                         np.uint8)
    for key in ("hello", "hello_wnhS"):
        g = refgold[key]
        r = U.find_all(U.Pattern(patterns[key]["opc"]), data.tobytes(), offsets=True)
        assert r.start.tolist() == g["starts"], key
        nl, ml, ln = _run(U, data, g["starts"])
        assert ln.tolist() == g["lines"], key
    nl, ml, ln = _run(U, data, refgold["hello"]["starts"])
    assert ml == refgold["hello"]["c_count"]  # ugrep -c Hello Hello.java
    assert nl == int(np.count_nonzero(data == 10))


MODES = ["0", "1", "2"]  # UGPU_LINES_MODE: auto, dense assign pass, sparse (quarter) assign pass


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("pname,kind", [("c2_foobarbaz", 1), ("c3_ident", 3), ("c4_word", 4)])
def test_corpus_lines(U, patterns, pname, kind, mode, monkeypatch):
    monkeypatch.setenv("UGPU_LINES_MODE", mode)
    from oracle_lib import gen
    data = gen(kind, 21, 0, 16 << 20)
    r = U.find_all(U.Pattern(patterns[pname]["opc"]), data.tobytes(), offsets=True)
    starts = r.start.astype(np.int64)
    got = _run(U, data, starts)
    want = _np(data, starts)
    assert got[0] == want[0] and got[1] == want[1]
    assert np.array_equal(got[2], want[2])


@pytest.mark.parametrize("mode", MODES)
def test_edge_buffers(U, mode, monkeypatch):
    monkeypatch.setenv("UGPU_LINES_MODE", mode)
    rng = np.random.default_rng(3)
    cases = []
    # newlines on and around 4 KiB tile and 16-byte granule borders, next to 0x0b/0x09
    d = np.full(3 * 4096 + 77, ord("a"), np.uint8)
    for p in (0, 15, 16, 17, 4095, 4096, 4097, 8191, 8192, 3 * 4096 + 76):
        d[p] = 10
    d[[1, 18, 4098]] = 0x0b
    d[[14, 4094]] = 0x09
    cases.append(d)
    cases.append(np.full(10000, 10, np.uint8))                     # only newlines
    cases.append(np.frombuffer(b"no newline at all" * 500, np.uint8))
    cases.append((rng.integers(0, 4, 1 << 20) * 3 + 7).astype(np.uint8))  # 7, 10, 13, 16: 1/4 newlines
    for d in cases:
        for nst in (1, 7, 5000):  # sparse to dense match lists
            starts = np.sort(rng.choice(len(d), size=min(len(d), nst), replace=False))
            got = _run(U, d, starts)
            want = _np(d, starts)
            assert got[0] == want[0] and got[1] == want[1] and np.array_equal(got[2], want[2])
        starts = np.sort(rng.choice(len(d), size=min(len(d), 5000), replace=False))
        got = _run(U, d, starts)
        want = _np(d, starts)
        assert got[0] == want[0] and got[1] == want[1] and np.array_equal(got[2], want[2])
    got = _run(U, np.zeros(0, np.uint8), [])
    assert got[:2] == (0, 0)
    # newline count without matches
    d = cases[3]
    assert _run(U, d, [])[0] == int(np.count_nonzero(d == 10))


@pytest.mark.parametrize("mode", MODES)
def test_many_waves_clusters(U, mode, monkeypatch):
    """64 MiB (thousands of wave ranges): match clusters of > 64 starts inside
    one quarter and one tile, runs of empty ranges, starts on range borders."""
    monkeypatch.setenv("UGPU_LINES_MODE", mode)
    rng = np.random.default_rng(11)
    n = (64 << 20) + 123
    d = np.where(rng.random(n) < 0.02, 10, 97).astype(np.uint8)
    parts = [np.arange(5000, 5300), np.arange(1 << 20, (1 << 20) + 4096, 3),
             rng.choice(n, 2000, replace=False), np.array([0, 4095, 4096, n - 1])]
    starts = np.unique(np.concatenate(parts)).astype(np.int64)
    got = _run(U, d, starts)
    want = _np(d, starts)
    assert got[0] == want[0] and got[1] == want[1] and np.array_equal(got[2], want[2])
