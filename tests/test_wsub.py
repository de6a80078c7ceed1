"""Option W (ugrep -w) on xc_kernel for class-plus tables whose bytes are a
proper subset of the ASCII word bytes ([A-Za-z]+, [a-z]+, [a-z_]+): the
subset mode of xc_kernel.hip (CW, ScanParams::xc_w = 2).  The word bytes
outside X are coded 0x02 so that at_wb sees them; a run of X followed by such
a byte ("abc1": at_we fails, no match) makes the wave flag the range and the
host redoes it with wfind_kernel, as for bytes >= 0x80.

CPU: the plan puts these tables on xc_kernel under option W.
GPU: equal to the oracle's option-W FIND (pinned to the reference's W lists,
tests/test_word.py) on letter-only text (the fast path), on code with digits
and underscores next to letters (the fallback), on edge cases at every cut,
and through shards and streams."""
import numpy as np
import pytest

from oracle_lib import OracleDfa, gen

PATS = ["[A-Za-z]+", "[a-z]+", "[a-z_]+", "[A-Z]+"]
EDGE = (b"abc abc1 1abc a_b ab_ _ab x\nword. word, a1b2 c3 d 9 __ q_ _q ABC AbC aBc\n"
        b"end-of-line\tTab\x00nul z\n" * 3)


def test_plan_subset_mode():
    import ugrep_amd as U
    for rx in PATS:
        assert U.host_plan(rx, word=True)["kernel"] == 5, rx  # xc_kernel
    assert U.host_plan("[A-Za-z_][A-Za-z0-9_]*", word=True)["kernel"] == 5  # (X = the word bytes: mode 1)


@pytest.fixture(scope="module")
def U():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _dev(arr):
    import torch
    t = torch.zeros(arr.size + 64, dtype=torch.uint8, device="cuda")
    t[:arr.size].copy_(torch.from_numpy(np.ascontiguousarray(arr)))
    torch.cuda.synchronize()
    return t[:arr.size]


def _check(U, rx, data, offsets=True):
    opc = U.compile_regex(rx)
    o = OracleDfa(opc)
    pat = U.Pattern(opc, word=True)
    want = o.find_w(data, want_list=offsets)
    got = U.find_all(pat, _dev(data), offsets=offsets)
    assert (got.count, got.digest, got.dcap) == want[:3], rx
    if offsets:
        assert [list(t) for t in got.triples()] == want[3], rx
    return pat, want


@pytest.mark.gpu
def test_letters_fast_path(U):
    data = gen(1, 17, 0, 32 << 20)  # C2 corpus: letters, spaces, newlines
    for rx in PATS:
        _check(U, rx, data, offsets=(rx == "[A-Za-z]+"))


@pytest.mark.gpu
def test_code_with_digits_falls_back(U):
    data = gen(3, 18, 0, 4 << 20)  # C3 corpus: identifiers with digits and '_'
    for rx in PATS:
        _check(U, rx, data)


@pytest.mark.gpu
def test_edges_every_cut(U):
    e = np.frombuffer(EDGE, np.uint8)
    base = gen(1, 19, 0, 1 << 20)
    for rx in PATS:
        for off in (0, 1, 1023, 1024, 4095, 4096, 65535):
            d = base.copy()
            d[off:off + e.size] = e[:max(0, min(e.size, d.size - off))]
            _check(U, rx, d, offsets=off in (0, 4095))


@pytest.mark.gpu
def test_shards_and_streams(U):
    data = gen(1, 20, 0, 8 << 20)
    data[5 << 20:(5 << 20) + 6] = np.frombuffer(b" abc1 ", np.uint8)  # one run that must not match
    for rx in ("[A-Za-z]+", "[a-z]+"):
        pat, want = _check(U, rx, data)
        m = U.find_all_multi(pat, data, ndev=3, offsets=False)
        assert (m.count, m.digest, m.dcap) == want[:3], rx
        s = U.Stream(pat)
        rng = np.random.default_rng(4)
        pos, recs = 0, []
        while pos < data.size:
            k = int(rng.integers(1, 1 << 20))
            ch = data[pos:pos + k]
            pos += ch.size
            recs.extend(list(t) for t in s.feed(ch, final=pos >= data.size).triples())
        s.close()
        assert recs == want[3], rx
