"""GPU: wide tables -- DFAs whose dense table has more than 64 Ki entries
(states x class row), e.g. two Unicode classes in a row (\\w+ \\w+: ~800 states
x 128 classes).  tables.cpp stores them with u32 row offsets (FMT_WIDE) and
the exact-walk kernels (wfind_kernel, fix_kernel, chain_fix, the forest) read
them from global memory.  Record by record against the oracle restatement
(which has no size limit), plain, option W, option N with anchors, streams,
multi-device shards and the records path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

WIDE = [r"\w+ \w+", r"\p{L}+ \w+|\d+ \p{L}+", r"\w+\W+\w+", r"\w\w\w"]


@pytest.fixture(scope="module")
def U():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _corpus(n):
    from test_multi import _w_corpus
    return _w_corpus(n)


def test_wide_tables_are_wide(U):
    for rx in WIDE:
        info = U.Pattern(U.compile_regex(rx)).info()
        assert info["format"] == 2 and info["kernel"] == 4, (rx, info)


def test_wide_find_all_equals_oracle(U):
    from oracle_lib import OracleDfa
    data = _corpus(2 << 20)
    dev = torch.from_numpy(data).cuda()
    torch.cuda.synchronize()
    for rx in WIDE:
        opc = U.compile_regex(rx)
        o = OracleDfa(opc)
        want = o.find(data, want_list=True)
        r = U.find_all(U.Pattern(opc), dev, offsets=True)
        assert (r.count, r.digest, r.dcap) == want[:3], rx
        assert r.triples() == want[3], rx
        for start in (1, 99999):
            r = U.find_all(U.Pattern(opc), dev, start=start, offsets=False)
            assert (r.count, r.digest, r.dcap) == o.find(data, start=start)[:3], (rx, start)
        w = U.find_all(U.Pattern(opc, word=True), dev, offsets=True)
        assert w.triples() == o.find_w(data, want_list=True)[3], rx


def test_wide_anchors_streams_shards_records(U):
    from oracle_lib import OracleDfa
    data = _corpus(1 << 20)
    rng = np.random.default_rng(9)
    for rx, nul in ((r"^\w+ \w+", True), (r"\w+ \w+$", True), (r"\w+ \w+", False)):
        opc = U.compile_regex(rx)
        pat = U.Pattern(opc, empty=nul)
        want = OracleDfa(opc).find(data, want_list=True, nul=nul)
        st = U.Stream(pat, keep=4096)
        trip, i = [], 0
        for c in sorted(set(int(x) for x in rng.integers(1, data.size, 20))) + [data.size]:
            trip += st.feed(data[i:c].tobytes(), final=c == data.size).triples()
            i = c
        assert trip == want[3], (rx, "stream")
        r = U.find_all_multi(pat, data, ndev=5, offsets=True)
        assert r.triples() == want[3], (rx, "multi")
        rec = U.Records(pat, data)
        assert rec.triples() == want[3], (rx, "records")
