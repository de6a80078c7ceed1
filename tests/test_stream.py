"""GPU: streaming FIND (ugpu_stream).  Feeding any chunking
of an input -- one byte at a time, ragged sizes, chunks that split matches,
matches longer than the carry margin -- yields exactly the FIND result of the
oracle restatement over the whole input (tests/oracle_lib.py, itself pinned to
the reference matcher by tests/test_oracle.py), record by record."""
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


def _stream(U, pat, data, sizes, keep, offsets=True):
    st = U.Stream(pat, keep=keep)
    trip, cnt, dg, dc, i = [], 0, 0, 0, 0
    k = 0
    while True:
        n = sizes[k % len(sizes)]
        k += 1
        chunk = data[i:i + n]
        i += len(chunk)
        final = i >= len(data)
        r = st.feed(chunk.tobytes(), final=final, offsets=offsets)
        if offsets:
            trip += r.triples()
        cnt += r.count
        dg = (dg + r.digest) % (1 << 64)
        dc = (dc + r.dcap) % (1 << 64)
        if final:
            break
    return trip, cnt, dg, dc


def _whole(U, pat, data):
    """The oracle's FIND over the whole input: (triples, count, digest, dcap)."""
    from oracle_lib import OracleDfa
    cnt, dg, dc, lst = OracleDfa(pat.opc).find(np.ascontiguousarray(data), want_list=True)
    return lst, cnt, dg, dc


@pytest.mark.parametrize("pname,kind", [("c2_foobarbaz", 1), ("c3_ident", 3), ("c4_word", 4)])
def test_stream_equals_whole_buffer(U, patterns, pname, kind):
    from oracle_lib import gen
    data = gen(kind, 11, 0, 3 << 20)
    pat = U.Pattern(patterns[pname]["opc"])
    want = _whole(U, pat, data)
    rng = np.random.default_rng(kind)
    for sizes, keep in (([1 << 20], 0), ([int(x) for x in rng.integers(1, 70000, 50)], 4096),
                        ([int(x) for x in rng.integers(1, 300, 50)] + [500000], 64)):
        got = _stream(U, pat, data, sizes, keep)
        assert got == want, (pname, keep)


def test_stream_small_chunks_and_long_matches(U, patterns):
    # 'aa' over a long run of a's: every match spans chunk ends, the open walk
    # is longer than the carry margin (retries), and one-byte chunks
    pat = U.Pattern(patterns["aa"]["opc"])
    data = np.frombuffer(b"b" + b"a" * 20001 + b"\nab aaab aab\n" + b"a" * 7, np.uint8)
    want = _whole(U, pat, data)
    for sizes, keep in (([1], 16), ([3, 1, 4, 1, 5, 9, 2, 6], 16), ([997], 64)):
        assert _stream(U, pat, data, sizes, keep) == want
    # identifier runs much longer than the margin
    pat = U.Pattern(patterns["c3_ident"]["opc"])
    data = np.frombuffer((b"x" * 100000 + b" 9a_b " + b"y" * 3000) * 3, np.uint8)
    want = _whole(U, pat, data)
    assert _stream(U, pat, data, [12345, 777], 256) == want


def test_stream_count_mode_and_settled(U, patterns):
    from oracle_lib import gen
    data = gen(3, 5, 0, 1 << 20)
    pat = U.Pattern(patterns["c3_ident"]["opc"])
    want = _whole(U, pat, data)
    got = _stream(U, pat, data, [65536], 0, offsets=False)
    assert got[1:] == want[1:]
    st = U.Stream(pat, keep=1024)
    st.feed(data[:200000].tobytes())
    assert 200000 - 1024 <= st.settled() <= 200000
    r = st.feed(b"", final=True)
    assert st.settled() == 200000
    with pytest.raises(U.UgpuError):
        st.feed(b"x")


def test_stream_forest_fallback(U, patterns):
    """Streams whose feeds fall to the forest FIND (a tiny stitch budget forces it;
    ragged last blocks, non-final feeds with walks open at the readable end) keep
    the oracle's whole-input result, record by record."""
    import os
    from oracle_lib import gen
    os.environ["UGPU_FIX_BUDGET"] = "1"
    os.environ["UGPU_MERGE_BUDGET"] = "1"
    try:
        for pname, kind in (("c3_ident", 3), ("c4_word", 4), ("aa", 1)):
            data = gen(kind, 13, 0, (1 << 20) + 777)
            pat = U.Pattern(patterns[pname]["opc"])
            want = _whole(U, pat, data)
            for sizes, keep in (([12345, 70001], 4096), ([300000], 64)):
                assert _stream(U, pat, data, sizes, keep) == want, (pname, keep)
    finally:
        os.environ.pop("UGPU_FIX_BUDGET", None)
        os.environ.pop("UGPU_MERGE_BUDGET", None)


def test_stream_flush_settles_decided_matches(U, patterns):
    """UGPU_FEED_FLUSH (an input that would block): every match the fed bytes
    decide comes back from that feed -- all of them when the bytes end at a
    separator -- and the concatenation over any chunking still equals the
    oracle's FIND over the whole input."""
    from oracle_lib import gen
    for pname, kind in (("c2_foobarbaz", 1), ("c4_word", 4)):
        data = gen(kind, 5, 0, 1 << 20)
        pat = U.Pattern(patterns[pname]["opc"])
        want = _whole(U, pat, data)
        rng = np.random.default_rng(kind)
        st = U.Stream(pat)
        trip, i = [], 0
        cuts = sorted(set(int(x) for x in rng.integers(1, data.size, 40)))
        for c in cuts + [data.size]:
            chunk = data[i:c]
            r = st.feed(chunk.tobytes(), final=c == data.size, flush=c < data.size)
            trip += r.triples()
            i = c
            if c < data.size:
                # every match that ends before the last separator of the bytes so
                # far is final after this feed
                sep = int(np.nonzero(np.isin(data[:c], np.frombuffer(b" \n", np.uint8)))[0][-1])
                assert [t for t in want[0] if t[0] + t[1] <= sep] == [t for t in trip if t[0] + t[1] <= sep], (pname, c)
        assert trip == want[0], pname


def test_stream_option_w(U):
    """Option W on streamed input: the carry keeps the 4 bytes before the
    settled position, so at_wb at a chunk start reads the true code point
    before it; chunk cuts inside code points and words, flushed and plain
    feeds -- the concatenation equals the oracle's option-W FIND."""
    from oracle_lib import OracleDfa
    from test_multi import W_PATTERNS, _w_corpus
    data = _w_corpus(1 << 20)
    rng = np.random.default_rng(5)
    for rx in W_PATTERNS:
        opc = U.compile_regex(rx)
        pat = U.Pattern(opc, word=True)
        want = OracleDfa(opc).find_w(data, want_list=True)
        for flush in (False, True):
            st = U.Stream(pat, keep=4096)
            trip, i = [], 0
            cuts = sorted(set(int(x) for x in rng.integers(1, data.size, 60)))
            for c in cuts + [data.size]:
                r = st.feed(data[i:c].tobytes(), final=c == data.size, flush=flush and c < data.size)
                trip += r.triples()
                i = c
            assert trip == want[3], (rx, flush)
