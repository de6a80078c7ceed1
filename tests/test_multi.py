"""GPU: the native multi-device entry point ugpu_find_all_multi (include/ugpu.h)
-- one process drives the devices, [start, len) cut into ndev shards at
arbitrary byte offsets, shard k on device k mod the visible devices (on a
one-card box every shard is a virtual shard of the same card, with its own
stream, table copy lookup, input copy and scanner), chains resolved across the
cuts by ugpu_chain_fix, records copied from each shard's device into its
slice of the result.

Expected values: the REFERENCE matcher's count/digest/dcap over the same bytes
(tests/golden/streams.json c2_512m, c3_256m), and record by record the
single-device ugpu_find_all and the oracle restatement.  The reference has no
multi-device counterpart: what is pinned is that sharding
changes nothing."""
import json
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


@pytest.fixture(scope="module")
def streams():
    from oracle_lib import GOLDEN
    with open(os.path.join(GOLDEN, "streams.json")) as f:
        return json.load(f)


def test_multi_reference_digests(U, streams, patterns):
    """c2_512m / c3_256m from host memory at 2, 3, 8 and 13 shards (cuts inside
    words and matches), and from device memory at 8 shards, == the reference."""
    from oracle_lib import gen
    for key in ("c2_512m", "c3_256m"):
        g = streams[key]
        host = gen(g["kind"], g["seed"], 0, g["bytes"])
        pat = U.Pattern(patterns[g["pattern"]]["opc"])
        want = (g["count"], g["digest"], g["dcap"])
        for ndev in (2, 3, 8, 13):
            r = U.find_all_multi(pat, host, ndev=ndev, offsets=False)
            assert (r.count, r.digest, r.dcap) == want, (key, ndev)
        dev = torch.from_numpy(host).to("cuda")
        torch.cuda.synchronize()
        r = U.find_all_multi(pat, dev, ndev=8, offsets=False)
        assert (r.count, r.digest, r.dcap) == want, key
        del dev
        torch.cuda.empty_cache()


def test_multi_records_equal_single_device(U, patterns):
    """OFFSETS records of every config table at odd shard counts and a nonzero
    start == ugpu_find_all on one device, record by record."""
    from oracle_lib import gen
    for pname, kind in (("c2_foobarbaz", 1), ("c3_ident", 3), ("c4_word", 4), ("c1_lorem", 4)):
        host = gen(kind, 3, 0, 24 << 20)
        pat = U.Pattern(patterns[pname]["opc"])
        for start in (0, 777777):
            one = U.find_all(pat, host, start=start, offsets=True)
            for ndev in (2, 5, 16):
                r = U.find_all_multi(pat, host, ndev=ndev, start=start, offsets=True)
                assert (r.count, r.digest, r.dcap) == (one.count, one.digest, one.dcap), (pname, ndev, start)
                assert np.array_equal(r.start, one.start) and np.array_equal(r.length, one.length), (pname, ndev)
                assert np.array_equal(r.cap, one.cap), (pname, ndev)


def test_multi_long_matches_and_unsynchronised_chains(U):
    """A 3 MiB identifier across several cuts (longer than the 1 MiB halo: the
    shard is scanned again with the rest of the buffer readable), and 'aa' over
    a run of 'a' cut at odd and even offsets (chains that never meet: the
    forest FIND inside ugpu_chain_fix), == the oracle."""
    from oracle_lib import OracleDfa, gen
    code = gen(3, 5, 0, 12 << 20)
    code[(4 << 20) + 5:(7 << 20) + 5] = ord("x")
    opc = U.compile_regex("[A-Za-z_][A-Za-z0-9_]*")
    pat = U.Pattern(opc)
    cnt, dg, dc, lst = OracleDfa(opc).find(code, want_list=True)
    for ndev in (5,):
        r = U.find_all_multi(pat, code, ndev=ndev, offsets=True)
        assert (r.count, r.digest, r.dcap) == (cnt, dg, dc), ndev
        assert r.triples() == lst, ndev
    aas = np.full(3 << 20, ord("a"), np.uint8)
    opc = U.compile_regex("aa")
    pat = U.Pattern(opc)
    want = OracleDfa(opc).find(aas)[:3]
    for ndev in (2, 3):
        r = U.find_all_multi(pat, aas, ndev=ndev, offsets=False)
        assert (r.count, r.digest, r.dcap) == want, ndev


W_PATTERNS = [r"\w+", r"[A-Za-z_][A-Za-z0-9_]*", "foo|bar|baz", r"\p{L}+\d*", "de|dei|é"]


def _w_corpus(n):
    """Mixed ASCII / 2-, 3- and 4-byte UTF-8 words, so that shard cuts land
    inside code points and inside words."""
    from oracle_lib import gen
    data = gen(4, 8, 0, n).copy()
    rng = np.random.default_rng(11)
    pieces = ["é".encode(), "日本".encode(), "𝔘x".encode(), b"foo_bar", b" de ", b"dei\n"]
    for at in rng.integers(0, n - 16, n // 64):
        p = pieces[int(at) % len(pieces)]
        data[int(at):int(at) + len(p)] = np.frombuffer(p, np.uint8)
    return data


def test_multi_option_w_shards(U):
    """Option W across shard cuts: each shard's copy begins 4 bytes before it,
    so at_wb at the cut reads the true code point before it; the stitch walks
    with the W rules.  Records equal the oracle's option-W FIND and
    ugpu_find_all."""
    from oracle_lib import OracleDfa
    host = _w_corpus(3 << 20)
    for rx in W_PATTERNS:
        opc = U.compile_regex(rx)
        pat = U.Pattern(opc, word=True)
        want = OracleDfa(opc).find_w(host, want_list=True)
        one = U.find_all(pat, torch.from_numpy(host).cuda(), offsets=True)
        assert (one.count, one.digest, one.dcap) == want[:3], rx
        for ndev in (3, 7, 16):
            r = U.find_all_multi(pat, host, ndev=ndev, offsets=True)
            assert (r.count, r.digest, r.dcap) == want[:3], (rx, ndev)
            assert r.triples() == want[3], (rx, ndev)
