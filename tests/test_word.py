"""ugrep -w (Matcher option W): the oracle restatement and the GPU path
(wfind_kernel + fix_kernel through the C ABI) against the reference's match
lists (tests/golden/word_cases.json, tools/gen_word_golden.py: libreflex
compiled from /root/reference, reflex::Matcher(pat, input, "W"))."""
import json
import os

import numpy as np
import pytest

from oracle_lib import OracleDfa, gen

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "word_cases.json")) as _f:
    CASES = json.load(_f)
with open(os.path.join(HERE, "golden", "word_edge.txt"), "rb") as _f:
    EDGE = np.frombuffer(_f.read(), np.uint8)


def _input(c):
    return EDGE if c["gen"] is None else gen(*c["gen"])


def test_oracle_w_matches_reference():
    for c in CASES:
        r = OracleDfa(c["opc"]).find_w(_input(c), want_list=c["list"] is not None)
        assert r[:3] == (c["count"], c["digest"], c["dcap"]), (c["pattern"], c["input"])
        if c["list"] is not None:
            assert r[3] == c["list"], (c["pattern"], c["input"])


def test_w_differs_from_plain_find():
    """The fixtures exercise W: plain FIND finds more matches on the edge text."""
    c = next(c for c in CASES if c["pattern"] == "foo" and c["input"] == "edge")
    assert OracleDfa(c["opc"]).find(EDGE)[0] > c["count"] > 0


def test_compiled_tables_with_w():
    """W over tables from the native compiler == W over the reference's tables."""
    import ugrep_amd as U
    for c in CASES[::4]:
        mine = U.compile_regex(c["pattern"], fixed=c["mode"] == "F")
        assert OracleDfa(mine).find_w(_input(c))[:3] == (c["count"], c["digest"], c["dcap"]), c["pattern"]


@pytest.mark.gpu
def test_gpu_w_matches_reference():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    for c in CASES:
        buf = _input(c)
        dev = torch.from_numpy(np.ascontiguousarray(buf)).to("cuda")
        torch.cuda.synchronize()
        pat = U.Pattern(c["opc"], word=True)
        res = U.find_all(pat, dev, offsets=c["list"] is not None)
        assert (res.count, res.digest, res.dcap) == (c["count"], c["digest"], c["dcap"]), (c["pattern"], c["input"])
        if c["list"] is not None:
            assert res.triples() == c["list"], (c["pattern"], c["input"])


@pytest.mark.gpu
def test_gpu_w_large_vs_oracle():
    """Tens of MiB (many records, stitched by fix_kernel), identifier and word
    patterns with W, and a nonzero search start, == the oracle."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    for kind, rx in ((3, "[A-Za-z_][A-Za-z0-9_]*"), (4, r"\w+"), (1, "foo|bar|baz"), (4, "o+")):
        host = gen(kind, 9, 0, 24 << 20)
        dev = torch.from_numpy(host).to("cuda")
        torch.cuda.synchronize()
        opc = U.compile_regex(rx)
        pat = U.Pattern(opc, word=True)
        res = U.find_all(pat, dev)
        assert (res.count, res.digest, res.dcap) == OracleDfa(opc).find_w(host)[:3], rx
        res = U.find_all(pat, dev, start=12345)
        assert (res.count, res.digest, res.dcap) == OracleDfa(opc).find_w(host, start=12345)[:3], rx
