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


def test_word_plus_is_recognised():
    """The engine serves W on \\w+ tables by the non-W kernels when the bytes
    are valid UTF-8; it recognises them by table equivalence with its own \\w+."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_equivalent
    w = U.compile_regex(r"\w+")
    ref = next(c["opc"] for c in CASES if c["pattern"] == r"\w+")
    assert host_equivalent(ref, w)
    for rx in (r"\w*x", r"[A-Za-z_][A-Za-z0-9_]*", r"\S+", r"\w+\d"):
        assert not host_equivalent(U.compile_regex(rx), w), rx


@pytest.mark.gpu
def test_gpu_w_word_plus_fast_path():
    """\\w+ with W: on valid UTF-8 the scan runs the non-W kernel (UGPU_TOT_WFAST) and
    equals the oracle's W restatement; invalid UTF-8 (a stray continuation byte
    after a word character changes at_wb) and entries after a word character
    fall back to wfind_kernel, also exact."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    ref = next(c["opc"] for c in CASES if c["pattern"] == r"\w+")
    host = gen(4, 17, 0, 24 << 20)
    bad = host.copy()
    bad[5 << 20] = ord("x")
    bad[(5 << 20) + 1] = 0x80  # "x\x80a": at_wb(a) looks back past the stray byte
    bad[(5 << 20) + 2] = ord("a")
    for opc in (ref, U.compile_regex(r"\w+")):
        pat = U.Pattern(opc, word=True)
        assert pat.info()["kernel"] == 6  # (the non-W kernel: xc_kernel's U mode)
        for data, fast in ((host, True), (bad, False)):
            dev = torch.from_numpy(data).to("cuda")
            torch.cuda.synchronize()
            want = OracleDfa(opc).find_w(data)[:3]
            sc = U.Scanner(pat)
            sc.scan(dev.data_ptr(), 0, data.size, data.size, True, 0, torch.cuda.current_stream().cuda_stream)
            t = sc.totals()
            assert (t.count, t.digest, t.dcap) == want
            assert bool(t.flags & 16) == fast
            res = U.find_all(pat, dev, offsets=True)
            assert (res.count, res.digest, res.dcap) == want
        # entries: after a space (fast), inside a word (fallback)
        dev = torch.from_numpy(host).to("cuda")
        torch.cuda.synchronize()
        sp = int(np.nonzero(host[1000:] == ord(" "))[0][0]) + 1001
        for start in (sp, sp + 1, 777):
            res = U.find_all(pat, dev, start=start)
            assert (res.count, res.digest, res.dcap) == OracleDfa(opc).find_w(host, start=start)[:3], start


@pytest.mark.gpu
def test_gpu_w_word_plus_edges():
    """\\w+ with W runs xc_kernel's U mode (one pass, no isutf8 pass): at a run
    start after a byte >= 0x80 it evaluates at_wb; where that decodes a word
    character (a stray continuation byte after one) the range goes to
    wfind_kernel (no UGPU_TOT_WFAST).  Cut-off leads and non-word code points
    beside words, and high bytes away from words, keep the fast path.  Every
    result equals the oracle's W restatement."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    ref = next(c["opc"] for c in CASES if c["pattern"] == r"\w+")
    base = gen(4, 23, 0, 3 << 20)
    at = 1 << 20
    base[at - 16:at + 48] = ord(" ")  # (the inserts sit between spaces)
    cases = [(b"", True), (b" \xff \xc3 \x80\x80 ", True), (b" x\x80a ", False), (b" ab\xc3 ", True),
             (b" \xe4\xb8ab ", True), (b" word\xe2\x82\xac ", True), (b" \xc3\xa9t\xc3\xa9\xc3 ", True),
             (b" \xe2\x82\xac\xe2\x82\xac ", True), (b" \xe2\x82\xacab ", True), (b" \xc3\x82\xaca ", False),
             (b" x\x80\x80\x80a ", False), (b" \xce\xb1\x80\xce\xb2 ", False), (b" _\x80a ", False)]
    for opc in (ref, U.compile_regex(r"\w+")):
        pat = U.Pattern(opc, word=True)
        for ins, fast in cases:
            data = base.copy()
            data[at:at + len(ins)] = np.frombuffer(ins, np.uint8)
            dev = torch.from_numpy(data).to("cuda")
            torch.cuda.synchronize()
            want = OracleDfa(opc).find_w(data, want_list=True)
            sc = U.Scanner(pat)
            sc.scan(dev.data_ptr(), 0, data.size, data.size, True, 0, torch.cuda.current_stream().cuda_stream)
            t = sc.totals()
            assert (t.count, t.digest, t.dcap) == want[:3], ins
            assert bool(t.flags & 16) == fast, ins
            res = U.find_all(pat, dev, offsets=True)
            assert res.triples() == want[3], ins


@pytest.mark.gpu
def test_gpu_w_identifiers_on_xc():
    """Option W on the identifier table runs xc_kernel with the W rules
    (UGPU_TOT_WFAST) on ASCII input -- runs that begin with a digit, entries
    inside words and after digits, several grids -- and falls back to
    wfind_kernel when bytes >= 0x80 appear; all equal to the oracle."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    ref = next(c["opc"] for c in CASES if c["pattern"] == "[A-Za-z_][A-Za-z0-9_]*")
    pat = U.Pattern(ref, word=True)
    assert pat.info()["kernel"] == 5
    code = gen(3, 19, 0, 6 << 20)
    code[4096:4096 + 3000] = ord("7")  # a digit run across chunks, then letters
    code[4096 + 3000:4096 + 3010] = ord("q")
    utf = gen(4, 19, 0, 2 << 20)
    st = torch.cuda.current_stream().cuda_stream
    for data, fast in ((code, True), (utf, False)):
        dev = torch.from_numpy(data).to("cuda")
        torch.cuda.synchronize()
        want_all = OracleDfa(ref).find_w(data)[:3]
        for g in ("", "3", "77"):
            if g:
                os.environ["UGPU_MAX_GRID"] = g
            try:
                sc = U.Scanner(pat)
                sc.scan(dev.data_ptr(), 0, data.size, data.size, True, 0, st)
                t = sc.totals()
            finally:
                os.environ.pop("UGPU_MAX_GRID", None)
            assert (t.count, t.digest, t.dcap) == want_all, g
            assert bool(t.flags & 16) == fast
        for start in (1, 4096 + 2999, 4096 + 3001, 12345, 1 << 20):
            res = U.find_all(pat, dev, start=start)
            assert (res.count, res.digest, res.dcap) == OracleDfa(ref).find_w(data, start=start)[:3], start
        res = U.find_all(pat, dev, offsets=True)
        cnt, dg, dc, lst = OracleDfa(ref).find_w(data, want_list=True)
        assert (res.count, res.digest, res.dcap) == (cnt, dg, dc)
        assert res.triples() == lst
    # a range starting on a 1024-byte chunk border right after a multi-byte
    # character: at_wb there decodes that character (word: no match starts at
    # the border; non-word: one does), which xc_kernel's chunks never see
    base = gen(3, 23, 0, 1 << 20)
    for ch in ("\u00e9", "\u20ac", "\u00d7"):
        data = base.copy()
        enc = np.frombuffer(ch.encode(), np.uint8)
        for border in (2048, 4096, 65536):
            data[border - enc.size:border] = enc
            data[border:border + 5] = np.frombuffer(b"abcde", np.uint8)
        dev = torch.from_numpy(data).to("cuda")
        torch.cuda.synchronize()
        for border in (2048, 4096, 65536):
            res = U.find_all(pat, dev, start=border, offsets=True)
            cnt, dg, dc, lst = OracleDfa(ref).find_w(data, start=border, want_list=True)
            assert (res.count, res.digest, res.dcap) == (cnt, dg, dc), (ch, border)
            assert res.triples() == lst, (ch, border)
            assert (lst[0][0] == border) == (ch != "\u00e9"), (ch, border, lst[:2])


@pytest.mark.gpu
def test_gpu_w_word_start_filter():
    """Option W on prefiltered tables drops the candidates that follow an
    ASCII letter (ScanParams::wstart).  Patterns whose first
    bytes are letters, digits, '_' and non-word bytes, over text where they
    follow letters, digits, '_', UTF-8 letters and separators, at lane and
    chunk borders: equal to the oracle with the filter on and off
    (UGPU_WSTART=0), whole buffers and OFFSETS."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    rng = np.random.default_rng(11)
    toks = ["ing", "xing", "_ing", "9ing", "éing", "ing9", "sing", "-ing", "ing-", "ing_", "ingé", "a", " ", " ", "\n",
            "-", "_", "é", "ж", "7", "walking", "sing ing", "in g"]
    parts = [toks[int(i)] for i in rng.integers(0, len(toks), 400000)]
    host = np.frombuffer("".join(parts).encode(), np.uint8).copy()
    # planted at 16-byte lane and 1 KiB chunk borders
    for p in range(1024 - 3, host.size - 8, 4096):
        host[p:p + 5] = np.frombuffer(b"aing ", np.uint8)
    for p in range(16 * 7 - 1, host.size - 8, 16 * 61):
        host[p:p + 4] = np.frombuffer(b"ing ", np.uint8)
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    n_sparse = 0
    for rx in ("[a-z]+ing", "ing", "-ing", "_ing|ing", "[0-9]ing", "ing|[a-z]ing", "é?ing"):
        opc = U.compile_regex(rx)
        want = OracleDfa(opc).find_w(host, want_list=True)
        for ws in ("1", "0"):
            os.environ["UGPU_WSTART"] = ws
            try:
                pat = U.Pattern(opc, word=True)
                n_sparse += pat.info()["kernel"] == 0
                res = U.find_all(pat, dev, offsets=True)
            finally:
                os.environ.pop("UGPU_WSTART", None)
            assert (res.count, res.digest, res.dcap) == want[:3], (rx, ws)
            assert res.triples() == want[3], (rx, ws)
    assert n_sparse >= 6  # (the filter is sparse_kernel's)
