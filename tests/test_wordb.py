"""Word boundaries \\b \\B \\< \\> (META_WBB .. META_EWE edges,
include/reflex/pattern.h:933-940), on the engine's context walk.

The reference tests these meta edges after fetching the byte at the current
position (lib/matcher.cpp:317-404) through include/reflex/matcher.h:1194-1319:
at_wb / at_bw of the match begin, at_ew / at_we of the position.  RE/flex
moves begin-of-match assertions to the accept side (\\bfoo\\b ends in
META_WBE -> META_WBB -> TAKE), so acceptance is a function of the state and a
context of six bits (ugrep_amd/csrc/ctx_bits.hpp; tables.cpp acap over 64
contexts).  Quirks the fixtures pin: at_we as the meta edges call it decodes a
lead byte's code point from the byte after it (a following multi-byte word
character counts as a boundary), and at_wb decodes a continuation byte before
the match back from cur_, which each accept moves.

Expected values are the reference's (tests/golden/wordb_cases.json, written by
tests/golden/make_wordb_golden.py with oracle/_ref/ref_harness), with its match
predictor off (the DFA semantics) and, where different, as ugrep runs it.
CPU: the oracle restatement and a Python walk over the engine's per-context
accepts reproduce them; the drop-in adapter's rule for sending such tables to
the GPU agrees with the reference as run on every fixture.  GPU: whole-buffer
FIND, shards and streams reproduce them."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa, gen

with open(os.path.join(GOLDEN, "wordb_cases.json")) as _f:
    SPEC = json.load(_f)
CASES = SPEC["cases"]

# an assertion between consumed bytes: the meta target goes on with byte edges
# (the interpreter backtracks, lib/matcher.cpp:405-460) -- refused by the
# oracle and the engine, left to the CPU matcher
UNSUPPORTED = {"a\\Bb", "foo\\b bar"}
_INPUTS = {}


def _input(name):
    if name not in _INPUTS:
        if name == "edge":
            _INPUTS[name] = np.frombuffer(bytes.fromhex(SPEC["meta"]["edge_hex"]), np.uint8).copy()
        else:
            spec = next(i["spec"] for i in SPEC["meta"]["inputs"] if i["name"] == name)
            if spec.startswith("file:"):
                path = spec[5:]
                if not os.path.isabs(path):
                    path = os.path.join(os.path.dirname(os.path.dirname(GOLDEN)), path)
                _INPUTS[name] = np.frombuffer(open(path, "rb").read(), np.uint8).copy()
            else:
                kind, seed, off, ln = (int(x) for x in spec[4:].split(":"))
                _INPUTS[name] = gen(kind, seed, off, ln)
    return _INPUTS[name]


def test_fixture_coverage():
    assert len(CASES) >= 150
    kinds = set()
    for c in CASES:
        for w in c["opc"]:
            if (w & 0x00FF0000) == 0 and 0 < (w >> 24) <= 8:
                kinds.add(w >> 24)
    assert kinds == set(range(1, 9)), kinds  # every word-boundary meta edge occurs
    # the predictor differences exist (so the adapter rule below is tested)
    assert any(r["run"] is not None for c in CASES for r in c["results"])


def _predictor_exact(opc):
    """integration/reflex_gpu_matcher.h predictor_exact for word-boundary
    tables without line anchors: the language is finite and no state whose
    accept depends on the word context goes on with byte edges."""
    import ugrep_amd as U
    info = U.host_plan(opc)
    sh = info["shape"]
    return bool(sh & U._lib.SHAPE_FINITE) and not sh & U._lib.SHAPE_WORD_COND


def test_reference_as_run_agrees_on_gpu_eligible_patterns():
    """Where the adapter sends a word-boundary table to the GPU, the reference
    as ugrep runs it (its match predictor on: the lookback cut lbk_ and the
    needle pin_ of lib/pattern.cpp:3990-4290, applied by lib/matcher.cpp:52-86
    and :640-660) gives the DFA semantics (predictor off) on every fixture
    input.  The prediction can only reject a position the DFA matches at after
    a cycle (the lookback cut) or where an accept waits for the context while
    bytes may follow; the rule excludes both.  The fixtures include the rule's
    boundary shapes: shared prefixes under different boundary kinds, \\b
    after a fixed repeat of classes."""
    seen = eligible_shapes = 0
    for c in CASES:
        if c["pattern"] in UNSUPPORTED or c["nul"] or "^" in c["pattern"] or "$" in c["pattern"]:
            continue
        if not any((w & 0x00FF0000) == 0 and 0 < (w >> 24) <= 8 for w in c["opc"]):
            continue  # (no word-boundary edge in this table)
        if _predictor_exact(c["opc"]):
            seen += 1
            eligible_shapes += c["pattern"] in (r"\bfoo\b|\bfoo\B", r"\b(a|ab|abc)\b", r"\b\w{3}\b",
                                                r"\b[a-z]{2}\d\b", r"\b\d{2,3}\b")
            for r in c["results"]:
                assert r["run"] is None, (c["pattern"], c["mode"], r["input"])
    assert seen >= 60 and eligible_shapes >= 5, (seen, eligible_shapes)


def test_oracle_matches_reference():
    for c in CASES:
        o = OracleDfa(c["opc"])
        assert o.supported == (c["pattern"] not in UNSUPPORTED), c["pattern"]
        if not o.supported:
            continue
        for r in c["results"]:
            got = o.find(_input(r["input"]), want_list=r["list"] is not None, nul=c["nul"])
            assert got[:3] == (r["count"], r["digest"], r["dcap"]), (c["pattern"], c["mode"], r["input"])
            if r["list"] is not None:
                assert got[3] == r["list"], (c["pattern"], c["mode"], r["input"])


# ---- a Python walk over the engine's tables (tables.cpp acap, 64 contexts)
_WORD = None


def _isword(cp):
    global _WORD
    if _WORD is None:
        import re
        src = open(os.path.join(os.path.dirname(GOLDEN), "..", "ugrep_amd", "csrc", "unicode_ranges.inc")).read()
        body = src[src.index("k_word_ranges"):]
        body = body[body.index("{") + 1:body.index("};")]
        _WORD = [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{\s*0x([0-9A-Fa-f]+)\s*,\s*0x([0-9A-Fa-f]+)\s*\}", body)]
    lo, hi = 0, len(_WORD) - 1
    while lo <= hi:
        mid = (lo + hi) // 2
        if cp < _WORD[mid][0]:
            hi = mid - 1
        elif cp > _WORD[mid][1]:
            lo = mid + 1
        else:
            return True
    return False


def _utf8(d, k):
    n = len(d)
    rd = lambda i: d[i] if i < n else 0  # noqa: E731
    c = rd(k)
    if c < 0x80:
        return c
    c1 = rd(k + 1)
    if c < 0xC0 or (c == 0xC0 and c1 != 0x80) or c == 0xC1 or (c1 & 0xC0) != 0x80:
        return 0xFFFD
    c1 &= 0x3F
    if c < 0xE0:
        return ((c & 0x1F) << 6) | c1
    c2 = rd(k + 2)
    if (c == 0xE0 and c1 < 0x20) or (c2 & 0xC0) != 0x80:
        return 0xFFFD
    c2 &= 0x3F
    if c < 0xF0:
        return ((c & 0x0F) << 12) | (c1 << 6) | c2
    c3 = rd(k + 3)
    if (c == 0xF0 and c1 < 0x10) or (c == 0xF4 and c1 >= 0x10) or c >= 0xF5 or (c3 & 0xC0) != 0x80:
        return 0xFFFD
    return ((c & 0x07) << 18) | (c1 << 12) | (c2 << 6) | (c3 & 0x3F)


def _alnum(c):
    return 48 <= c <= 57 or 65 <= (c & ~0x20) <= 90


def _ctx_pos(d, q):
    """eol | ew << 1 | we << 2 at position q (ctx_bits.hpp)"""
    n = len(d)
    eol = q >= n or d[q] == 10 or (d[q] == 13 and q + 1 < n and d[q + 1] == 10)
    if q == 0:
        ew = False
    else:
        c = d[q - 1]
        if c == 10:
            ew = False
        elif c == 95:
            ew = True
        elif (c & 0xC0) == 0x80 and q >= 2:
            k = q - 2
            if (d[k] & 0xC0) == 0x80 and k > 0:
                k -= 1
                if (d[k] & 0xC0) == 0x80 and k > 0:
                    k -= 1
            ew = _isword(_utf8(d, k))
        else:
            ew = _alnum(c)
    if q >= n:
        we = True
    else:
        c = d[q]
        we = False if c == 95 else (not _isword(_utf8(d, q + 1))) if (c & 0xC0) == 0xC0 else not _alnum(c)
    return int(eol) | int(ew) << 1 | int(we) << 2


def _ctx_walk(d, p, cur):
    """bol | wb << 1 | bw << 2 of a walk from p, last accept ending at cur, shifted by 3"""
    bol = p == 0 or d[p - 1] == 10
    if p == 0:
        wb = True
    else:
        c = d[p - 1]
        if c == 10:
            wb = True
        elif c == 95:
            wb = False
        elif (c & 0xC0) == 0x80:
            k = cur - 1
            if k > 0:
                k -= 1
                if (d[k] & 0xC0) == 0x80 and k > 0:
                    k -= 1
                    if (d[k] & 0xC0) == 0x80 and k > 0:
                        k -= 1
            wb = not _isword(_utf8(d, k))
        else:
            wb = not _alnum(c)
    c = d[p] if p < len(d) else 0
    bw = True if c == 95 else _isword(_utf8(d, p)) if (c & 0xC0) == 0xC0 else _alnum(c)
    return (int(bol) | int(wb) << 1 | int(bw) << 2) << 3


def _ctx(nctx, d, p, cur, q):
    """the acap context of a walk from p (last accept ending at cur) at q:
    64 word contexts, or the 4 line contexts bol * 2 + eol"""
    if nctx == 64:
        return _ctx_walk(d, p, cur) + _ctx_pos(d, q)
    bol = p == 0 or d[p - 1] == 10
    return int(bol) * 2 + (_ctx_pos(d, q) & 1)


def _walk_find(tab, acap, nctx, data, nul):
    trans, cls, row = tab["trans"], tab["cls"], tab["info"]["row"]
    log_row = row.bit_length() - 1
    fmt = tab["info"]["format"]
    d = bytes(data)
    n = len(d)
    out = []
    p = 0
    while p < n:
        e = int(tab["start"])
        last, a = -1, 0
        c0 = int(acap[(e >> log_row) * nctx + _ctx(nctx, d, p, p, p)])
        if c0:
            last, a = p, c0
        q = p
        while q < n:
            col = d[q] if fmt == 0 else int(cls[d[q]])
            e = int(trans[e + col])
            if e == 0:
                break
            q += 1
            c1 = int(acap[(e >> log_row) * nctx + _ctx(nctx, d, p, last if last >= 0 else p, q)])
            if c1:
                last, a = q, c1
        if last > p or (last == p and nul):
            out.append([p, last - p, a])
        p = last if last > p else p + 1
    return out


def test_engine_context_tables_match_reference():
    """tables.cpp's per-context accepts of the reference's meta edges, walked
    in Python, give the reference's match lists on the small inputs."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_context
    for c in CASES:
        if c["pattern"] in UNSUPPORTED:
            with pytest.raises(U.Unsupported):
                U.host_tables(c["opc"])
            continue
        info = U.host_plan(c["opc"])
        if info["format"] == 2:
            continue  # (wide tables: no u16 host form; the GPU test runs them)
        tab = U.host_tables(c["opc"])
        nctx = tab["info"]["contexts"]
        assert nctx in (4, 64), (c["pattern"], nctx)
        acap, anchored, _ = host_context(c["opc"])
        assert anchored
        for r in c["results"]:
            if r["list"] is None or r["input"] != "edge":
                continue
            assert _walk_find(tab, acap, nctx, _input(r["input"]), c["nul"]) == r["list"], (c["pattern"], c["mode"])


# ---- GPU: the context walk (wfind_kernel, fix_kernel merges, forest) on the
# reference's own opcode tables
def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return torch


@pytest.mark.gpu
def test_gpu_find_all_matches_reference():
    torch = _torch()
    import ugrep_amd as U
    n = 0
    for c in CASES:
        if c["pattern"] in UNSUPPORTED:
            with pytest.raises(U.Unsupported):
                U.Pattern(c["opc"], empty=c["nul"])
            continue
        pat = U.Pattern(c["opc"], empty=c["nul"])
        info = pat.info()
        # prefiltered tables: sparse_kernel's context walks; the rest: wfind_kernel
        assert info["kernel"] == (0 if info["prefilter_ppm"] and info["format"] == 0 else 4), c["pattern"]
        for r in c["results"]:
            data = _input(r["input"])
            dev = torch.from_numpy(data).to("cuda")
            torch.cuda.synchronize()
            got = U.find_all(pat, dev, offsets=r["list"] is not None)
            assert (got.count, got.digest, got.dcap) == (r["count"], r["digest"], r["dcap"]), (c["pattern"], c["mode"], r["input"])
            if r["list"] is not None:
                assert [list(t) for t in got.triples()] == r["list"], (c["pattern"], c["mode"], r["input"])
            n += 1
    assert n > 800


@pytest.mark.gpu
def test_gpu_shards_and_streams_match_reference():
    """ugpu_find_all_multi (virtual shards: each shard's context bytes, at_ew
    and at_wb across the cut) and the stream API (chunks of 997 bytes: the
    carried prefix and the halo of at_we's look past the lead byte)."""
    _torch()
    import ugrep_amd as U
    for c in CASES:
        if c["pattern"] in UNSUPPORTED:
            continue
        pat = U.Pattern(c["opc"], empty=c["nul"])
        for r in c["results"]:
            if r["input"] not in ("edge", "Hello.java", "gen4_256k"):
                continue
            data = _input(r["input"])
            want = (r["count"], r["digest"], r["dcap"])
            got = U.find_all_multi(pat, data, ndev=3, offsets=False)
            assert (got.count, got.digest, got.dcap) == want, ("multi", c["pattern"], c["mode"], r["input"])
            st = U.Stream(pat)
            cnt = dg = dc = 0
            step = 997
            for k in range(0, len(data), step):
                res = st.feed(data[k:k + step], final=k + step >= len(data))
                cnt += res.count
                dg = (dg + res.digest) & ((1 << 64) - 1)
                dc = (dc + res.dcap) & ((1 << 64) - 1)
            if len(data) == 0:
                st.feed(data, final=True)
            assert (cnt, dg, dc) == want, ("stream", c["pattern"], c["mode"], r["input"])


# ---- the native compiler (regex_compile.cpp): \b \B \< \> before the first
# or after the last atom of a top-level alternative
COMPILER_REFUSES = {"a\\Bb", "foo\\b bar"}


def test_compiler_word_boundaries_match_reference():
    """ugpu_compile's meta-edge encoding, in the RE/flex mode (the converted
    regex the reference Pattern holds, as the drop-in adapter compiles it) and
    the ERE mode: accepts per context equal to the reference's tables
    (ugpu_tables_equivalent_host compares all 64 contexts), and the Python walk
    over the engine's tables gives the reference's match lists."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_context, host_equivalent
    walked = 0
    for c in CASES:
        forms = [("reflex", bytes.fromhex(c["conv"]))]
        if c["mode"] in ("re", "reN"):
            forms.append(("ere", c["pattern"]))
        for form, rx in forms:
            if c["pattern"] in COMPILER_REFUSES:
                with pytest.raises(U.Unsupported):
                    U.compile_regex(rx, reflex=form == "reflex")
                continue
            opc = U.compile_regex(rx, reflex=form == "reflex")
            assert host_equivalent(opc, c["opc"]), (c["pattern"], c["mode"], form)
            info = U.host_plan(opc)
            ref = U.host_plan(c["opc"])
            assert (info["kernel"], info["contexts"]) == (ref["kernel"], ref["contexts"]) or \
                info["states"] != ref["states"], c["pattern"]
            if info["format"] == 2:
                continue
            tab = U.host_tables(opc)
            acap, _, _ = host_context(opc)
            for r in c["results"]:
                if r["list"] is None or r["input"] != "edge":
                    continue
                assert _walk_find(tab, acap, info["contexts"], _input(r["input"]), c["nul"]) == r["list"], \
                    (c["pattern"], c["mode"], form)
                walked += 1
    assert walked >= 200


SPARSE_CTX = [r"\bfoo\b", r"\<(in|ut)\>", r"\bdolor\b", r"\Boo\B", r"x\>", r"\<con", r"um\>", r"^foo", r"ing$",
              r"\b(lorem|ipsum|sit)\b", r"\<(foo|bar|baz)\>", r"\b(in|ut)\b"]


def _ctx_corpus(n):
    """lorem text, C2 words and the C4 UTF-8 corpus in 64 KiB slices, with
    CR LF line ends, '_' and digits next to the pattern words"""
    from oracle_lib import gen, GOLDEN
    lorem = np.frombuffer(open(os.path.join(GOLDEN, "lorem.utf8.txt"), "rb").read(), np.uint8)
    parts = [np.tile(lorem, 8)[:64 << 10], gen(1, 3, 0, 64 << 10), gen(4, 3, 0, 64 << 10),
             np.frombuffer(b"foo_foo 9foo foo9 \r\nfoo\r\n_in ut\xc3\xa9ut in\xe2\x82\xacin xing\n" * 512, np.uint8)]
    out = np.concatenate(parts * (n // sum(p.size for p in parts) + 1))[:n]
    return np.ascontiguousarray(out)


@pytest.mark.gpu
def test_gpu_sparse_context_walks_match_oracle():
    """prefiltered word-boundary and line-anchor tables run
    sparse_kernel with context walks (kernel 0).  Against the oracle's
    restatement of the meta tests (pinned to the reference fixtures above)
    on 6 MiB of mixed text: totals, match lists (OFFSETS, staged and WRITE
    pass), three virtual shards, and the same scans on wfind_kernel
    (UGPU_SPARSE=0)."""
    torch = _torch()
    import ugrep_amd as U
    from oracle_lib import OracleDfa
    data = _ctx_corpus(6 << 20)
    dev = torch.from_numpy(data).to("cuda")
    torch.cuda.synchronize()
    for rx in SPARSE_CTX:
        opc = U.compile_regex(rx)
        pat = U.Pattern(opc)
        assert pat.info()["kernel"] == 0, rx
        cnt, dg, dc, lst = OracleDfa(opc).find(data, want_list=True)
        got = U.find_all(pat, dev, offsets=True)
        assert (got.count, got.digest, got.dcap) == (cnt, dg, dc), rx
        assert [list(t) for t in got.triples()] == lst, rx
        m = U.find_all_multi(pat, data, ndev=3, offsets=False)
        assert (m.count, m.digest, m.dcap) == (cnt, dg, dc), rx
        os.environ["UGPU_SPARSE"] = "0"
        try:
            pw = U.Pattern(opc)
            g2 = U.find_all(pw, dev, offsets=False)
        finally:
            os.environ.pop("UGPU_SPARSE", None)
        assert (g2.count, g2.digest, g2.dcap) == (cnt, dg, dc), rx
