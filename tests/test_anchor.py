"""Line anchors (^ / $: META_BOL / META_EOL edges, include/reflex/pattern.h:942-943)
and Matcher option N (empty matches: ugrep -Y, and -x which also wraps the
pattern as ^(?:...)$, src/cnf.hpp:167-185, src/ugrep.cpp:8381-8386).

Expected values are the reference's (tests/golden/anchor_cases.json, written by
tests/golden/make_anchor_golden.py with oracle/_ref/ref_harness: the reference
libreflex Matcher with options "" or "N"), for 41 patterns in Unicode and -U
byte mode over an edge-case text (empty lines, CR LF, lone CR, a last line
without newline, leading newlines), the reference's CLI inputs and corpus
slices.  Each result is the reference Matcher with its match predictor off
(every position a FIND candidate: the DFA semantics of lib/matcher.cpp:125-546,
which the engine implements) and, where it differs, "run": the Matcher as ugrep
runs it.  The predictor rejects positions the DFA matches at through meta edges
for anchored patterns without option N and for interior anchors ("a$|ab": the
reference CLI prints 0 for ugrep -c 'a$|ab' on "xa\nb\nzzzz\n"); ugrep itself
sets N for every pattern that starts with ^ or ends with $ (src/cnf.hpp:201-206)
and for -x, and on exactly that class (gpu_eligible below, the drop-in
adapter's rule) the two agree on every fixture.

CPU: the oracle restatement (orc_find_a) and a Python walk over the engine's
per-context accept table (tables.cpp acap, ugpu_tables_context_host) both
reproduce them.  GPU: ugpu_find_all / ugpu_find_all_multi / the stream API
reproduce them, with match records."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa, gen

with open(os.path.join(GOLDEN, "anchor_cases.json")) as _f:
    SPEC = json.load(_f)
CASES = SPEC["cases"]


def _load(name):
    if name == "edge":
        return np.frombuffer(bytes.fromhex(SPEC["meta"]["edge_hex"]), np.uint8).copy()
    spec = next(i["spec"] for i in SPEC["meta"]["inputs"] if i["name"] == name)
    if spec.startswith("file:"):
        path = spec[5:]
        if not os.path.isabs(path):
            path = os.path.join(os.path.dirname(os.path.dirname(GOLDEN)), path)
        return np.frombuffer(open(path, "rb").read(), np.uint8).copy()
    kind, seed, off, ln = (int(x) for x in spec[4:].split(":"))
    return gen(kind, seed, off, ln)


_INPUTS = {}


def _input(name):
    if name not in _INPUTS:
        _INPUTS[name] = _load(name)
    return _INPUTS[name]


# meta-edge targets that go on consuming bytes (the interpreter then runs two
# walks through its backtrack point, lib/matcher.cpp:405-423): refused by the
# oracle and by the engine (tables.cpp), left to the CPU matcher
UNSUPPORTED = {"(^|,)foo"}
# wide tables (states x class row > 65536, u32 entries: tables.cpp FMT_WIDE)
# have no u16 host form for the Python walk below; the GPU runs them
TOO_LARGE = {("^(?:\\w+ \\w+)$", "re"), ("^(?:\\w+ \\w+)$", "reN")}


def _refused(c):
    return c["pattern"] in UNSUPPORTED or (c["pattern"], c["mode"]) in TOO_LARGE


def gpu_eligible(regex, nul):
    """The drop-in adapter's rule for tables with ^/$ edges
    (integration/reflex_gpu_matcher.h anchors_outer): option N on, and the
    anchors only a leading ^ and/or a trailing $ of the regex (^ and $ inside
    bracket expressions and escaped ones are literals)."""
    if not nul:
        return False
    i, n, inner = 0, len(regex), []
    while i < n:
        ch = regex[i]
        if ch == "\\":
            i += 2
            continue
        if ch == "[":
            j = i + 1
            if j < n and regex[j] == "^":
                j += 1
            if j < n and regex[j] == "]":
                j += 1
            while j < n and regex[j] != "]":
                j += 2 if regex[j] == "\\" else 1
            i = j + 1
            continue
        if ch in "^$" and not (ch == "^" and i == 0) and not (ch == "$" and i == n - 1):
            inner.append(i)
        i += 1
    return not inner


def test_fixture_coverage():
    assert len(CASES) >= 150
    assert sum(1 for c in CASES if c["nul"]) >= 75
    # the reference's own tables carry the edges the engine must read
    assert any(OracleDfa(c["opc"]).anchored for c in CASES)
    # the predictor differences the fixtures document exist (so the rule below is tested)
    assert any(r["run"] is not None for c in CASES for r in c["results"] if c["nul"])
    assert any(r["run"] is not None for c in CASES for r in c["results"] if not c["nul"])


def test_reference_as_run_agrees_on_gpu_eligible_patterns():
    """Where the adapter sends an anchored table to the GPU, the reference as
    ugrep runs it (predictor on) gives the DFA semantics on every fixture."""
    seen = 0
    for c in CASES:
        if c["pattern"] in UNSUPPORTED or not OracleDfa(c["opc"]).anchored:
            continue
        if gpu_eligible(c["pattern"], c["nul"]):
            seen += 1
            for r in c["results"]:
                assert r["run"] is None, (c["pattern"], c["mode"], r["input"])
    assert seen >= 50
    assert not gpu_eligible("a$|ab", True) and not gpu_eligible("^\\w+", False)
    assert gpu_eligible("^(?:[^\\n]*r)$", True) and gpu_eligible("^\\$x\\^$", True)


def test_oracle_matches_reference():
    for c in CASES:
        o = OracleDfa(c["opc"])
        assert o.supported == (c["pattern"] not in UNSUPPORTED), c["pattern"]
        if not o.supported:
            continue
        for r in c["results"]:
            data = _input(r["input"])
            got = o.find(data, want_list=r["list"] is not None, nul=c["nul"])
            assert got[:3] == (r["count"], r["digest"], r["dcap"]), (c["pattern"], c["mode"], r["input"])
            if r["list"] is not None:
                assert got[3] == r["list"], (c["pattern"], c["mode"], r["input"])


def _walk_find(tab, acap, data, nul):
    """FIND over the engine's dense tables + per-context accepts (tables.hpp
    acap), restated in Python: bol fixed at the walk start, eol tested on the
    byte after each position."""
    trans, cls, row = tab["trans"], tab["cls"], tab["info"]["row"]
    log_row = row.bit_length() - 1
    fmt = tab["info"]["format"]
    data = bytes(data)
    n = len(data)
    out = []

    def acc(e, bol, q):
        s = e >> log_row
        eol = q >= n or data[q] == 10 or (data[q] == 13 and q + 1 < n and data[q + 1] == 10)
        return int(acap[s * 4 + bol * 2 + int(eol)])

    p = 0
    while p < n:
        bol = 1 if p == 0 or data[p - 1] == 10 else 0
        e = int(tab["start"])
        last, a = -1, 0
        c0 = acc(e, bol, p)
        if c0:
            last, a = p, c0
        q = p
        while q < n:
            col = data[q] if fmt == 0 else int(cls[data[q]])
            e = int(trans[e + col])
            if e == 0:
                break
            q += 1
            c1 = acc(e, bol, q)
            if c1:
                last, a = q, c1
        if last > p or (last == p and nul):
            out.append([p, last - p, a])
        p = last if last > p else p + 1
    return out


def test_engine_context_tables_match_reference():
    """tables.cpp's conversion of the reference's meta edges (acap) walked in
    Python gives the reference's match lists on the small inputs."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_context
    for c in CASES:
        if _refused(c):
            with pytest.raises(U.Unsupported):
                U.host_tables(c["opc"])
            continue
        tab = U.host_tables(c["opc"])
        acap, anchored, _ = host_context(c["opc"])
        for r in c["results"]:
            if r["list"] is None:
                continue
            data = _input(r["input"])
            assert _walk_find(tab, acap, data, c["nul"]) == r["list"], (c["pattern"], c["mode"], r["input"])


# anchors the native compiler refuses (not a leading ^ / trailing $ of a
# top-level alternative: regex_compile.cpp) -- the CPU matcher keeps them
# (round 6: anchors in a leading or trailing group are distributed over the
# alternative, regex_compile.cpp rx_assertion_groups -- (^|,)foo compiles as
# ^foo|,foo -- and these fixtures pin that the reference matches the same)
COMPILER_REFUSES = set()


def test_compiler_anchors_match_reference():
    """regex_compile.cpp's META_BOL / META_EOL encoding of ^ and $, in the ERE
    mode (the user's regex) and the RE/flex mode (the converted regex the
    reference Pattern holds, as the drop-in adapter compiles it), walked over
    the engine's tables: the reference's match lists."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_context
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
            if (c["pattern"], c["mode"]) in TOO_LARGE:
                with pytest.raises(U.Unsupported):
                    U.host_tables(opc)
                continue
            tab = U.host_tables(opc)
            acap, anchored, _ = host_context(opc)
            ref = OracleDfa(c["opc"])
            # (the reference's tables of anchor groups keep meta edges the
            # oracle refuses; the compiled ones are anchored either way)
            assert anchored == (ref.anchored if ref.supported else True), (c["pattern"], form)
            for r in c["results"]:
                if r["list"] is None:
                    continue
                got = _walk_find(tab, acap, _input(r["input"]), c["nul"])
                assert got == r["list"], (c["pattern"], c["mode"], form, r["input"])
                walked += 1
    assert walked >= 400


# ---------------------------------------------------------------- GPU
def _dev(data):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda")
    torch.cuda.synchronize()
    return t


@pytest.mark.gpu
def test_gpu_anchor_cases_match_reference():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    devs = {}
    for c in CASES:
        if c["pattern"] in UNSUPPORTED:
            with pytest.raises(U.Unsupported):
                U.Pattern(c["opc"], empty=c["nul"])
            continue
        pat = U.Pattern(c["opc"], empty=c["nul"])
        for r in c["results"]:
            if r["input"] not in devs:
                devs[r["input"]] = _dev(_input(r["input"]))
            res = U.find_all(pat, devs[r["input"]], offsets=r["list"] is not None)
            assert (res.count, res.digest, res.dcap) == (r["count"], r["digest"], r["dcap"]), \
                (c["pattern"], c["mode"], r["input"])
            if r["list"] is not None:
                assert res.triples() == r["list"], (c["pattern"], c["mode"], r["input"])


@pytest.mark.gpu
def test_gpu_anchor_starts_streams_and_shards():
    """Search starts inside lines and after newlines, stream chunkings (the
    chunk border inside and at the start of lines: the line context is
    carried), and multi-device shards cut at arbitrary offsets (each shard's
    first byte takes its line context from the byte before): all == the oracle
    (itself pinned to the reference above)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    data = gen(1, 7, 0, 1 << 20)
    data[1000:1004] = np.frombuffer(b"\r\n\n\n", np.uint8)
    picks = [c for c in CASES if c["pattern"] in ("^(?:foo|ba+r)$", "^(?:\\w+)$", "^$", "^\\w+", "\\w+$", "^a|b",
                                                  "^(?:.*)$", "a*", "^ *", " *$")]
    assert len(picks) >= 20
    dev = _dev(data)
    rng = np.random.default_rng(3)
    for c in picks:
        o = OracleDfa(c["opc"])
        pat = U.Pattern(c["opc"], empty=c["nul"])
        for start in (1, 999, 1002, 1003, 77777):
            res = U.find_all(pat, dev, start=start)
            assert (res.count, res.digest, res.dcap) == o.find(data, start=start, nul=c["nul"])[:3], (c["pattern"], start)
        want = o.find(data, want_list=True, nul=c["nul"])
        st = U.Stream(pat, keep=4096)
        trip, i = [], 0
        cuts = sorted(set(int(x) for x in rng.integers(1, data.size, 30)) | {1001, 1002, 1004})
        for cut in cuts + [data.size]:
            r = st.feed(data[i:cut].tobytes(), final=cut == data.size)
            trip += r.triples()
            i = cut
        assert trip == want[3], (c["pattern"], c["mode"], "stream")
        for ndev in (3, 8):
            r = U.find_all_multi(pat, data, ndev=ndev, offsets=True)
            assert (r.count, r.digest, r.dcap) == want[:3], (c["pattern"], c["mode"], ndev)
            assert r.triples() == want[3], (c["pattern"], c["mode"], ndev)
