"""CPU: the C-ABI library loads and exports its header, and its host-side table
builder (opcode words -> dense device tables) reproduces the reference's
matches when walked on the CPU with the exact FIND chain."""
import ctypes
import os

import numpy as np
import pytest

import ugrep_amd
from ugrep_amd import _lib
from oracle_lib import case_input

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# line anchors (anchor_bol, anchor_eol) are supported since round 3 and word
# boundaries since round 4 (per-context accepts: tests/test_anchor.py,
# tests/test_wordb.py); lookahead is not
# (lookahead runs on the GPU since round 6, tests/test_lookahead.py; what stays
# unsupported: the buffer anchors \A \Z and indent metas -- the reference's
# words for -U '\Afoo', from oracle/_ref/ref_harness dump)
UNSUPPORTED = set()
BOB_FOO = [1717960706, 16777215, 1869545476, 16777215, 1869545478, 16777215, 184549384, 16777215, 4261412865, 16777215]
ANCHORED = {"anchor_bol", "anchor_eol", "word_boundary"}


def test_exports_every_declared_symbol():
    names = _lib.declared_symbols()
    assert len(names) >= 15
    for n in names:
        assert hasattr(_lib.lib, n), n
    assert ugrep_amd.lib.ugpu_version().startswith(b"ugrep_amd")


def test_build_id_matches_sources():
    """Provenance: the loaded libugrep_amd.so embeds the hash of the sources it
    was built from (ugpu_build_id, tools/srchash.py); _lib warns on a stale one."""
    import subprocess
    import sys
    from ugrep_amd import _lib
    bid, ok = _lib.build_id()
    assert bid.startswith("src:") and " git:" in bid, bid
    assert ok, (bid, _lib._source_hash())
    here = subprocess.check_output([sys.executable, os.path.join(REPO, "tools", "srchash.py"), REPO], text=True)
    assert bid.split()[0] == "src:" + here.strip()


def test_unsupported_patterns(patterns):
    for name, p in patterns.items():
        if name in UNSUPPORTED:
            with pytest.raises(ugrep_amd.Unsupported):
                ugrep_amd.host_tables(p["opc"])
        else:
            ugrep_amd.host_tables(p["opc"])
            from ugrep_amd.matcher import host_context
            assert host_context(p["opc"])[1] == (name in ANCHORED), name


def test_buffer_anchor_rejected():
    with pytest.raises(ugrep_amd.Unsupported):
        ugrep_amd.host_tables(BOB_FOO)
    with pytest.raises(ugrep_amd.Unsupported):
        ugrep_amd.host_plan(BOB_FOO)


def test_malformed_table_rejected():
    with pytest.raises(ugrep_amd.UgpuError):
        ugrep_amd.host_tables([0x61610005])  # goto past the end
    with pytest.raises(ugrep_amd.UgpuError):
        ugrep_amd.host_tables([])


def test_config_table_shapes(patterns):
    # C1 6 opcode blocks, C2 8, C3 2, C4 398 states / 110 byte classes (+ dead state here)
    expect = {"c1_lorem": (7, 256), "c2_foobarbaz": (9, 256), "c3_ident": (3, 256), "c4_word": (399, 128)}
    for name, (states, row) in expect.items():
        t = ugrep_amd.host_tables(patterns[name]["opc"])
        assert (t["info"]["states"], t["info"]["row"]) == (states, row), name
    t = ugrep_amd.host_tables(patterns["c4_word"]["opc"])
    # true column-equivalence classes: 99 (the survey counted 110 range-boundary classes)
    assert t["info"]["classes"] <= 110
    t = ugrep_amd.host_tables(patterns["c2_foobarbaz"]["opc"])
    assert 0 < t["info"]["prefilter_ppm"] < 5000  # sparse prefilter: b/f, then a/o, then o/r/z
    assert ugrep_amd.host_tables(patterns["c3_ident"]["opc"])["info"]["prefilter_ppm"] == 0  # dense


def _py_find(t, data):
    trans, cls, caps = t["trans"].tolist(), t["cls"].tolist(), t["caps"].tolist()
    start, accb, fmt = t["start"], t["accb"], t["info"]["format"]
    lr = t["info"]["row"].bit_length() - 1
    n = len(data)
    p, out = 0, []
    while p < n:
        s, q, last, le = start, p, p, 0
        while q < n:
            e = trans[s | data[q]] if fmt == 0 else trans[s + cls[data[q]]]
            if e == 0:
                break
            s = e
            q += 1
            if e >= accb:
                last, le = q, e
        if last > p:
            out.append([p, last - p, caps[le >> lr]])
            p = last
        else:
            p += 1
    return out


def test_host_tables_reproduce_reference_matches(patterns, cases):
    done = 0
    for c in cases:
        if c["input"]["type"] != "hex" or c["pattern"] in UNSUPPORTED | ANCHORED | {"lookahead"}:
            continue  # (anchored tables: the context walk of tests/test_anchor.py; lookahead: tests/test_lookahead.py)
        t = ugrep_amd.host_tables(patterns[c["pattern"]]["opc"])
        data = case_input(c["input"]).tolist()
        assert _py_find(t, data) == c["matches"], (c["pattern"], c["input"]["name"])
        done += 1
    assert done > 200


def _bucket_bits(ft, b):
    return ft[b & 7] & ft[8 + ((b >> 3) & 7)] & ft[16 + (b >> 6)]


def _group_hit(R0, R1, R2):
    """Group g accepts bytes (i, i+1, i+2): B_g bit g, C_g bit 2+g, D_g bit 4+g."""
    return any((R0 >> g) & 1 and (R1 >> (2 + g)) & 1 and (R2 >> (4 + g)) & 1 for g in (0, 1))


def _prefilter_candidates(ft, data):
    """Positions some group accepts, as sparse_kernel.hip computes them (bytes
    past the end pass their tests)."""
    R = [_bucket_bits(ft, b) for b in data] + [0x3F, 0x3F]
    return {i for i in range(len(data)) if _group_hit(R[i], R[i + 1], R[i + 2])}


def test_prefilter_keeps_every_match_start(patterns, cases):
    """The prefilter may pass extra positions but never drops a match start."""
    seen_sparse = set()
    for c in cases:
        if c["pattern"] in UNSUPPORTED or c["matches"] is None or not c["matches"]:
            continue
        enabled, ft = ugrep_amd.host_prefilter(patterns[c["pattern"]]["opc"])
        if not enabled:
            continue
        seen_sparse.add(c["pattern"])
        cand = _prefilter_candidates(ft.tolist(), case_input(c["input"]).tolist())
        starts = [m[0] for m in c["matches"]]
        assert all(s in cand for s in starts), (c["pattern"], c["input"].get("name"))
    assert {"c1_lorem", "c2_foobarbaz", "hello", "the_then", "aa"} <= seen_sparse


def test_prefilter_selectivity_c2():
    """foo|bar|baz: groups {f}{o}{o} and {b}{a}{r,z} are exact on text bytes:
    of all 3-byte strings over printable ASCII + '\\n', exactly foo, bar, baz pass."""
    import itertools, json, os
    opc = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "patterns.json")))["c2_foobarbaz"]["opc"]
    enabled, ft = ugrep_amd.host_prefilter(opc)
    assert enabled
    ft = ft.tolist()
    text = [10] + list(range(0x20, 0x7f))
    R = {b: _bucket_bits(ft, b) for b in text}
    assert all(r < 0x40 for r in R.values())  # bits 6, 7 stay 0 (the kernel's combine relies on it)
    passed = {bytes(t) for t in itertools.product(text, repeat=3) if _group_hit(R[t[0]], R[t[1]], R[t[2]])}
    assert passed == {b"foo", b"bar", b"baz"}


def test_result_struct_layout():
    assert ctypes.sizeof(_lib.Totals) == 48
    assert ctypes.sizeof(_lib.DfaInfo) == 44


def _xt_find(t, x, data):
    """FIND over `data` with the transducer table x, one lookup per byte, the
    way dense_kernel.hip's lockstep loop runs it (no re-reads)."""
    R, start, accb, fmt = t["info"]["row"], t["start"], t["accb"], t["info"]["format"]
    cls, caps, lr = t["cls"].tolist(), t["caps"].tolist(), R.bit_length() - 1
    x = x.tolist()
    m, p, last, le, out = start, 0, 0, 0, []
    for q, b in enumerate(data):
        e = x[(m & ~(R - 1)) + (b if fmt == 0 else cls[b])]
        if e & 1:  # XT_DEAD: emit [p, last), restart at this byte
            if last > p:
                out.append([p, last - p, caps[le >> lr]])
            p = last = q if e & 2 else q + 1
        if e >= accb:
            last, le = q + 1, e & ~(R - 1)
        m = e
    if last > p:  # end of input cuts the walk
        out.append([p, last - p, caps[le >> lr]])
    return out


def test_transducer_reproduces_reference_matches(patterns, cases):
    """Restart-local tables: the one-lookup-per-byte transducer gives the
    reference's match lists (dense_kernel.hip lockstep path)."""
    local = {}
    for name, p in patterns.items():
        if name not in UNSUPPORTED:
            local[name] = ugrep_amd.host_transducer(p["opc"])
    assert local["c3_ident"] is not None and local["c4_word"] is not None
    assert any(v is None for v in local.values())  # backtracking tables exist and are detected
    done = 0
    for c in cases:
        if c["input"]["type"] != "hex" or c["pattern"] in UNSUPPORTED or local.get(c["pattern"]) is None:
            continue
        t = ugrep_amd.host_tables(patterns[c["pattern"]]["opc"])
        data = case_input(c["input"]).tolist()
        assert _xt_find(t, local[c["pattern"]], data) == c["matches"], (c["pattern"], c["input"]["name"])
        done += 1
    assert done > 100


def test_line_goldens_restated(refgold):
    """The line-number rule the ugpu_lines tests check against (1 + newlines
    before the start; -c = distinct lines of the starts) reproduces the
    reference's -n and -c outputs for Hello.java."""
    import os
    data = np.frombuffer(open(os.path.join(os.path.dirname(__file__), "golden", "Hello.java"), "rb").read(), np.uint8)
    nlpos = np.flatnonzero(data == 10)
    for key in ("hello", "hello_wnhS"):
        g = refgold[key]
        lines = 1 + np.searchsorted(nlpos, np.asarray(g["starts"]), side="left")
        assert lines.tolist() == g["lines"]
    assert len(np.unique(1 + np.searchsorted(nlpos, np.asarray(refgold["hello"]["starts"])))) == refgold["hello"]["c_count"]


@pytest.mark.parametrize("pname", ["c3_ident", "digits", "dot"])
def test_immediate_transducer_semantics(patterns, cases, pname):
    """The byte-id table of xi_kernel (tables.hpp 'immediate'): one walk over the
    ids gives count = #START, sum start = sum of START positions and sum len =
    #IN bytes; digest / dcap must equal the oracle's on seeded corpora and on
    the golden small cases.  Non-immediate tables are refused."""
    from oracle_lib import OracleDfa, gen
    from ugrep_amd.matcher import host_immediate
    opc = patterns[pname]["opc"]
    x, sync = host_immediate(opc)
    assert all(x[0, sync] == x[r, sync] for r in range(x.shape[0]))  # a sync byte resets every walk
    assert x[0, sync] & 4 and not x[0, sync] & 3
    M = (1 << 64) - 1
    inputs = [gen(kind, 5, 0, 40000) for kind in (1, 3, 4)]
    inputs += [case_input(c["input"]) for c in cases if c["pattern"] == pname]
    for buf in inputs:
        ids = np.zeros(buf.size, np.uint8)
        s = 0
        for i, b in enumerate(buf.tolist()):
            s = x[s, b]
            ids[i] = s
        st = np.flatnonzero(ids & 1)
        cnt, ss, ln = st.size, int(st.sum()), int(np.count_nonzero(ids & 2))
        o = OracleDfa(opc).find(buf)
        assert (cnt, (31 * ss + ln) & M) == (o[0], o[1])
    for other in ("c2_foobarbaz", "c4_word", "s_plus", "float"):
        assert host_immediate(patterns[other]["opc"]) is None
