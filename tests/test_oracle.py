"""CPU: pin the oracle restatement (oracle/restate.c) to the reference.

Every expected value here came from the reference matcher itself (oracle/_ref,
compiled from /root/reference/lib; tests/golden/make_golden.py) or from the
reference's own golden outputs (tests/out/*.out, parsed into refgold.json).
"""
import numpy as np
import pytest

from oracle_lib import OracleDfa, case_input, gen

UNSUPPORTED = set()  # (lookahead is restated since round 6: its cases below, tests/test_lookahead.py)
# restated by orc_find_a (tests/test_anchor.py, tests/test_wordb.py)
ANCHORED = {"anchor_bol", "anchor_eol", "word_boundary"}


def test_unsupported_tables_rejected(patterns):
    for name, p in patterns.items():
        d = OracleDfa(p["opc"])
        assert d.supported == (name not in UNSUPPORTED), name
        assert d.supported is False or d.anchored == (name in ANCHORED), name


def test_refgold_hello_offsets(patterns, refgold):
    """Offsets printed by `ugrep -U -ounkbT` in the reference's tests/out goldens."""
    for pname in ("hello", "hello_wnhS"):
        d = OracleDfa(patterns[pname]["opc"])
        data = case_input(dict(type="file", name=refgold[pname]["file"]))
        _, _, _, lst = d.find(data, want_list=True)
        assert [m[0] for m in lst] == refgold[pname]["starts"]


def test_c1_anchor_64mib(patterns):
    """C1 over lorem tiled to 64 MiB = 14 250 matches, digest 14 823 334 357 500."""
    d = OracleDfa(patterns["c1_lorem"]["opc"])
    data = case_input(dict(type="file", name="lorem.utf8.txt", total=1 << 26))
    cnt, dg, _, _ = d.find(data)
    assert (cnt, dg) == (14250, 14823334357500)


def test_small_cases_full_lists(patterns, cases):
    n = 0
    for c in cases:
        if c.get("big") or c["pattern"] in UNSUPPORTED | ANCHORED:
            continue
        d = OracleDfa(patterns[c["pattern"]]["opc"])
        data = case_input(c["input"])
        want_list = c["matches"] is not None
        cnt, dg, dc, lst = d.find(data, want_list=want_list)
        assert (cnt, dg, dc) == (c["count"], c["digest"], c["dcap"]), (c["pattern"], c["input"].get("name"))
        if want_list:
            assert lst == c["matches"], (c["pattern"], c["input"])
        n += 1
    assert n > 300


@pytest.mark.parametrize("pname,kind", [("c2_foobarbaz", 1), ("c2_foobarbaz", 2), ("c3_ident", 3), ("c4_word", 4)])
def test_big_digests(patterns, cases, pname, kind):
    """64 MiB config digests computed by the reference."""
    c = [c for c in cases if c.get("big") and c["pattern"] == pname and c["input"].get("kind") == kind][0]
    d = OracleDfa(patterns[pname]["opc"])
    cnt, dg, dc, _ = d.find(case_input(c["input"]))
    assert (cnt, dg, dc) == (c["count"], c["digest"], c["dcap"])


def test_planted_known_answer(patterns):
    """C2' corpus: foo|bar|baz matches exactly the planted cells (no oracle needed)."""
    d = OracleDfa(patterns["c2_foobarbaz"]["opc"])
    buf = gen(2, 99, 0, 1 << 22)
    cells = buf.reshape(-1, 64)
    planted = sum(1 for row in cells if (b"foo" in row.tobytes() or b"bar" in row.tobytes() or b"baz" in row.tobytes()))
    cnt, _, _, _ = d.find(buf)
    assert cnt == planted and cnt > 500


def test_newline_split_equals_sequential(patterns):
    """The CPU baseline splits at newlines (ugrep's worker model); exact for these patterns."""
    for pname, kind in (("c2_foobarbaz", 1), ("c3_ident", 3), ("c4_word", 4)):
        d = OracleDfa(patterns[pname]["opc"])
        buf = gen(kind, 5, 0, 1 << 21)
        assert d.find(buf)[:3] == d.find_mt(buf, 7)


def test_generator_cells_are_independent():
    """Any slice of the corpus equals the same range of a larger generation."""
    for kind in (1, 2, 3, 4):
        full = gen(kind, 42, 0, 1 << 16)
        part = gen(kind, 42, 777, 5000)
        assert np.array_equal(full[777:5777], part)


def test_isutf8_restatement_pinned_to_reference():
    """orc_isutf8 (restated scalar loop) and orc_utf8_first_bad (the kernel's
    local rule) both agree with the compiled reference's reflex::isutf8 on every
    golden case (tests/golden/make_utf8_golden.py)."""
    import json
    import os
    import oracle_lib as O
    with open(os.path.join(os.path.dirname(__file__), "golden", "utf8.json")) as f:
        gold = json.load(f)
    assert len(gold["cases"]) > 3000
    for h, ref in gold["cases"]:
        b = bytes.fromhex(h)
        assert O.isutf8(b) == ref, h
        assert (O.utf8_first_bad(b) is None) == ref, h
    for inp in gold["inputs"]:
        assert O.isutf8(case_input(inp)) == inp["isutf8"]


def test_init_window_trim():
    """GrepWorker::init_is_binary's trailing-sequence rule (src/ugrep.cpp:3998-4015)."""
    import oracle_lib as O
    assert O.is_binary(b"", init_window=True) is False
    assert O.is_binary(b"abc\xc3", init_window=True) is False  # cut-off lead ignored
    assert O.is_binary(b"abc\xc3") is True
    assert O.is_binary(b"abc\xe2\x82", init_window=True) is False
    assert O.is_binary(b"ab\x80", init_window=True) is True  # continuation after ASCII
    assert O.is_binary(b"a\x80\x80\x80\x80", init_window=True) is True  # 4 continuations back
    assert O.is_binary(b"\xc3\xa9", init_window=True) is False
    assert O.is_binary(b"a\x00b", nul_only=True) is True
    assert O.is_binary(b"a\xffb", nul_only=True) is False
    assert O.is_binary(b"a\x00b", null_data=True) is False


def test_oracle_long_streams_vs_reference(patterns):
    """The restatement over the 128-512 MiB corpus prefixes of
    tests/golden/streams.json equals the reference matcher's count, digest and
    dcap (pins the fixture the multi-shard GPU tests and bench.py rely on)."""
    import json
    import os
    from oracle_lib import GOLDEN, OracleDfa, gen
    with open(os.path.join(GOLDEN, "streams.json")) as f:
        streams = json.load(f)
    for name, s in streams.items():
        buf = gen(s["kind"], s["seed"], 0, s["bytes"])
        got = OracleDfa(patterns[s["pattern"]]["opc"]).find_mt(buf, 8)
        assert got == (s["count"], s["digest"], s["dcap"]), name
        del buf
