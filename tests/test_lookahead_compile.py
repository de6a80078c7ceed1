"""Lookahead in the native compiler (ugpu_compile, regex_compile.cpp
Parser::lookahead_group): X(?=Y) compiled with HEAD/TAIL markers where the
reference's Pattern places them (lib/pattern.cpp:1331-1359, :2374-2419) and
emitted as TAIL la / HEAD la words (:2953-2964), so that the drop-in adapter,
which recompiles ugrep's converted regex, sends lookahead patterns to the GPU.

Expected values are the reference's (tests/golden/lookahead_compile.json,
written by tests/golden/make_lookahead_compile_golden.py with
oracle/_ref/ref_harness): its opcode words and its Matcher's FIND over an edge
text, for 33 patterns -- nullable prefixes and lookaheads, lookahead inside
repeats and alternatives, text after the lookahead, Unicode mode, and the
shapes the compiler refuses.

CPU: the compiled table is equivalent to the reference's, states' TAIL/HEAD
words included (tables_equivalent), and the oracle walking it reproduces the
reference's match list.  Tables whose start state records a HEAD that some TAIL
reads can end in an empty match, where the reference's FIND asks its advance
function (lib/matcher.cpp:682-707): the table builder refuses them.  GPU: the
compiled tables and the reference's own give the reference's list."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa

with open(os.path.join(GOLDEN, "lookahead_compile.json")) as _f:
    SPEC = json.load(_f)
CASES = SPEC["cases"]
EDGE = np.frombuffer(bytes.fromhex(SPEC["edge_hex"]), np.uint8).copy()
# the compiler refuses these (nested / adjacent lookaheads: the reference
# merges their ranges into one index; lookahead with anchors or word boundaries)
REFUSED = {r"a(?=b(?=c))", r"a(?=b)(?=c)", r"^a(?=b)", r"a(?=b)$", r"\ba(?=b)", r"[a-z]+(?=ing|s\b)"}
# the table builder refuses these (an empty match is possible)
EMPTY_MATCH = {r"(?=x)", r"a*(?=b)"}


def _conv(c):
    return bytes.fromhex(c["conv"])


def test_fixture():
    assert len(CASES) >= 30
    assert sum(1 for c in CASES if c["opc"] is not None) >= 30
    assert sum(c["count"] for c in CASES if c["opc"] is not None) > 100


def test_compiled_tables_equal_reference():
    import ugrep_amd as U
    from ugrep_amd.matcher import host_equivalent
    done = 0
    for c in CASES:
        if c["opc"] is None:
            continue
        if c["pattern"] in REFUSED:
            with pytest.raises(U.Unsupported):
                U.compile_regex(_conv(c), reflex=True)
            continue
        mine = U.compile_regex(_conv(c), reflex=True)
        assert any((w >> 24) in (0xFB, 0xFC) for w in mine), c["pattern"]
        if c["pattern"] in EMPTY_MATCH:
            for opc in (mine, c["opc"]):
                with pytest.raises(U.Unsupported):
                    U.host_tables(opc)
            continue
        assert host_equivalent(mine, c["opc"]), c["pattern"]
        cnt, dg, dc, lst = OracleDfa(mine).find(EDGE, want_list=True)
        assert (cnt, dg, dc) == (c["count"], c["digest"], c["dcap"]), c["pattern"]
        assert lst == c["list"], c["pattern"]
        done += 1
    assert done >= 24


def test_equivalence_sees_lookahead_words():
    """A table that differs only in its TAIL/HEAD words is not equivalent."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_equivalent
    m = U.compile_regex("(?m)foo(?=bar)", reflex=True)
    assert host_equivalent(m, [(0xFB000001 if (w >> 24) == 0xFC else w) for w in m]) is False
    assert host_equivalent(m, [(0xFC000000 if (w >> 24) == 0xFB else w) for w in m]) is False


def test_ere_mode_and_refusals():
    import ugrep_amd as U
    from ugrep_amd.matcher import host_equivalent
    ref = next(c for c in CASES if c["pattern"] == "foo(?=bar)|foo") if any(
        c["pattern"] == "foo(?=bar)|foo" for c in CASES) else None
    assert ref is not None
    assert host_equivalent(U.compile_regex("foo(?=bar)|foo"), ref["opc"])
    for rx in ("a(?=)", "(?!x)y", "a(?=b(?=c))", "a(?=b)(?=c)"):
        with pytest.raises((U.Unsupported, U.UgpuError)):
            U.compile_regex(rx)


def test_plan_takes_compiled_lookahead():
    import ugrep_amd as U
    for c in CASES:
        if c["opc"] is None or c["pattern"] in REFUSED | EMPTY_MATCH:
            continue
        info = U.host_plan(U.compile_regex(_conv(c), reflex=True))
        assert info["kernel"] == 4 and info["shape"] & U._lib.SHAPE_LOOKAHEAD, c["pattern"]


@pytest.mark.gpu
def test_gpu_compiled_and_reference_tables():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    dev = torch.zeros(EDGE.size + 64, dtype=torch.uint8, device="cuda")
    dev[:EDGE.size].copy_(torch.from_numpy(EDGE))
    dev = dev[:EDGE.size]
    done = 0
    for c in CASES:
        if c["opc"] is None or c["pattern"] in EMPTY_MATCH:
            continue
        tabs = [c["opc"]] + ([] if c["pattern"] in REFUSED else [U.compile_regex(_conv(c), reflex=True)])
        for opc in tabs:
            try:
                pat = U.Pattern(opc)
            except U.Unsupported:
                assert c["pattern"] in REFUSED, c["pattern"]  # (anchors, word boundaries)
                continue
            got = U.find_all(pat, dev, offsets=True)
            assert (got.count, got.digest, got.dcap) == (c["count"], c["digest"], c["dcap"]), c["pattern"]
            assert [list(t) for t in got.triples()] == c["list"], c["pattern"]
            done += 1
    assert done >= 50
