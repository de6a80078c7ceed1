"""Negative patterns: REDO accepts (ugrep -N PATTERN, wrapped as (?^PATTERN),
src/ugrep.cpp:6487, src/cnf.cpp:503).

The reference's Pattern marks a DFA state REDO when it holds a negated accept
(lib/pattern.cpp:2358-2363, opcode 0xFD000000 at :2945-2947).  The FIND walk
takes REDO like a TAKE -- the last accept wins (lib/matcher.cpp:151-156,
:218-225) -- and a match whose last accept is REDO is not reported: the search
resumes at its end (:732-738).  The engine keeps the accept index kCapRedo for
such states (ugrep_amd/csrc/ctx_bits.hpp); every emitter skips it.

Expected values are the reference Matcher's (tests/golden/redo_cases.json,
written by tests/golden/make_redo_golden.py with oracle/_ref/ref_harness).
CPU: the oracle restatement reproduces them; the native compiler's tables for
the converted regex are equivalent to the reference's.  GPU: whole-buffer
FIND (sparse, dense and wfind_kernel tables), shards, streams and OFFSETS."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa, gen

with open(os.path.join(GOLDEN, "redo_cases.json")) as _f:
    SPEC = json.load(_f)
CASES = SPEC["cases"]
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


def _has_redo(opc):
    return any(w == 0xFD000000 for w in opc)


def test_fixture_coverage():
    assert len(CASES) >= 12
    assert all(_has_redo(c["opc"]) for c in CASES)
    # some match is stepped over: the reference reports fewer matches than the
    # same pattern without its negative alternatives would
    assert any(r["list"] for c in CASES for r in c["results"])


def test_oracle_matches_reference():
    for c in CASES:
        o = OracleDfa(c["opc"])
        assert o.supported, c["pattern"]
        for r in c["results"]:
            cnt, dg, dc, lst = o.find(_input(r["input"]), want_list=r["list"] is not None)
            assert (cnt, dg, dc) == (r["count"], r["digest"], r["dcap"]), (c["pattern"], r["input"])
            if r["list"] is not None:
                assert lst == r["list"], (c["pattern"], r["input"])


def test_compiler_negative_patterns_equivalent():
    """ugpu_compile on the converted regex (the drop-in adapter's input,
    UGPU_RX_REFLEX): tables equivalent to the reference's, REDO included
    (ugpu_tables_equivalent_host compares accept indices, REDO being one)."""
    import ugrep_amd as U
    from ugrep_amd.matcher import host_equivalent
    for c in CASES:
        opc = U.compile_regex(bytes.fromhex(c["conv"]), reflex=True)
        assert _has_redo(opc), c["pattern"]
        assert host_equivalent(opc, c["opc"]), c["pattern"]
        r = next(r for r in c["results"] if r["input"] == "edge")
        assert OracleDfa(opc).find(_input("edge"), want_list=True)[3] == r["list"], c["pattern"]


def test_plan_and_refusals():
    """REDO tables have no single accept index (no transducer, carry-chain or
    code-point-run kernel, 16-byte records); empty matches under option N are
    refused (the CPU matcher keeps them); a negative pattern
    inside a sequence or a group is refused by the compiler."""
    import ugrep_amd as U
    kernels = set()
    for c in CASES:
        info = U.host_plan(c["opc"])
        kernels.add(info["kernel"])
        assert info["kernel"] in (0, 1, 4), (c["pattern"], info)
        assert not info["shape"] & U._lib.SHAPE_ONE_ACCEPT
        # (option W: since round 6 on the W walks, tests/test_redo_w.py)
        assert U.host_plan(c["opc"], word=True)["kernel"] in (0, 4), c["pattern"]
    assert {0, 1} <= kernels  # (both the prefiltered and the dense path are covered)
    for rx in (r"x(?^foo)|f\w+", r"(a(?^b))", r"(?^foo)|^bar", r"(?^a)|\bb"):
        with pytest.raises(U.Unsupported):
            U.compile_regex(rx)


# ---- GPU
def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return torch


@pytest.mark.gpu
def test_gpu_redo_matches_reference():
    """Every case and input, reference tables and compiled ones: totals and
    match lists (OFFSETS) equal the reference's; three virtual shards and a
    stream of 997-byte chunks give the same totals."""
    torch = _torch()
    import ugrep_amd as U
    n = 0
    for c in CASES:
        for opc in (c["opc"], U.compile_regex(bytes.fromhex(c["conv"]), reflex=True)):
            pat = U.Pattern(opc)
            for r in c["results"]:
                data = _input(r["input"])
                want = (r["count"], r["digest"], r["dcap"])
                dev = torch.from_numpy(data).to("cuda")
                torch.cuda.synchronize()
                got = U.find_all(pat, dev, offsets=r["list"] is not None)
                assert (got.count, got.digest, got.dcap) == want, (c["pattern"], r["input"])
                if r["list"] is not None:
                    assert [list(t) for t in got.triples()] == r["list"], (c["pattern"], r["input"])
                m = U.find_all_multi(pat, data, ndev=3, offsets=False)
                assert (m.count, m.digest, m.dcap) == want, ("multi", c["pattern"], r["input"])
                if r["input"] in ("edge", "Hello.java"):
                    st = U.Stream(pat)
                    cnt = dg = dc = 0
                    for k in range(0, len(data), 997):
                        res = st.feed(data[k:k + 997], final=k + 997 >= len(data))
                        cnt += res.count
                        dg = (dg + res.digest) & ((1 << 64) - 1)
                        dc = (dc + res.dcap) & ((1 << 64) - 1)
                    assert (cnt, dg, dc) == want, ("stream", c["pattern"], r["input"])
                n += 1
    assert n >= 150


@pytest.mark.gpu
def test_gpu_redo_large_against_oracle():
    """8 MiB of mixed corpora: totals and record lists against the oracle (which
    the fixtures pin), for every case on its own kernel and, for the
    prefiltered ones, on the dense kernel too (UGPU_SPARSE=0)."""
    torch = _torch()
    import ugrep_amd as U
    parts = [gen(1, 9, 0, 1 << 20), gen(3, 9, 0, 1 << 20), gen(4, 9, 0, 1 << 20), np.tile(_input("edge"), 3000)]
    data = np.ascontiguousarray(np.concatenate(parts * 3)[:8 << 20])
    dev = torch.from_numpy(data).to("cuda")
    torch.cuda.synchronize()
    for c in CASES:
        o = OracleDfa(c["opc"])
        ws, wl, wc = o.find_arrays(data)
        cnt, dg, dc, _ = o.find(data)
        pat = U.Pattern(c["opc"])
        got = U.find_all(pat, dev, offsets=True)
        assert (got.count, got.digest, got.dcap) == (cnt, dg, dc), c["pattern"]
        assert np.array_equal(np.asarray(got.start, np.uint64), ws), c["pattern"]
        assert np.array_equal(np.asarray(got.length, np.uint64), wl), c["pattern"]
        assert np.array_equal(np.asarray(got.cap, np.uint64), wc), c["pattern"]
        if pat.info()["kernel"] == 0:
            os.environ["UGPU_SPARSE"] = "0"
            try:
                g2 = U.find_all(U.Pattern(c["opc"]), dev, offsets=False)
            finally:
                os.environ.pop("UGPU_SPARSE", None)
            assert (g2.count, g2.digest, g2.dcap) == (cnt, dg, dc), ("dense", c["pattern"])
