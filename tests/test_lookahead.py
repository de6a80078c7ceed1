"""Lookahead (X(?=Y)) on the GPU: HEAD/TAIL words (lib/pattern.cpp:2953-2964).

The reference's FIND walk runs each state's block on entry: TAKE (the match
would end here), then TAIL la (the match end moves back to where HEAD la was
recorded in this walk), then HEAD la (record the position); the records are
cleared per walk (lib/matcher.cpp:104, :139-175, :226-237).  The engine keeps
each state's TAIL/HEAD masks (tables.hpp look) and walks such tables with the
lookahead walk (device_common.hpp kWalkLook) on wfind_kernel, with the same
stitching, shards, streams and OFFSETS as every other table.

Expected values are the reference Matcher's (tests/golden/lookahead_cases.json,
written by tests/golden/make_lookahead_golden.py with oracle/_ref/ref_harness).
CPU: the oracle restatement reproduces them; the plan routes the tables to the
lookahead walk.  GPU: whole buffers, scans that start mid-buffer, shards, a
stream fed in ragged chunks, OFFSETS, record by record."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa, gen

with open(os.path.join(GOLDEN, "lookahead_cases.json")) as _f:
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


def _has_lookahead(opc):
    return any((w >> 24) in (0xFB, 0xFC) for w in opc)


def test_fixture_coverage():
    assert len(CASES) >= 12
    assert all(_has_lookahead(c["opc"]) for c in CASES)
    assert sum(r["count"] for c in CASES for r in c["results"]) > 10000


def test_oracle_matches_reference():
    for c in CASES:
        o = OracleDfa(c["opc"])
        assert o.supported, c["pattern"]
        for r in c["results"]:
            cnt, dg, dc, lst = o.find(_input(r["input"]), want_list=r["list"] is not None)
            assert (cnt, dg, dc) == (r["count"], r["digest"], r["dcap"]), (c["pattern"], r["input"])
            if r["list"] is not None:
                assert lst == r["list"], (c["pattern"], r["input"])


def test_plan_routes_to_the_lookahead_walk():
    import ugrep_amd as U
    for c in CASES:
        info = U.host_plan(c["opc"])
        assert info["kernel"] == 4, c["pattern"]  # wfind_kernel (kWalkLook)
        assert info["shape"] & U._lib.SHAPE_LOOKAHEAD, c["pattern"]
    # lookahead with anchors or a negative pattern stays on the CPU (option W
    # runs since round 6: tests/test_lookahead_w.py)
    for rx in (r"^foo(?=bar)", r"(?^x)|foo(?=bar)"):
        try:
            opc = U.compile_regex(rx)
        except U.Unsupported:
            continue
        with pytest.raises(U.Unsupported):
            U.host_plan(opc)
    assert U.host_plan(CASES[0]["opc"], word=True)["kernel"] == 4


# ----------------------------------------------------------------- GPU


@pytest.fixture(scope="module")
def U():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _dev(arr):
    import torch
    t = torch.zeros(arr.size + 64, dtype=torch.uint8, device="cuda")
    t[:arr.size].copy_(torch.from_numpy(np.ascontiguousarray(arr)))
    torch.cuda.synchronize()
    return t[:arr.size]


@pytest.mark.gpu
def test_gpu_against_reference(U):
    for c in CASES:
        pat = U.Pattern(c["opc"])
        assert pat.info()["kernel"] == 4, c["pattern"]
        for r in c["results"]:
            data = _input(r["input"])
            dev = _dev(data)
            got = U.find_all(pat, dev, offsets=r["list"] is not None)
            assert (got.count, got.digest, got.dcap) == (r["count"], r["digest"], r["dcap"]), (c["pattern"], r["input"])
            if r["list"] is not None:
                assert [list(t) for t in got.triples()] == r["list"], (c["pattern"], r["input"])


@pytest.mark.gpu
def test_gpu_large_starts_shards_streams(U):
    """8 MiB of the C3 corpus: whole buffer, a scan from an odd start, 3-way
    shards, OFFSETS and a ragged stream, all equal to the oracle."""
    data = gen(3, 9, 0, 8 << 20)
    dev = _dev(data)
    for c in CASES:
        o = OracleDfa(c["opc"])
        pat = U.Pattern(c["opc"])
        cnt, dg, dc, lst = o.find(data, want_list=True)
        got = U.find_all(pat, dev, offsets=True)
        assert (got.count, got.digest, got.dcap) == (cnt, dg, dc), c["pattern"]
        assert [list(t) for t in got.triples()] == lst, c["pattern"]
        st = 12345
        w = o.find(data, start=st)
        g2 = U.find_all(pat, dev, start=st, offsets=False)
        assert (g2.count, g2.digest, g2.dcap) == w[:3], c["pattern"]
        m = U.find_all_multi(pat, data, ndev=3, offsets=False)
        assert (m.count, m.digest, m.dcap) == (cnt, dg, dc), c["pattern"]
        s = U.Stream(pat)
        rng = np.random.default_rng(3)
        pos, recs = 0, []
        while pos < data.size:
            k = int(rng.integers(1, 1 << 20))
            chunk = data[pos:pos + k]
            pos += chunk.size
            r = s.feed(chunk, final=pos >= data.size)
            recs.extend(list(t) for t in r.triples())
        s.close()
        assert recs == lst, c["pattern"]
