"""Lookahead X(?=Y) under option W (ugrep -w): the walk starts only where
at_wb holds (lib/matcher.cpp:107), a TAKE counts only where at_we holds at
the position the TAKE happens (:142, :208) -- before TAIL moves the match end
back to the recorded HEAD position, which is not tested (:157-175).

Expected values are the reference Matcher's with option W
(tests/golden/lookahead_w_cases.json, `make_lookahead_golden.py --word` with
oracle/_ref/ref_harness, mode suffix "W").  CPU: the oracle restatement
(orc_find_w) and the plan.  GPU: the reference's tables and the compiled
ones on wfind_kernel's lookahead walk, whole buffers, three virtual shards
and streams."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa, gen

with open(os.path.join(GOLDEN, "lookahead_w_cases.json")) as _f:
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


def test_fixture_coverage():
    assert len(CASES) >= 19 and all(c["mode"].endswith("W") for c in CASES)
    assert sum(r["count"] for c in CASES for r in c["results"]) > 10000


def test_oracle_matches_reference_w():
    for c in CASES:
        o = OracleDfa(c["opc"])
        assert o.supported, c["pattern"]
        for r in c["results"]:
            got = o.find_w(_input(r["input"]), want_list=r["list"] is not None)
            assert got[:3] == (r["count"], r["digest"], r["dcap"]), (c["pattern"], c["mode"], r["input"])
            if r["list"] is not None:
                assert got[3] == r["list"], (c["pattern"], c["mode"], r["input"])


def test_plan_takes_lookahead_under_w():
    import ugrep_amd as U
    for c in CASES:
        for opc in (c["opc"], U.compile_regex(bytes.fromhex(c["conv"]), reflex=True)):
            info = U.host_plan(opc, word=True)
            assert info["kernel"] == 4 and info["shape"] & U._lib.SHAPE_LOOKAHEAD, c["pattern"]


@pytest.mark.gpu
def test_gpu_lookahead_w_matches_reference():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    n = 0
    for c in CASES:
        for opc in (c["opc"], U.compile_regex(bytes.fromhex(c["conv"]), reflex=True)):
            pat = U.Pattern(opc, word=True)
            for r in c["results"]:
                data = _input(r["input"])
                want = (r["count"], r["digest"], r["dcap"])
                dev = torch.from_numpy(data).to("cuda")
                got = U.find_all(pat, dev, offsets=r["list"] is not None)
                assert (got.count, got.digest, got.dcap) == want, (c["pattern"], c["mode"], r["input"])
                if r["list"] is not None:
                    assert [list(t) for t in got.triples()] == r["list"], (c["pattern"], c["mode"], r["input"])
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
    assert n >= 200
