"""Line anchors and word boundaries inside a group at the start or the end of
a top-level alternative: (^|,)foo, foo($|,), (\\bfoo|bar), ((^|,)foo|bar).

The native compiler distributes such a group over its alternative
((^|,)foo -> ^foo|,foo, each copy with the alternative's accept index;
ugrep_amd/csrc/regex_compile.cpp rx_assertion_groups), so the assertions end
up at the ends of top-level alternatives, where the per-context accepts hold
them.  Expected values are the reference's
(tests/golden/asgroup_cases.json, written by
tests/golden/make_asgroup_golden.py with oracle/_ref/ref_harness): the match
lists with its match predictor off (the DFA semantics).

CPU: the compiled tables (the ugrep-converted regex in RE/flex mode, and the
pattern in ERE mode) reproduce the reference's lists, accept indices included
(dcap), through the oracle; groups with assertions elsewhere stay refused.
GPU: whole-buffer FIND, shards and streams reproduce them."""
import json
import os

import numpy as np
import pytest

from oracle_lib import GOLDEN, OracleDfa

with open(os.path.join(GOLDEN, "asgroup_cases.json")) as _f:
    SPEC = json.load(_f)
CASES = SPEC["cases"]
_INPUTS = {}
# a begin anchor in a group with \s or $ in a trailing one: the reference
# moves ^ to the accept side, where its EOL edge (which holds before "\r\n")
# ends the match before \s could take the '\r' (the edge text's "\nfoo\r\n":
# 3 bytes, where ^foo\s|^foo$ takes 4) -- refused by the distribution, the
# CPU matcher keeps it
REFUSED = {r"(^|\s)foo(\s|$)"}


def _input(name):
    if name not in _INPUTS:
        if name == "edge":
            _INPUTS[name] = np.frombuffer(bytes.fromhex(SPEC["meta"]["edge_hex"]), np.uint8).copy()
        else:
            spec = next(i["spec"] for i in SPEC["meta"]["inputs"] if i["name"] == name)
            path = spec[5:]
            if not os.path.isabs(path):
                path = os.path.join(os.path.dirname(os.path.dirname(GOLDEN)), path)
            _INPUTS[name] = np.frombuffer(open(path, "rb").read(), np.uint8).copy()
    return _INPUTS[name]


def _forms(c):
    return [("reflex", bytes.fromhex(c["conv"])), ("ere", c["pattern"])]


def test_fixture_coverage():
    assert len(CASES) >= 25
    assert sum(r["count"] for c in CASES for r in c["results"]) > 1000
    assert any("^" in c["pattern"] for c in CASES) and any("$" in c["pattern"] for c in CASES)
    assert any("\\b" in c["pattern"] for c in CASES) and any("\\<" in c["pattern"] for c in CASES)


def test_compiler_distributes_assertion_groups():
    import ugrep_amd as U
    n = 0
    for c in CASES:
        for form, rx in _forms(c):
            if c["pattern"] in REFUSED:
                with pytest.raises(U.Unsupported):
                    U.compile_regex(rx, reflex=form == "reflex")
                continue
            opc = U.compile_regex(rx, reflex=form == "reflex")
            o = OracleDfa(opc)
            assert o.supported, (c["pattern"], form)
            for r in c["results"]:
                got = o.find(_input(r["input"]), want_list=True)
                assert got[:3] == (r["count"], r["digest"], r["dcap"]), (c["pattern"], form, r["input"])
                assert got[3] == r["list"], (c["pattern"], form, r["input"])
                n += 1
    assert n >= 150


def test_compiler_refuses_other_interior_assertions():
    import ugrep_amd as U
    for rx in ["x(^|,)foo", "(^|,)+foo", "(a)(^|,)", "(foo($|,)|bar)x", "a\\bb", "foo(\\b|x)y", "(?i:(^|,)foo)"]:
        with pytest.raises(U.Unsupported):
            U.compile_regex(rx)


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return torch


@pytest.mark.gpu
def test_gpu_assertion_groups_match_reference():
    torch = _torch()
    import ugrep_amd as U
    n = 0
    for c in CASES:
        if c["pattern"] in REFUSED:
            continue
        opc = U.compile_regex(bytes.fromhex(c["conv"]), reflex=True)
        pat = U.Pattern(opc)
        for r in c["results"]:
            data = _input(r["input"])
            want = (r["count"], r["digest"], r["dcap"])
            dev = torch.from_numpy(data).to("cuda")
            got = U.find_all(pat, dev, offsets=True)
            assert (got.count, got.digest, got.dcap) == want, (c["pattern"], r["input"])
            assert [list(t) for t in got.triples()] == r["list"], (c["pattern"], r["input"])
            got = U.find_all_multi(pat, data, ndev=3, offsets=False)
            assert (got.count, got.digest, got.dcap) == want, ("multi", c["pattern"], r["input"])
            st = U.Stream(pat)
            cnt = dg = dc = 0
            for k in range(0, len(data), 333):
                res = st.feed(data[k:k + 333], final=k + 333 >= len(data))
                cnt += res.count
                dg = (dg + res.digest) & ((1 << 64) - 1)
                dc = (dc + res.dcap) & ((1 << 64) - 1)
            assert (cnt, dg, dc) == want, ("stream", c["pattern"], r["input"])
            n += 1
    assert n >= 80
