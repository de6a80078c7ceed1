"""CPU: the C-ABI library loads and exports its header, and its host-side table
builder (opcode words -> dense device tables) reproduces the reference's
matches when walked on the CPU with the exact FIND chain."""
import ctypes

import pytest

import ugrep_amd
from ugrep_amd import _lib
from oracle_lib import case_input

UNSUPPORTED = {"anchor_bol", "anchor_eol", "word_boundary", "lookahead"}


def test_exports_every_declared_symbol():
    names = _lib.declared_symbols()
    assert len(names) >= 15
    for n in names:
        assert hasattr(_lib.lib, n), n
    assert ugrep_amd.lib.ugpu_version().startswith(b"ugrep_amd")


def test_unsupported_patterns(patterns):
    for name, p in patterns.items():
        if name in UNSUPPORTED:
            with pytest.raises(ugrep_amd.Unsupported):
                ugrep_amd.host_tables(p["opc"])
        else:
            ugrep_amd.host_tables(p["opc"])


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
    assert t["info"]["needles"] == 1  # first bytes {b, f} = one term (b & 0xfb) == 0x62


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
        if c["input"]["type"] != "hex" or c["pattern"] in UNSUPPORTED:
            continue
        t = ugrep_amd.host_tables(patterns[c["pattern"]]["opc"])
        data = case_input(c["input"]).tolist()
        assert _py_find(t, data) == c["matches"], (c["pattern"], c["input"]["name"])
        done += 1
    assert done > 200


def test_result_struct_layout():
    assert ctypes.sizeof(_lib.Totals) == 48
    assert ctypes.sizeof(_lib.DfaInfo) == 32
