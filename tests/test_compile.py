"""Regex -> opcode compiler (ugpu_compile, ugrep_amd/csrc/regex_compile.cpp)
against the reference's own compiled tables.

The fixture tests/golden/compile_cases.npz holds, per case, the opcode words
the reference Pattern produced (tools/gen_compile_golden.py, libreflex built
from /root/reference; empty = the reference throws regex_error).  Parity is
language equivalence per accept index (tests/dfa_equiv.py), which is exactly
"identical FIND results on every input" (SURVEY Appendix A).  The GPU test
runs compiled tables through the HIP engine and checks every match record
against the oracle restatement driven by the reference's table.
"""
import os

import numpy as np
import pytest

from dfa_equiv import counterexample

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    z = np.load(os.path.join(HERE, "golden", "compile_cases.npz"))
    offs, words = z["offsets"], z["words"]
    out = []
    for i, (mode, pat) in enumerate(zip(z["modes"], z["patterns"])):
        ref = words[offs[i]:offs[i + 1]]
        out.append((str(mode), bytes(pat).decode("utf-8"), ref if len(ref) else None))
    return out


CASES = _cases()


def _compile(U, mode, rx):
    return U.compile_regex(rx, fixed=(mode == "F"), icase=(mode == "i"))


def test_fixture_covers_configs():
    pats = {(m, p) for m, p, _ in CASES}
    for key in (("re", "foo|bar|baz"), ("re", "[A-Za-z_][A-Za-z0-9_]*"), ("re", r"\w+"), ("F", "lorem")):
        assert key in pats
    assert len(CASES) > 200


@pytest.mark.parametrize("chunk", range(4))
def test_compile_equivalent_to_reference(chunk):
    import ugrep_amd as U
    bad = []
    for mode, rx, ref in CASES[chunk::4]:
        if ref is None:
            with pytest.raises(U.UgpuError) as e:
                _compile(U, mode, rx)
            assert not isinstance(e.value, U.Unsupported), (mode, rx)
            continue
        try:
            mine = _compile(U, mode, rx)
        except U.Unsupported as e:
            # documented limitation: \p{Lu}/\p{Ll}/\p{Lt} under -i
            assert mode == "i" and "under -i" in str(e), (mode, rx, e)
            continue
        ce = counterexample(mine, ref)
        if ce is not None:
            bad.append((mode, rx, ce))
    assert not bad, bad[:5]


def _reflex_cases():
    z = np.load(os.path.join(HERE, "golden", "reflex_cases.npz"))
    offs, words, ro, rx = z["offsets"], z["words"], z["roffsets"], z["regex"]
    return [(str(m), bytes(rx[ro[i]:ro[i + 1]]), words[offs[i]:offs[i + 1]]) for i, m in enumerate(z["modes"])]


REFLEX_CASES = _reflex_cases()


@pytest.mark.parametrize("chunk", range(4))
def test_reflex_mode_equivalent_to_reference(chunk):
    """UGPU_RX_REFLEX: the converted regex the reference Pattern holds (its public
    Pattern::operator[](0); tests/golden/reflex_cases.npz, tools/gen_reflex_golden.py)
    compiles to a table language-equivalent to the reference's own, for every
    case of compile_cases.npz the reference accepts (Unicode classes, -i, -F
    quoting, inline modifiers).  This is how the drop-in adapter builds its tables."""
    import ugrep_amd as U
    bad, unsup = [], []
    for mode, conv, ref in REFLEX_CASES[chunk::4]:
        try:
            mine = U.compile_regex(conv, reflex=True)
        except U.Unsupported as e:
            unsup.append((mode, conv[:60], str(e)))
            continue
        ce = counterexample(mine, ref)
        if ce is not None:
            bad.append((mode, conv[:80], ce))
    assert not bad, bad[:5]
    assert not unsup, unsup[:5]


def test_reflex_mode_rejects_meta():
    import ugrep_amd as U
    # ^ / $ are supported as the leading / trailing anchor of a top-level
    # alternative under (?m) (tests/test_anchor.py); without (?m) ^ would be the
    # buffer begin, and inside groups the reference keeps meta edges that go on
    # consuming bytes (word boundaries likewise: at the ends of top-level
    # alternatives only, tests/test_wordb.py)
    for rx in (b"^a", b"(?m)x(^a)", b"(?m)a$b", b"(?m)(a$)b", b"(?m)a\\bfoo", b"(?m)(\\bfoo)+", b"(?m)x*?y", b"(?m)(?!x)y", b"(?mx)a b", b"(?m)\\x{100}"):
        with pytest.raises(U.Unsupported):
            U.compile_regex(rx, reflex=True)
    # (round 6: a group at an alternative's start or end with the anchors at
    # its own ends is distributed, tests/test_asgroup.py)
    for rx in (b"(?m)(^a)", b"(?m)(a$)", b"(?m)(\\bfoo)"):
        U.compile_regex(rx, reflex=True)


def test_config_tables_are_loadable():
    """Compiled tables pass the device-table builder (host side) and pick the
    same kernel class as the reference's tables for the BASELINE configs."""
    import ugrep_amd as U
    ref = {(m, p): r for m, p, r in CASES}
    for mode, rx in (("re", "foo|bar|baz"), ("re", "[A-Za-z_][A-Za-z0-9_]*"), ("re", r"\w+"), ("F", "lorem")):
        a = U.host_tables(_compile(U, mode, rx))["info"]
        b = U.host_tables(ref[(mode, rx)])["info"]
        assert a["kernel"] == b["kernel"], (rx, a, b)
        assert a["states"] <= b["states"]


@pytest.mark.parametrize("rx", ["x(^a)", "a$b", "a^", r"a\bfoo", r"x(\<x)", r"\b+x", "a*?", "a+?", r"(a)\1", r"\p{NoSuchScript}", "[[:^alpha:]]",
                                "(?!x)", r"\Qa\E", r"\p{Lu}"])
def test_unsupported_constructs(rx):
    import ugrep_amd as U
    with pytest.raises(U.Unsupported):
        U.compile_regex(rx, icase=(rx == r"\p{Lu}"))


def test_long_gotos():
    """Tables past 0xFFFE words use LONG gotos (lib/pattern.cpp:2877-2939) and
    stay equivalent: a large alternation of distinct words."""
    import ugrep_amd as U
    import random
    rng = random.Random(5)
    words = sorted({"".join(rng.choice("abcdefghij") for _ in range(10)) for _ in range(5000)})
    opc = U.compile_regex("|".join(words))
    assert len(opc) > 0xFFFE
    assert any((w & 0xFFFF) == 0xFFFE for w in opc[:64])
    from dfa_equiv import _parse_opc
    nxt, caps = _parse_opc(opc)
    # walk each word: accepts with its 1-based alternative index
    for k in (0, 1, len(words) // 2, len(words) - 1):
        s = 1
        for ch in words[k].encode():
            s = nxt[s][ch]
        assert caps[s] == k + 1


@pytest.mark.gpu
def test_compiled_tables_on_gpu():
    """Compiled tables through the HIP engine == the oracle driven by the
    reference's tables, record by record, on a mixed UTF-8/code corpus."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    from oracle_lib import OracleDfa, gen
    host = np.concatenate([gen(4, 7, 0, 384 << 10), gen(3, 7, 0, 384 << 10), gen(1, 7, 0, 256 << 10)])
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    checked = 0
    for mode, rx, ref in CASES[::3]:
        if ref is None:
            continue
        try:
            pat = U.Pattern(_compile(U, mode, rx))
            res = U.find_all(pat, dev, offsets=True)
        except U.Unsupported:
            continue  # table too large for the 16-bit device tables or for LDS
        cnt, dg, dc, lst = OracleDfa(ref).find(host, want_list=True)
        assert (res.count, res.digest, res.dcap) == (cnt, dg, dc), (mode, rx)
        assert res.triples() == lst, (mode, rx)
        checked += 1
    assert checked > 40


@pytest.mark.gpu
def test_rare_sync_bytes_long_tails():
    """Patterns with rare sync bytes over UTF-8 words without digits: \\D
    (sync bytes = digits only; the host sends it to dense_kernel) and
    [^0-9]+ (xg_kernel, newline sync bytes, long tails summed in 64 bits per
    chunk).  Whole-buffer totals == oracle."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd as U
    from oracle_lib import OracleDfa, gen
    host = gen(4, 11, 0, 48 << 20)
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    # (\D\D is correct but pathological for dense_kernel: two never-converging
    # match phases make fix_kernel re-walk record by record)
    for rx in (r"\D", r"[^0-9]+"):
        opc = U.compile_regex(rx)
        pat = U.Pattern(opc)
        res = U.find_all(pat, dev)
        assert (res.count, res.digest, res.dcap) == OracleDfa(opc).find(host)[:3], rx
