"""GPU: xg_kernel, the FIND kernel of restart-local tables with state-determined
walk gaps (UTF-8 word patterns: \\w+ = BASELINE C4, \\S+, [^ \\t]+;
ugrep_amd/csrc/xg_kernel.hip), against the oracle restatement on ranges
[lo, hi) of the chain (counts, digests, exit).  Same lane/tile/edge scheme as
xi_kernel (tests/test_xi.py), so the same kinds of cases: missing sync bytes
for more than a segment or a tile, sync bytes on segment borders, ranges cut
inside matches, moved wave borders; plus UTF-8 specific ones (multi-byte word
and non-word characters around segment borders, random bytes)."""
import os

import numpy as np
import pytest

from test_xi import U, _dev, _oracle_range, _scan  # noqa: F401  (fixtures and helpers)

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GAP = ("c4_word", "s_plus", "nonspace")


@pytest.fixture(scope="module", autouse=True)
def _no_xu():
    """These tables are also code-point run tables (xc_kernel U mode, tests/test_xu.py);
    here they run xg_kernel."""
    os.environ["UGPU_XU"] = "0"
    yield
    os.environ.pop("UGPU_XU", None)


@pytest.fixture(scope="module")
def gpats(U, patterns, _no_xu):  # noqa: F811
    return {k: U.Pattern(patterns[k]["opc"]) for k in GAP}


def _inputs():
    from oracle_lib import gen
    n = 3 << 20
    out = {"utf8": gen(4, 41, 0, n), "code": gen(3, 42, 0, n), "words": gen(1, 43, 0, n)}
    b = gen(4, 44, 0, n)
    for pos, ln in ((5000, 3000), (1 << 20, 70000), ((2 << 20) - 7, 1500)):
        b[pos:pos + ln] = np.frombuffer(("é" * (ln // 2) + "x" * (ln % 2)).encode(), np.uint8)[:ln]
    out["long_words"] = b
    out["all_word"] = np.frombuffer(("Ωx" * (1 << 19)).encode(), np.uint8)[:1 << 20].copy()
    c = np.frombuffer(("€ab" * 400000).encode(), np.uint8)[:1 << 20].copy()  # non-word 3-byte chars
    c[1023::1024] = ord(" ")
    out["euro_border"] = c
    rng = np.random.default_rng(7)
    out["random"] = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    return out


@pytest.fixture(scope="module")
def ginputs():
    return _inputs()


@pytest.mark.parametrize("pname", GAP)
def test_kernel_choice(U, gpats, pname):  # noqa: F811
    assert gpats[pname].info()["kernel"] == 3


@pytest.mark.parametrize("pname", GAP)
def test_ranges_against_oracle(U, gpats, patterns, ginputs, pname):  # noqa: F811
    rng = np.random.default_rng(sum(pname.encode()))
    opc = patterns[pname]["opc"]
    for name, host in ginputs.items():
        n = host.size
        t = _dev(host)
        ranges = [(0, n), (0, 1), (1, 2), (0, 65536), (65536, 131072), (1000, 65536 * 3 + 5), (n - 70000, n)]
        for _ in range(2):
            lo = int(rng.integers(0, n))
            hi = int(rng.integers(lo, min(n, lo + int(rng.choice([100, 5000, 200000, 2 << 20]))) + 1))
            ranges.append((lo, hi))
        for lo, hi in ranges:
            got = _scan(U, gpats[pname], t, lo, hi, n)
            want = _oracle_range(opc, host, lo, hi)
            assert got == want, (pname, name, lo, hi, got, want)


def test_grid_moves_wave_borders(U, gpats, patterns, ginputs):  # noqa: F811
    for name in ("utf8", "long_words", "euro_border", "all_word"):
        host = ginputs[name]
        t = _dev(host)
        want = _oracle_range(patterns["c4_word"]["opc"], host, 0, host.size)
        for g in ("1", "3", "37", ""):
            if g:
                os.environ["UGPU_MAX_GRID"] = g
            else:
                os.environ.pop("UGPU_MAX_GRID", None)
            try:
                got = _scan(U, gpats["c4_word"], t, 0, host.size, host.size)
            finally:
                os.environ.pop("UGPU_MAX_GRID", None)
            assert got == want, (name, g)


def test_agrees_with_dense_kernel_256mib(U, gpats):  # noqa: F811
    n = 256 << 20
    t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    U.gen(4, 51, 0, t.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    res = []
    for xg in ("1", "0"):
        os.environ["UGPU_XG"] = xg
        try:
            res.append(_scan(U, gpats["c4_word"], t, 0, n, n))
            res.append(_scan(U, gpats["c4_word"], t, 777, n - 12345, n))
        finally:
            os.environ.pop("UGPU_XG", None)
    assert res[0] == res[2] and res[1] == res[3], res
