"""GPU: single-pass OFFSETS for prefiltered tables (sparse_kernel stages each
wave's records during the COUNT pass; stage_copy_kernel moves the records of
waves whose speculative chain was the true one, a WRITE pass the others).

Cases: the C2 corpus (all waves copied), matches planted across every wave
border of a small grid (re-entered waves go to the WRITE pass), a dense stretch
that overflows a wave's 1024 staging slots, and the staged and unstaged paths
against each other and the oracle, record by record."""
import os

import numpy as np
import pytest

from oracle_lib import OracleDfa, gen

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def U():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _records(U, pat, dev, n, stage, grid=None):
    st = torch.cuda.current_stream().cuda_stream
    if grid:
        os.environ["UGPU_MAX_GRID"] = str(grid)
    try:
        sc = U.Scanner(pat)
    finally:
        os.environ.pop("UGPU_MAX_GRID", None)
    sc.stage(stage)
    sc.scan(dev.data_ptr(), 0, n, n, True, 0, st)
    t = sc.totals()
    cnt = t.count
    s = torch.empty(max(cnt, 1), dtype=torch.int64, device="cuda")
    ln = torch.empty(max(cnt, 1), dtype=torch.int32, device="cuda")
    cp = torch.empty(max(cnt, 1), dtype=torch.int32, device="cuda")
    sc.offsets(s.data_ptr(), ln.data_ptr(), cp.data_ptr(), cnt, st)
    torch.cuda.synchronize()
    return list(zip(s[:cnt].cpu().tolist(), ln[:cnt].cpu().tolist(), cp[:cnt].cpu().tolist()))


def _check(U, opc, host, grid=None):
    pat = U.Pattern(opc)
    assert pat.info()["kernel"] == 0  # sparse_kernel
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    want = [tuple(r) for r in OracleDfa(opc).find(host, want_list=True)[3]]
    got = _records(U, pat, dev, host.size, True, grid)
    assert got == want
    assert _records(U, pat, dev, host.size, False, grid) == want


def test_staged_offsets_c2(U, patterns):
    _check(U, patterns["c2_foobarbaz"]["opc"], gen(1, 5, 0, 24 << 20))


def test_staged_offsets_matches_across_wave_borders(U, patterns):
    host = gen(2, 6, 0, 8 << 20)  # letters without b/f: only planted matches
    for t in range(4096, host.size - 4, 4096):
        host[t - 1:t + 2] = np.frombuffer(b"foo", np.uint8)  # crosses every tile (and wave) border
    for grid in (None, 7, 64):
        _check(U, patterns["c2_foobarbaz"]["opc"], host, grid)


def test_staged_offsets_overflow(U):
    opc = U.compile_regex("q")
    host = gen(2, 7, 0, 4 << 20)
    host[(1 << 20):(1 << 20) + 200000] = ord("q")  # far more than 1024 records in one wave
    _check(U, opc, host)
    _check(U, opc, host, 3)
