"""GPU: binary-file detection: reflex::isutf8
(lib/simd.cpp:169-421), memchr NUL, and ugrep's is_binary / init_is_binary
(src/ugrep.cpp:699-711, :3998-4015) on the device.

Pinned to the reference's own answers: tests/golden/utf8.json holds
reflex::isutf8 of the compiled reference (both the AVX512BW-dispatching and
the AVX2 build) on 3712 inputs placed around its 16/32-byte SIMD blocks; the
first failing offset is checked against the oracle restatement
(oracle/restate.c orc_utf8_first_bad, itself checked against the goldens in
tests/test_oracle.py).  Large buffers check tile (4 KiB) and wave-range
borders, cut-off sequences at the exact end, misaligned pointers and
early exit with several failures."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "utf8.json")


@pytest.fixture(scope="module")
def U():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


class Dev:
    """A device buffer holding `data` at byte offset `align`, surrounded by
    bytes that would fail every check (0x80 before, 0x00 after)."""

    def __init__(self, data, align=0):
        import torch
        data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray)
                                    else data)
        self.n = data.size
        host = np.full(self.n + align + 64, 0x80, np.uint8)
        host[align + self.n:] = 0
        host[align:align + self.n] = data
        self.t = torch.from_numpy(host).to("cuda")
        torch.cuda.synchronize()
        self.ptr = self.t.data_ptr() + align


def test_golden_cases(U, gold):
    import torch
    cases = [bytes.fromhex(h) for h, _ in gold["cases"]]
    # one device arena, each case at its own (varying) alignment
    offs, pos = [], 0
    for i, c in enumerate(cases):
        pos = (pos + 15) // 16 * 16 + (i % 16)
        offs.append(pos)
        pos += len(c) + 8
    host = np.full(pos + 64, 0x80, np.uint8)
    for c, o in zip(cases, offs):
        host[o:o + len(c)] = np.frombuffer(c, np.uint8)
    t = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    bad = []
    for (h, ref), c, o in zip(gold["cases"], cases, offs):
        fb = U.check_utf8(t.data_ptr() + o, len(c))
        if (fb is None) != ref or fb != O.utf8_first_bad(c):
            bad.append((h, ref, fb))
    assert not bad, bad[:5]


def test_golden_inputs(U, gold):
    for inp in gold["inputs"]:
        data = O.case_input(inp)
        d = Dev(data, 3)
        assert U.isutf8(d.ptr, d.n) == inp["isutf8"], inp


def _c4(n, seed=7):
    return O.gen(4, seed, 0, n)


@pytest.mark.parametrize("n", [4096, 16384, 64 << 10, (1 << 20) + 4096, (8 << 20) + 16])
def test_cut_at_end(U, n):
    """A lead (or a partial sequence) as the last bytes: fails at len."""
    base = np.full(n, ord("a"), np.uint8)
    for tail in (b"\xc3", b"\xe2\x82", b"\xf0\x90\x80", b"\xf0\x90"):
        data = base.copy()
        data[n - len(tail):] = np.frombuffer(tail, np.uint8)
        for align in (0, 5):
            d = Dev(data, align)
            assert U.check_utf8(d.ptr, d.n) == O.utf8_first_bad(data) == n
    ok = base.copy()
    ok[n - 2:] = np.frombuffer(b"\xc3\xa9", np.uint8)
    assert U.check_utf8(Dev(ok).ptr, n) is None


def test_planted_errors_on_borders(U):
    n = 64 << 20
    base = _c4(n)
    assert O.utf8_first_bad(base) is None
    d = Dev(base)
    assert U.check_utf8(d.ptr, n) is None
    import torch
    rng = np.random.default_rng(5)
    spots = [0, 1, 15, 16, 1023, 1024, 4095, 4096, 4097, 16383, 16384, 65535, 65536, n // 2, n - 4097, n - 1]
    spots += rng.integers(0, n, 24).tolist()
    for s in spots:
        for byte in (0x00, 0x80, 0xc3, 0xff):
            data = base.copy()
            data[s] = byte
            want = O.utf8_first_bad(data)
            d.t[s] = byte
            torch.cuda.synchronize()
            got = U.check_utf8(d.ptr, n)
            d.t[s] = int(base[s])
            assert got == want, (s, byte, got, want)


def test_first_of_many(U):
    """Several failures: the lowest offset wins across waves (early exit)."""
    n = 32 << 20
    data = _c4(n, 3)
    rng = np.random.default_rng(9)
    idx = np.sort(rng.integers(1 << 20, n, 200))
    data[idx] = 0xff
    d = Dev(data, 7)
    assert U.check_utf8(d.ptr, n) == O.utf8_first_bad(data) == int(idx[0])


def test_nul(U):
    n = 8 << 20
    data = np.full(n, ord("x"), np.uint8)
    d = Dev(data, 1)
    assert U.find_nul(d.ptr, n) is None
    for s in (0, 17, 4095, 4096, 1 << 20, n - 1):
        data2 = data.copy()
        data2[s] = 0
        data2[min(n - 1, s + 100)] = 0
        assert U.find_nul(Dev(data2, s % 16).ptr, n) == s == O.first_nul(data2)
    utf = _c4(n)  # UTF-8 without NUL
    assert U.find_nul(Dev(utf).ptr, n) is None


def test_empty(U):
    d = Dev(b"", 0)
    assert U.check_utf8(d.ptr, 0) is None
    assert U.find_nul(d.ptr, 0) is None
    assert U.is_binary(d.ptr, 0, init_window=True) is False


def test_is_binary_flags(U, gold):
    import itertools
    cases = [bytes.fromhex(h) for h, _ in gold["cases"][::7]]
    cases += [b"abc\xc3", b"abc\xe2\x82", b"ab\x80", b"\x80\x80\x80\x80\x80", b"a\x00b\xc3\xa9",
              b"\xf0\x90\x80\x80", b"x\xf0\x90\x80\x80\x80"]
    for c in cases:
        d = Dev(c, len(c) % 16)
        for nd, no, iw in itertools.product((False, True), repeat=3):
            want = O.is_binary(c, null_data=nd, nul_only=no, init_window=iw)
            got = U.is_binary(d.ptr, len(c), null_data=nd, nul_only=no, init_window=iw)
            assert got == want, (c.hex(), nd, no, iw)
