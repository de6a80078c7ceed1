"""Dominated restarts: the FIND chain's serial re-walks (fix_kernel's merges and
its resolved open walks, device_common.hpp chain_step / dom_restart) skip the
positions a failed walk crossed in states that dominate the start state
(tables.hpp dom: L(start) is a subset of L(s)).  The reference restarts one
position after a failed match (lib/matcher.cpp:692-713); the skip changes no
result, only the cost of a needle-free run (one walk instead of one per
position).

CPU: the bits equal a brute-force inclusion check on the host tables, and a
Python restatement of the chain with the skip equals the oracle's FIND on
texts with long needle-free runs.
GPU: prefiltered tables that are not loop-needle tables ([a-z]+(ing|ed) and
others) over needle-free runs of 5000 bytes and of 32 MiB, equal to the oracle
and within a wall-time bound."""
import os
import time

import numpy as np
import pytest

from oracle_lib import OracleDfa

# prefiltered (sparse_kernel) tables that are not loop-needle tables, and two
# dense ones; each dominates its start in every state its letter loop reaches
PATS = ["[a-z]+(ing|ed)", "[a-z]*q[a-z]*x", "a[a-z]*(ing|ed)", "[a-z]+(ab|cd|ef)x"]
MORE = ["foo|bar|baz", "[A-Za-z_][A-Za-z0-9_]*", "[0-9]+\\.[0-9]+", "x[a-z]*y|q+r", "(ab)+c", "a.*b", "[a-z]+[0-9]"]


def _tables(rx):
    import ugrep_amd as U
    opc = U.compile_regex(rx)
    return opc, U.host_tables(opc)


def _brute_dom(h):
    """L(start) <= L(s) for every state s, by a lock-step search of the pairs."""
    info, trans, cls = h["info"], h["trans"].astype(np.int64), h["cls"]
    R, S = info["row"], info["states"]
    accb = h["accb"] // R
    start = h["start"] // R
    cols = sorted(set(int(c) for c in cls)) if info["format"] != 0 else list(range(256))
    nxt = trans.reshape(S, R)[:, cols] // R
    out = np.zeros(S, bool)
    for s in range(1, S):
        seen, todo, bad = {(start, s)}, [(start, s)], False
        while todo and not bad:
            a, b = todo.pop()
            if a == 0:
                continue
            if b == 0 or (a >= accb and b < accb):
                bad = True
                break
            for na, nb in zip(nxt[a], nxt[b]):
                if na and (na, nb) not in seen:
                    seen.add((na, nb))
                    todo.append((int(na), int(nb)))
        out[s] = not bad
    return out


@pytest.mark.parametrize("rx", PATS + MORE)
def test_dom_bits_equal_brute_force(rx):
    from ugrep_amd.matcher import host_dom
    opc, h = _tables(rx)
    got = host_dom(opc)
    assert got is not None, rx
    S = h["info"]["states"]
    assert np.array_equal(got[:S], _brute_dom(h)), rx
    assert not got[S:].any()


def test_dom_all():
    """dom_all: every non-accepting state reachable from the start dominates
    it (sparse_kernel's failed long walks skip to the byte they died on)."""
    from ugrep_amd.matcher import host_dom
    for rx in PATS + ["[a-z]+[0-9]", "[A-Za-z_][A-Za-z0-9_]*"]:
        opc, h = _tables(rx)
        bits, al = host_dom(opc, want_all=True)
        assert al, rx
    for rx in ["foo|bar|baz", "(ab)+c", "x[a-z]*y|q+r"]:
        opc, h = _tables(rx)
        bits, al = host_dom(opc, want_all=True)
        assert not al, rx


def test_dom_holds_along_the_letter_loops():
    """The states a letter run keeps these tables in all dominate the start."""
    from ugrep_amd.matcher import host_dom
    for rx in PATS:
        opc, h = _tables(rx)
        dom = host_dom(opc)
        R = h["info"]["row"]
        trans = h["trans"].astype(np.int64)
        s = h["start"]
        for b in b"abcdfghjklmnopstuvwz" * 3:
            e = int(trans[s + b] if h["info"]["format"] == 0 else trans[s + h["cls"][b]])
            if e == 0:
                break
            assert dom[e // R], (rx, chr(b))
            s = e


def _chain_with_skip(h, dom, data, start=0):
    """The FIND chain over data with the dominated-restart skip (a restatement
    of chain_step with w.dom, uncapped): list of (start, len, cap)."""
    info, trans = h["info"], h["trans"]
    R, fmt, cls = info["row"], info["format"], h["cls"]
    accb, caps = h["accb"], h["caps"]
    data, trans, cls = data.tolist(), trans.tolist(), cls.tolist()
    n, p, out = len(data), start, []
    while p < n:
        s, q, last, le, skip = h["start"], p, p, 0, 0
        while q < n:
            e = trans[s + (data[q] if fmt == 0 else cls[data[q]])]
            if e == 0:
                skip = skip or q + 1
                break
            s, q = e, q + 1
            if e >= accb:
                last, le = q, e
            if not skip and not dom[e // R]:
                skip = q
        skip = skip or q
        if last > p:
            out.append([p, last - p, int(caps[le // R])])
            p = last
        else:
            p = max(skip, p + 1)
    return out


def _runs_text(rng, n, run_len, letters=b"abcdfghjklmnopstuvwz"):
    """Words and punctuation with needle-free letter runs of run_len planted."""
    words = [b"testing", b"sailed", b"abx", b"qux", b"aing", b"aed", b"cdx", b"ab", b"x", b"q", b"12.5", b"foo", b"bar"]
    out = bytearray()
    while len(out) < n:
        k = rng.integers(0, 10)
        if k == 0:
            out += bytes(rng.choice(np.frombuffer(letters, np.uint8), run_len))
        else:
            out += words[rng.integers(0, len(words))]
        out += b" ,\n"[rng.integers(0, 3):][:1]
    return np.frombuffer(bytes(out[:n]), np.uint8).copy()


@pytest.mark.parametrize("rx", PATS + MORE)
def test_chain_with_skip_equals_oracle(rx):
    from ugrep_amd.matcher import host_dom
    opc, h = _tables(rx)
    dom = host_dom(opc)
    rng = np.random.default_rng(7)
    o = OracleDfa(opc)
    for run_len in (3, 40, 700):
        data = _runs_text(rng, 20000, run_len)
        want = o.find(data, want_list=True)[3]
        assert _chain_with_skip(h, dom, data) == want, (rx, run_len)
        assert _chain_with_skip(h, dom, data, start=1234) == o.find(data, start=1234, want_list=True)[3], rx


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
@pytest.mark.parametrize("rx", PATS)
def test_run_5000_against_oracle(U, rx):
    """5000-byte needle-free runs at tile and wave borders: equal to the
    oracle record by record, COUNT within 5 ms (1.6 s with the quadratic
    re-walk)."""
    rng = np.random.default_rng(11)
    base = np.frombuffer((b"the sailing boat passed qux abcdx " * 32000)[:1 << 20], np.uint8).copy()
    for pos in (4096 - 2500, 65536 - 100, 300001, (1 << 20) - 5000):
        base[pos:pos + 5000] = rng.choice(np.frombuffer(b"abcdfghjklmnopstuvwz", np.uint8), 5000)
    opc = U.compile_regex(rx)
    pat = U.Pattern(opc)
    dev = _dev(base)
    want = OracleDfa(opc).find(base, want_list=True)
    got = U.find_all(pat, dev, offsets=True)
    assert (got.count, got.digest, got.dcap) == want[:3], rx
    assert [list(t) for t in got.triples()] == want[3], rx
    U.find_all(pat, dev, offsets=False)
    t0 = time.perf_counter()
    r = U.find_all(pat, dev, offsets=False)
    dt = time.perf_counter() - t0
    assert (r.count, r.digest, r.dcap) == want[:3], rx
    assert dt < 0.005, (rx, dt)


@pytest.mark.gpu
@pytest.mark.parametrize("rx", PATS)
def test_run_32mib(U, rx):
    """One 32 MiB needle-free run between two short texts: the matches are
    those of the texts (the run holds none and ends at a space), found in
    under 2 s; offsets past the run shift by its length."""
    head = b"the sailing boat, abx qux aing wed cdx. "
    tail = b" testing ended; qxqx abcdx sailed aed."
    run = np.frombuffer(b"abcdfghjklmnopstuvwz", np.uint8)
    n = 32 << 20
    big = np.concatenate([np.frombuffer(head, np.uint8), np.resize(run, n), np.frombuffer(tail, np.uint8)])
    small = np.concatenate([np.frombuffer(head, np.uint8), np.resize(run, 1000), np.frombuffer(tail, np.uint8)])
    opc = U.compile_regex(rx)
    want = OracleDfa(opc).find(small, want_list=True)[3]
    shift = n - 1000
    want = [[s + (shift if s >= len(head) + 1000 else 0), ln, c] for s, ln, c in want]
    pat = U.Pattern(opc)
    dev = _dev(big)
    t0 = time.perf_counter()
    got = U.find_all(pat, dev, offsets=True)
    dt = time.perf_counter() - t0
    assert [list(t) for t in got.triples()] == want, rx
    assert dt < 2.0, (rx, dt)
    # shards cut inside the run
    m = U.find_all_multi(pat, big, ndev=3, offsets=False)
    assert m.count == len(want), rx
