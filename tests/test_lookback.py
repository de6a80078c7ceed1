"""Loop-needle tables (C+ N, e.g. [a-z]+ing): the sparse kernel's prefilter
looks for the needle N and each candidate walks back over C to its run's start
(ugrep_amd/csrc/host_api.cpp loop_needle, sparse_kernel.hip lb_batch; the
reference's lookback, lib/matcher.cpp:636-656, restated for the FIND chain;
DESIGN.md 3.15).

CPU: which tables the plan recognises (ugpu_dfa_plan_host shape bit
UGPU_SHAPE_LOOP_NEEDLE), with and without option W.
GPU: equal to the oracle, record by record, with the lookback on and off
(UGPU_LB=0), over text built to break it: runs longer than a lane's walk and
than a wave's range, runs at the buffer ends, self-overlapping needles, runs
of nothing but needles; scans that start inside a run, shards cut at every
kind of byte, streams, COUNT and OFFSETS, option W."""
import os

import numpy as np
import pytest

from oracle_lib import OracleDfa

NO = ["[a-z]*ing", "ing", "[a-z]+", "[a-z]+ing|foo", "a[a-z]+ing", "[a-z]+ING", "[a-z]+i", "[a-z]+in[a-z]g",
      # (round 6 needle sets: an infinite set, a one-byte string, a string
      # with a byte outside C, more than 16 strings)
      "[a-z]+(ing|ed)[a-z]*", "[a-z]+(ed|ing|s)", "x+(xx|xy)", "[a-z]+in[a-z]g|[a-z]+ed"]


def test_plan_loop_needle():
    import ugrep_amd as U
    from ugrep_amd._lib import SHAPE_LOOP_NEEDLE as LB
    for rx, _, _ in CASES:
        assert U.host_plan(rx)["shape"] & LB, rx
        assert U.host_plan(rx)["kernel"] == 0, rx
    for rx in NO:
        try:
            assert not U.host_plan(rx)["shape"] & LB, rx
        except U.Unsupported:
            pass
    # option W: only when every run byte is a word byte (then no match starts
    # inside a run)
    assert U.host_plan("[a-z]+ing", word=True)["shape"] & LB
    assert U.host_plan("[a-z@]+ing")["shape"] & LB
    assert not U.host_plan("[a-z@]+ing", word=True)["shape"] & LB
    assert not U.host_plan("[a-z-]+ing", word=True)["shape"] & LB
    assert U.host_plan("[A-Za-z]+tion", word=True)["shape"] & LB
    # without the lookback these have no prefilter and run other kernels
    os.environ["UGPU_LB"] = "0"
    try:
        assert U.host_plan("[A-Za-z]+tion")["kernel"] != 0
        assert U.host_plan("[a-z-]+ing")["kernel"] != 0
    finally:
        os.environ.pop("UGPU_LB", None)
    os.environ["UGPU_LB"] = "0"
    try:
        assert not U.host_plan("[a-z]+ing")["shape"] & LB
    finally:
        os.environ.pop("UGPU_LB", None)


# (pattern, needle, a byte of C).  The oracle is the reference's FIND without
# its lookback: a C-run's bytes after its last needle cost it quadratic time,
# so the long runs below end in a needle and needle-free runs stay short.
CASES = [("[a-z]+ing", "ing", "q"), ("[a-z]+aa", "aa", "q"), ("[a-z]+abab", "abab", "q"), ("[0-9]+00", "00", "7"),
         ("x+xx", "xx", "x"), ("[a-z_]+ing", "ing", "_"), ("[a-z@]+ing", "ing", "@"),
         # (no first-byte prefilter: 52 and 27 first bytes; the lookback alone
         # puts them on the sparse kernel)
         ("[A-Za-z]+tion", "tion", "Q"), ("[a-z-]+ing", "ing", "-"),
         # (round 6: a finite set of strings, C+ (N1|N2|...); the needle column is
         # the one the text plants, "ing" comes with the random tokens)
         ("[a-z]+(ing|ed)", "ed", "q"), ("[A-Za-z]+(tion|sion|ment)", "sion", "Q"), ("[0-9]+(00|50)", "50", "7"),
         ("[a-z]+(ab|cd|ef)x", "cdx", "q")]


def _text(seed, n_tok, needle, f):
    rng = np.random.default_rng(seed)
    toks = ["ing", "xing", "sing", "singing", "inging", "ingi", "in", "ng", "a", "bb", "Xing", "ING", " ", "\n", "-",
            "_", "é", "9", "walking", "thing ", "aa", "aaa", "abab", "ababab", "00", "1000", "tion", "nation",
            "Nation", "a-bing", "-xing", "a@bing", "@xing", "@@", "xy", "xxxy", "xyxy", "\0", " ", " ", "\n"]
    parts = [toks[int(i)] for i in rng.integers(0, len(toks), n_tok)]
    segs = [f + "bc" + needle + "".join(parts[: n_tok // 2])]
    # long runs: a lane's walk back (> 64 bytes), a wave's range (> 64 KiB),
    # runs of needles, runs around a needle, a needle-free run
    segs += [" " + f * 70000 + needle + " ", f * 3000 + " ", needle * 50000, " " + f * 200 + needle + f * 200 + " ",
             f * 150000 + needle + f * 100 + needle, " " + needle + f * 3 + needle + " "]
    segs += ["".join(parts[n_tok // 2:]), " " + f * 5 + needle + " " + f * 4 + needle]
    host = np.frombuffer("".join(segs).encode(), np.uint8).copy()
    # runs planted across 16-byte lanes, 1 KiB chunks and 4 KiB tiles
    plant = (" " + f * 6 + needle + " ").encode()
    for p in range(4096 - 5, host.size - 64, 4096 * 7):
        host[p:p + len(plant)] = np.frombuffer(plant, np.uint8)
    plant = (f * 3 + needle).encode()
    for p in range(1024 - 2, host.size - 64, 1024 * 13):
        host[p:p + len(plant)] = np.frombuffer(plant, np.uint8)
    return host


@pytest.fixture(scope="module")
def U():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


def _pattern(U, rx, lb, word=False):
    os.environ["UGPU_LB"] = lb
    try:
        pat = U.Pattern(rx, word=word)
    finally:
        os.environ.pop("UGPU_LB", None)
    from ugrep_amd._lib import SHAPE_LOOP_NEEDLE
    return pat, bool(pat.info()["shape"] & SHAPE_LOOP_NEEDLE)


@pytest.mark.gpu
def test_gpu_lookback_whole_and_starts(U):
    import torch
    for k, (rx, needle, f) in enumerate(CASES):
        host = _text(3 + k, 120000, needle, f)
        dev = torch.from_numpy(host).to("cuda")
        # scan starts inside runs: the 70000-byte run, the needle run, a planted one
        s70 = host.tobytes().index((f * 1000).encode()) + 500
        sn = host.tobytes().index((needle * 1000).encode()) + 1
        o = OracleDfa(U.compile_regex(rx))
        # (without the lookback, fix_kernel re-walks a needle-free run from every
        # position, quadratic: UGPU_LB=0 runs on the random-token part only)
        part = host[:190000].copy()
        for lb, h in (("1", host), ("0", part)):
            want = o.find(h, want_list=True)
            d = dev if lb == "1" else torch.from_numpy(part).to("cuda")
            pat, on = _pattern(U, rx, lb)
            assert on == (lb == "1"), rx
            r = U.find_all(pat, d, offsets=True)
            assert (r.count, r.digest, r.dcap) == want[:3], (rx, lb)
            assert r.triples() == want[3], (rx, lb)
            r = U.find_all(pat, d, offsets=False)
            assert (r.count, r.digest, r.dcap) == want[:3], (rx, lb)
        pat, _ = _pattern(U, rx, "1")
        for s in ((1, 3, s70, sn, 4096 * 7 + 1) if k < 2 else (2, s70)):
            w = o.find(host, start=s, want_list=True)
            r = U.find_all(pat, dev, start=s, offsets=True)
            assert r.triples() == w[3], (rx, s)


@pytest.mark.gpu
def test_gpu_lookback_shards_streams_records(U):
    import torch
    rng = np.random.default_rng(9)
    for k in (0, 2, 3, 7, 9, 12):
        rx, needle, f = CASES[k]
        host = _text(20 + k, 100000, needle, f)
        dev = torch.from_numpy(host).to("cuda")
        want = OracleDfa(U.compile_regex(rx)).find(host, want_list=True)
        pat, on = _pattern(U, rx, "1")
        assert on
        for nd in (2, 3, 5):
            r = U.find_all_multi(pat, dev, ndev=nd, offsets=True)
            assert r.triples() == want[3], (rx, nd)
        assert U.Records(pat, dev).triples() == want[3], rx
        st = U.Stream(pat, keep=4096)
        got, i = [], 0
        sizes = [int(x) for x in rng.integers(1, 300000, 64)] + [7, 1, 70001]
        k = 0
        while i < host.size:
            n = sizes[k % len(sizes)]
            k += 1
            got += st.feed(host[i:i + n].tobytes(), final=i + n >= host.size).triples()
            i += n
        st.close()
        assert got == want[3], rx


@pytest.mark.gpu
def test_gpu_lookback_word(U):
    import torch
    for k in (0, 3, 1, 6, 5, 7, 8, 9, 10, 11):
        rx, needle, f = CASES[k]
        host = _text(30 + k, 100000, needle, f)
        dev = torch.from_numpy(host).to("cuda")
        o = OracleDfa(U.compile_regex(rx))
        want = o.find_w(host, want_list=True)
        for lb in ("1", "0"):
            pat, on = _pattern(U, rx, lb, word=True)
            assert on == (lb == "1" and rx not in ("[a-z@]+ing", "[a-z-]+ing")), rx
            r = U.find_all(pat, dev, offsets=True)
            assert (r.count, r.digest, r.dcap) == want[:3], (rx, lb)
            assert r.triples() == want[3], (rx, lb)
        w = o.find_w(host, start=3, want_list=True)
        assert U.find_all(pat, dev, start=3).triples() == w[3], rx
        # (UGPU_SPARSE=0: wfind_kernel, which applies the W rules itself)
        os.environ["UGPU_SPARSE"] = "0"
        try:
            pat0 = U.Pattern(rx, word=True)
            assert U.find_all(pat0, dev, offsets=True).triples() == want[3], (rx, "wfind")
        finally:
            os.environ.pop("UGPU_SPARSE", None)


@pytest.mark.gpu
def test_gpu_lookback_giant_runs(U):
    """One run of 32 MiB of needles, one of 32 MiB of C with the needle at its
    end: the walks back cover each byte a bounded number of times (a quadratic
    lookback would not finish)."""
    import time
    import torch
    for body, rx in ((b"ing" * (11 << 20), "[a-z]+ing"), (b"a" * (32 << 20) + b"ing", "[a-z]+ing"),
                     (b"ab" * (16 << 20) + b"abab", "[a-z]+abab")):
        host = np.frombuffer(b" " + body + b" ", np.uint8).copy()
        dev = torch.from_numpy(host).to("cuda")
        want = OracleDfa(U.compile_regex(rx)).find(host, want_list=True)
        pat, on = _pattern(U, rx, "1")
        assert on
        U.find_all(pat, dev, offsets=False)
        t0 = time.perf_counter()
        r = U.find_all(pat, dev, offsets=True)
        dt = time.perf_counter() - t0
        assert r.triples() == want[3], rx
        assert dt < 2.0, (rx, dt)


def _fuzz_cases(seed, n):
    """Random C+ N patterns (and near misses that must not take the lookback)
    with texts of C-runs around needles."""
    rng = np.random.default_rng(seed)
    pools = ["abcdefghijklmnopqrstuvwxyz", "abc", "ab", "0123456789", "xyz_", "aeiou", "ABCabc", "a@b#"]
    out = []
    for _ in range(n):
        pool = pools[int(rng.integers(0, len(pools)))]
        k = int(rng.integers(1, len(pool) + 1))
        cset = sorted(set(rng.choice(list(pool), k, replace=True)))
        m = int(rng.integers(2, 6))
        needle = "".join(rng.choice(cset, m))
        cls = "[" + "".join(c if c not in "^]-\\" else "\\" + c for c in cset) + "]"
        rx = cls + "+" + needle
        # (C+ (N)+ is no near miss: N is in C*, so it is the language C+ N)
        near = [cls + "*" + needle, cls + "+" + needle + cls + "*"]
        if len(cset) == 1:  # (c* c^m and c+ c^m c* are c+ c^(m-1), c+ c^m: loop-needle languages)
            near = []
        same = cls + "+(" + needle + ")+"
        # text: runs of C (geometric lengths, a few long) holding needles, and separators
        parts = []
        for _ in range(4000):
            r = rng.random()
            if r < 0.5:
                parts.append("".join(rng.choice(cset, int(rng.geometric(0.2)))))
            elif r < 0.8:
                parts.append(needle)
            elif r < 0.995:
                parts.append(str(rng.choice([" ", "\n", ".", "-", "Z", "é", "\0"])))
            else:
                parts.append("".join(rng.choice(cset, int(rng.integers(100, 3000)))) + needle)
        out.append((rx, near, "".join(parts).encode(), set(cset), same))
    return out


def test_plan_fuzz_near_misses():
    """Near misses of C+ N never take the lookback (their languages differ)."""
    import ugrep_amd as U
    from ugrep_amd._lib import SHAPE_LOOP_NEEDLE as LB
    for rx, near, _, _, same in _fuzz_cases(7, 60):
        assert U.host_plan(rx)["shape"] & LB, rx
        assert U.host_plan(same)["shape"] & LB, same
        for nr in near:
            try:
                assert not U.host_plan(nr)["shape"] & LB, nr
            except U.Unsupported:
                pass


@pytest.mark.gpu
def test_gpu_lookback_fuzz(U):
    """100 random C+ N patterns (C from letters, digits, '_', punctuation;
    needles of 2-5 bytes, often self-overlapping) over texts of C-runs, with
    and without option W, and their near misses: equal to the oracle record by
    record."""
    import torch
    word = set("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_")
    for rx, near, text, cset, _ in _fuzz_cases(11, 100):
        host = np.frombuffer(text, np.uint8).copy()
        dev = torch.from_numpy(host).to("cuda")
        o = OracleDfa(U.compile_regex(rx))
        want = o.find(host, want_list=True)
        pat, on = _pattern(U, rx, "1")
        assert on, rx
        r = U.find_all(pat, dev, offsets=True)
        assert r.triples() == want[3], rx
        r = U.find_all_multi(pat, dev, ndev=3, offsets=True)
        assert r.triples() == want[3], (rx, "shards")
        w = o.find_w(host, want_list=True)
        patw, onw = _pattern(U, rx, "1", word=True)
        assert onw == cset.issubset(word), rx
        assert U.find_all(patw, dev, offsets=True).triples() == w[3], (rx, "W")
        for nr in near[:2]:
            want = OracleDfa(U.compile_regex(nr)).find(host, want_list=True)
            pat, on = _pattern(U, nr, "1")
            assert not on, nr
            assert U.find_all(pat, dev, offsets=True).triples() == want[3], nr


def _fuzz_multi_cases(seed, n):
    """Random C+ (N1|N2|...) patterns: two to four strings of 2-5 bytes of C."""
    rng = np.random.default_rng(seed)
    pools = ["abcdefghijklmnopqrstuvwxyz", "abc", "ab", "0123456789", "xyz_", "aeiou", "ABCabc", "a@b#"]
    out = []
    for _ in range(n):
        pool = pools[int(rng.integers(0, len(pools)))]
        cset = sorted(set(rng.choice(list(pool), int(rng.integers(2, len(pool) + 1)), replace=True)))
        needles = ["".join(rng.choice(cset, int(rng.integers(2, 6)))) for _ in range(int(rng.integers(2, 5)))]
        cls = "[" + "".join(c if c not in "^]-\\" else "\\" + c for c in cset) + "]"
        alt = "(" + "|".join(needles) + ")"
        rx = cls + "+" + alt
        near = [cls + "*" + alt, cls + "+" + alt + cls + "*"]
        parts = []
        for _ in range(4000):
            r = rng.random()
            if r < 0.5:
                parts.append("".join(rng.choice(cset, int(rng.geometric(0.2)))))
            elif r < 0.8:
                parts.append(needles[int(rng.integers(0, len(needles)))])
            elif r < 0.995:
                parts.append(str(rng.choice([" ", "\n", ".", "-", "Z", "é", "\0"])))
            else:
                parts.append("".join(rng.choice(cset, int(rng.integers(100, 3000)))) + needles[0])
        out.append((rx, near, "".join(parts).encode(), set(cset), cls + "+" + alt + "+"))
    return out


def test_plan_multi_needles():
    """C+ (N1|...) with a finite set of strings of >= 2 bytes of C takes the
    lookback (and C+ (N1|...)+, the same language)."""
    import ugrep_amd as U
    from ugrep_amd._lib import SHAPE_LOOP_NEEDLE as LB
    for rx, _, _, _, same in _fuzz_multi_cases(5, 80):
        assert U.host_plan(rx)["shape"] & LB, rx
        assert U.host_plan(same)["shape"] & LB, same


@pytest.mark.gpu
def test_gpu_lookback_multi_fuzz(U):
    """60 random C+ (N1|...) patterns over texts of C-runs holding their
    strings, whole, in 3 shards and with option W, and their near misses
    C* (N1|...) and C+ (N1|...) C* (the plan may or may not take those: the
    results must equal the oracle either way), record by record."""
    import torch
    word = set("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_")
    for rx, near, text, cset, _ in _fuzz_multi_cases(13, 60):
        host = np.frombuffer(text, np.uint8).copy()
        dev = torch.from_numpy(host).to("cuda")
        o = OracleDfa(U.compile_regex(rx))
        want = o.find(host, want_list=True)
        pat, on = _pattern(U, rx, "1")
        assert on, rx
        assert U.find_all(pat, dev, offsets=True).triples() == want[3], rx
        assert U.find_all_multi(pat, dev, ndev=3, offsets=True).triples() == want[3], (rx, "shards")
        assert U.find_all(pat, dev, offsets=False).count == want[0], (rx, "count")
        w = o.find_w(host, want_list=True)
        patw, onw = _pattern(U, rx, "1", word=True)
        assert onw == cset.issubset(word), rx
        assert U.find_all(patw, dev, offsets=True).triples() == w[3], (rx, "W")
        for nr in near:
            want = OracleDfa(U.compile_regex(nr)).find(host, want_list=True)
            pat, _ = _pattern(U, nr, "1")
            assert U.find_all(pat, dev, offsets=True).triples() == want[3], nr


@pytest.mark.gpu
def test_gpu_lookback_multi_giant_run(U):
    """A 32 MiB run of C whose only string of N ends it, after a short match,
    for a needle-set table: the walks back cover it a bounded number of times
    (the oracle walks it once, from its start)."""
    import time
    import torch
    host = np.frombuffer(b" xxed " + b"q" * (32 << 20) + b"ing xing ", np.uint8).copy()
    dev = torch.from_numpy(host).to("cuda")
    rx = "[a-z]+(ing|ed)"
    want = OracleDfa(U.compile_regex(rx)).find(host, want_list=True)
    pat, on = _pattern(U, rx, "1")
    assert on
    U.find_all(pat, dev, offsets=False)
    t0 = time.perf_counter()
    r = U.find_all(pat, dev, offsets=True)
    dt = time.perf_counter() - t0
    assert r.triples() == want[3]
    assert dt < 2.0, dt
