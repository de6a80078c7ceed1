"""GPU: BASELINE config C5's logic on one card -- one logical stream cut into
shards at arbitrary offsets (inside matches), every shard scanned from its own
device buffer with the HIP Scanner, the shard chains stitched by the same
protocol the multi-GPU bench runs (ugrep_amd.dist.resolve / stitch +
ugpu_chain_fix), the match records gathered in chain order (gather_offsets).

Expected values are the REFERENCE matcher's count/digest/dcap over the same
bytes (tests/golden/streams.json, tools: tests/golden/make_stream_golden.py),
and for C2 the oracle's full match list.  The reference has no multi-GPU
counterpart: what is pinned is that sharding changes nothing.
"""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

M64 = (1 << 64) - 1
HALO = 1 << 20


@pytest.fixture(scope="module")
def U():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import ugrep_amd
    return ugrep_amd


@pytest.fixture(scope="module")
def streams():
    from oracle_lib import GOLDEN
    with open(os.path.join(GOLDEN, "streams.json")) as f:
        return json.load(f)


def _stream():
    return torch.cuda.current_stream().cuda_stream


class Shard:
    """One GPU's shard [lo, hi) of the stream, in its own buffer [lo, read_end)."""

    def __init__(self, U, pat, whole, lo, hi, total):
        self.lo, self.hi = lo, hi
        self.read_end = min(total, hi + HALO)
        self.eof = self.read_end == total
        self.buf = torch.empty(self.read_end - lo + 16, dtype=torch.uint8, device="cuda")
        self.buf[:self.read_end - lo].copy_(whole[lo:self.read_end])
        self.sc = U.Scanner(pat)

    def scan(self, entry=None):
        e = self.lo if entry is None else min(entry, self.hi)
        self.sc.scan(self.buf.data_ptr(), e - self.lo, self.hi - self.lo, self.read_end - self.lo, self.eof, self.lo,
                      _stream())
        t = self.sc.totals()
        return dict(entry=t.entry + self.lo, exit=t.exit + self.lo, count=t.count, digest=t.digest, dcap=t.dcap)

    def fix(self, old, new):
        t = self.sc.chain_fix(self.buf.data_ptr(), 0, self.hi - self.lo, self.read_end - self.lo, self.eof, self.lo,
                              old - self.lo, new - self.lo, _stream())
        return dict(count=t.count, digest=t.digest, dcap=t.dcap, exit=None if t.exit == M64 else t.exit + self.lo)

    def records(self, count):
        st = torch.empty(max(count, 1), dtype=torch.int64, device="cuda")
        ln = torch.empty(max(count, 1), dtype=torch.int32, device="cuda")
        cp = torch.empty(max(count, 1), dtype=torch.int32, device="cuda")
        if count:
            self.sc.offsets(st.data_ptr(), ln.data_ptr(), cp.data_ptr(), count, _stream())
        return st[:count], ln[:count], cp[:count]


def _sharded(U, pat, whole, total, cuts):
    from ugrep_amd.dist import resolve
    bounds = [0] + list(cuts) + [total]
    shards = [Shard(U, pat, whole, bounds[i], bounds[i + 1], total) for i in range(len(bounds) - 1)]
    recs = [s.scan() for s in shards]
    out = resolve(recs, lambda r, old, new: shards[r].fix(old, new))
    # materialise the records of the true chain: a shard whose entry moved re-scans from it
    parts = []
    for r, s in enumerate(shards):
        cnt = recs[r]["count"]
        if out["entries"][r] != s.lo:
            cnt = s.scan(out["entries"][r])["count"]
        assert cnt == out["counts"][r], r
        parts.append(s.records(cnt))
    st = torch.cat([p[0] for p in parts])
    ln = torch.cat([p[1] for p in parts])
    cp = torch.cat([p[2] for p in parts])
    return out, st, ln, cp


def _digests(st, ln, cp):
    s = st.to(torch.int64)
    dg = int((s * 31 + ln.to(torch.int64)).sum().item()) & M64
    dc = int(((s + 1) * cp.to(torch.int64)).sum().item()) & M64
    return dg, dc


def _whole(U, kind, n):
    t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    U.gen(kind, 1, 0, t.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    return t


def test_c5_eight_shards_inside_matches(U, patterns, streams):
    """C2 'foo|bar|baz' over a 512 MiB C2-generator stream, 8 shards whose cuts
    fall strictly inside matches (so every boundary needs ugpu_chain_fix):
    totals equal the reference's, and the gathered record list equals the
    oracle's match list."""
    from oracle_lib import OracleDfa, gen
    s = streams["c2_512m"]
    n = s["bytes"]
    opc = patterns[s["pattern"]]["opc"]
    host = gen(s["kind"], 1, 0, n)
    cnt, dg, dc, lst = OracleDfa(opc).find(host, want_list=True)
    assert (cnt, dg, dc) == (s["count"], s["digest"], s["dcap"])  # oracle pinned to the reference
    ref = np.asarray(lst, dtype=np.uint64).reshape(-1, 3)
    cuts = []
    for k in range(1, 8):
        i = int(np.searchsorted(ref[:, 0], k * n // 8 + 12345 * k))
        cuts.append(int(ref[i, 0]) + 1 + (k & 1))  # strictly inside match i
    whole = _whole(U, s["kind"], n)
    pat = U.Pattern(opc)
    out, st, ln, cp = _sharded(U, pat, whole, n, cuts)
    assert out["fixes"] == 7
    assert (out["count"], out["digest"], out["dcap"]) == (s["count"], s["digest"], s["dcap"])
    assert np.array_equal(st.cpu().numpy().astype(np.uint64), ref[:, 0])
    assert np.array_equal(ln.cpu().numpy().astype(np.uint64), ref[:, 1])
    assert np.array_equal(cp.cpu().numpy().astype(np.uint64), ref[:, 2])


@pytest.mark.parametrize("name", ["c3_256m", "c4_128m"])
def test_dense_shards_arbitrary_cuts(U, patterns, streams, name):
    """C3 identifiers / C4 \\w+ streams (dense matches, xi/xg kernels) in 8
    shards cut at odd offsets (most land inside a match): stitched totals and the
    digests of the gathered records equal the reference's."""
    s = streams[name]
    n = s["bytes"]
    whole = _whole(U, s["kind"], n)
    pat = U.Pattern(patterns[s["pattern"]]["opc"])
    cuts = [k * n // 8 + 7919 * k + 3 for k in range(1, 8)]
    out, st, ln, cp = _sharded(U, pat, whole, n, cuts)
    want = (s["count"], s["digest"], s["dcap"])
    assert (out["count"], out["digest"], out["dcap"]) == want
    assert (st.numel(),) + _digests(st, ln, cp) == want
    assert out["fixes"] >= 1


def test_scan_shard_grows_the_halo(U):
    """A match longer than the halo (a 3 MiB run of `a` across the end of a
    4 MiB shard of digits, halo 64 KiB): dist.scan_shard grows the halo until
    the match ends inside it, and the shard's record is that one match.  Both
    a prefiltered table (`a+`: sparse_kernel, its long walk continued by the
    whole wave) and a dense one (`[a-z]+`: xc_kernel)."""
    from ugrep_amd.dist import scan_shard
    n = 8 << 20
    host = np.frombuffer(b"12 " * (n // 3 + 1), np.uint8)[:n].copy()
    host[3 << 20:6 << 20] = ord("a")
    whole = torch.from_numpy(host).to("cuda")

    def fetch(a, z):
        t = torch.zeros(z - a + 16, dtype=torch.uint8, device="cuda")
        t[:z - a].copy_(whole[a:z])
        torch.cuda.synchronize()
        return t

    for rx, kernel in (("a+", 0), ("[a-z]+", 5)):
        pat = U.Pattern(U.compile_regex(rx))
        assert pat.info()["kernel"] == kernel, rx
        sc = U.Scanner(pat)
        rec, buf, rend = scan_shard(sc, fetch, 0, 4 << 20, n, halo=64 << 10, stream=_stream())
        assert rend > 6 << 20  # (grown from 64 KiB past the end of the run; the exit must lie before it)
        # the one match of the shard: (3 MiB, 3 MiB, accept 1)
        s0 = 3 << 20
        assert (rec["count"], rec["digest"], rec["dcap"]) == (1, 31 * s0 + s0, s0 + 1), rx
        assert rec["exit"] == 6 << 20, rx


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c4_128m", "c3_256m"])
def test_offsets_record_by_record(U, patterns, streams, name):
    """The records of the table's own OFFSETS pass (C4: xc_kernel's U mode,
    xu_kernel + xu_write_kernel; C3: xc_kernel) over the whole stream, record
    by record against the oracle's match list (which is pinned to the
    reference's totals)."""
    from oracle_lib import OracleDfa, gen
    s = streams[name]
    n = s["bytes"]
    opc = patterns[s["pattern"]]["opc"]
    host = gen(s["kind"], 1, 0, n)
    o = OracleDfa(opc)
    ws, wl, wc = o.find_arrays(host)
    assert ws.size == s["count"]
    whole = _whole(U, s["kind"], n)
    res = U.find_all(U.Pattern(opc), whole[:n], offsets=True)
    assert (res.count, res.digest, res.dcap) == (s["count"], s["digest"], s["dcap"])
    assert np.array_equal(np.asarray(res.start, np.uint64), ws)
    assert np.array_equal(np.asarray(res.length, np.uint64), wl)
    assert np.array_equal(np.asarray(res.cap, np.uint64), wc)


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _rank(rank, world, port, opc, s, q):
    """One rank of the multi-process run: its own shard generated on the card,
    the HIP Scanner, dist.stitch and gather_offsets over gloo."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch as T
        import ugrep_amd as U
        from ugrep_amd.dist import gather_offsets, shard_bounds, stitch
        T.cuda.set_device(0)
        st_ = T.cuda.current_stream().cuda_stream
        lo, hi, read_end, eof = shard_bounds(s["bytes"], world, rank, HALO)
        buf = T.empty(read_end - lo + 16, dtype=T.uint8, device="cuda")
        U.gen(s["kind"], 1, lo, buf.data_ptr(), read_end - lo, st_)
        sc = U.Scanner(U.Pattern(opc))
        sc.scan(buf.data_ptr(), 0, hi - lo, read_end - lo, eof, lo, st_)
        t = sc.totals()

        def fix_fn(old, new):
            d = sc.chain_fix(buf.data_ptr(), 0, hi - lo, read_end - lo, eof, lo, old - lo, new - lo, st_)
            return dict(count=d.count, digest=d.digest, dcap=d.dcap, exit=None if d.exit == M64 else d.exit + lo)

        out = stitch(dict(entry=t.entry + lo, exit=t.exit + lo, count=t.count, digest=t.digest, dcap=t.dcap), fix_fn)
        cnt = t.count
        if out["entries"][rank] != lo:
            sc.scan(buf.data_ptr(), min(out["entries"][rank], hi) - lo, hi - lo, read_end - lo, eof, lo, st_)
            cnt = sc.totals().count
        a = T.empty(max(cnt, 1), dtype=T.int64, device="cuda")
        b = T.empty(max(cnt, 1), dtype=T.int32, device="cuda")
        c = T.empty(max(cnt, 1), dtype=T.int32, device="cuda")
        if cnt:
            sc.offsets(a.data_ptr(), b.data_ptr(), c.data_ptr(), cnt, st_)
        g = gather_offsets(a[:cnt].cpu(), b[:cnt].cpu(), c[:cnt].cpu(), dst=0)
        res = dict(out=out, n=None, dg=None)
        if g is not None:
            res["n"] = int(g[0].numel())
            res["dg"] = _digests(*g)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_multiprocess_gloo_four_ranks(U, patterns, streams):
    """Four processes on the one card, each scanning its own 64 MiB shard of the
    256 MiB C3 stream with the HIP Scanner, stitched with dist.stitch (gloo
    all_gather + broadcast of ugpu_chain_fix corrections) and the records
    gathered to rank 0: everything equals the reference."""
    import torch.multiprocessing as mp
    s = streams["c3_256m"]
    opc = patterns[s["pattern"]]["opc"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_rank, args=(r, world, port, opc, s, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = (s["count"], s["digest"], s["dcap"])
    for r in range(world):
        o = res[r]["out"]
        assert (o["count"], o["digest"], o["dcap"]) == want, r
    assert (res[0]["n"],) + tuple(res[0]["dg"]) == want


def _halo_stream(n):
    """"12 " filler; 'q' | 'x' 'a' + 6 MiB of 'b' across the 4 MiB cut
    (tests/test_dist_halo.py's case)."""
    mib = 1 << 20
    data = np.frombuffer(b"12 " * (n // 3 + 1), np.uint8)[:n].copy()
    data[4 * mib - 1] = ord("q")
    data[4 * mib] = ord("x")
    data[4 * mib + 1] = ord("a")
    data[4 * mib + 2:10 * mib + 2] = ord("b")
    return data


def _halo_rank(rank, world, port, opc, q):
    """One rank of the HALO case: dist.Shard over the HIP Scanner, stitch over gloo."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch as T
        import ugrep_amd as U
        from ugrep_amd.dist import Shard, shard_bounds, stitch
        T.cuda.set_device(0)
        st_ = T.cuda.current_stream().cuda_stream
        data = _halo_stream(16 << 20)
        lo, hi, _, _ = shard_bounds(data.size, world, rank, 64 << 10)

        def fetch(a, z):
            t = T.zeros(z - a + 16, dtype=T.uint8, device="cuda")
            t[:z - a].copy_(T.from_numpy(data[a:z]))
            T.cuda.synchronize()
            return t

        sh = Shard(U.Scanner(U.Pattern(opc)), fetch, lo, hi, data.size, 64 << 10, stream=st_)
        out = stitch(sh.scan(), sh.fix)
        cnt = sh.scan(out["entries"][rank])["count"] if out["entries"][rank] != lo else out["counts"][rank]
        q.put((rank, dict(out=out, grown=sh.grown, cnt=cnt)))
    finally:
        dist.destroy_process_group()


def test_multiprocess_fix_grows_the_halo(U):
    """four processes on the one card, xa|ab+|qx, a 6 MiB
    run of 'b' right after the first cut and a 64 KiB halo: rank 1's TRUE
    chain (entered after shard 0's "qx") walks the 6 MiB "ab+" match past its
    halo, ugpu_chain_fix fails with UGPU_HALO, and dist.Shard grows the halo on
    that rank before the broadcast.  Totals equal the oracle's."""
    import torch.multiprocessing as mp
    from oracle_lib import OracleDfa
    opc = U.compile_regex("xa|ab+|qx")
    data = _halo_stream(16 << 20)
    want = OracleDfa(opc).find(data)[:3]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_halo_rank, args=(r, world, port, opc, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        o = res[r]["out"]
        assert (o["count"], o["digest"], o["dcap"]) == want, r
    assert res[1]["grown"] >= 1
    assert sum(res[r]["cnt"] for r in range(world)) == want[0]
