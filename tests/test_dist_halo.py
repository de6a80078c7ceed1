"""CPU (gloo, world_size 3): the multi-process stitch when the TRUE chain walks
past a shard's readable end.

Pattern xa|ab+|qx; shard 0 ends with 'q', shard 1 starts with "xa" followed by
a 6 MiB run of 'b'.  Rank 1's speculative chain reads "xa" and never needs its
64 KiB halo; the true chain enters at the 'a' (shard 0's "qx" ends there) and
walks the 6 MiB "ab+" match past the halo, so ugpu_chain_fix fails with
UGPU_HALO.  dist.Shard grows the halo on the owner rank and retries before the
broadcast; the stitched totals must equal one sequential scan, and the run must
end inside the timeout.  A fix that fails for good must make every rank raise
(the failure travels in the broadcast), not leave the others blocked in it.

Each rank's scanner is a CPU stand-in with the engine's interface and its HALO
rule, built on the oracle restatement (test infrastructure)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

M64 = (1 << 64) - 1
MIB = 1 << 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream_bytes():
    """12 MiB: "12 " filler, 'q' | 'x' 'a' + 6 MiB of 'b' across the 4 MiB cut."""
    n = 12 * MIB
    data = np.frombuffer(b"12 " * (n // 3 + 1), np.uint8)[:n].copy()
    data[4 * MIB - 1] = ord("q")
    data[4 * MIB] = ord("x")
    data[4 * MIB + 1] = ord("a")
    data[4 * MIB + 2:10 * MIB + 2] = ord("b")
    return data


class _T:
    """ugpu_scan_totals' fields."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class OracleScanner:
    """The Scanner interface used by dist.Shard (scan / totals / chain_fix) on
    the oracle.  Positions handed in are buffer-relative (bias = the buffer's
    first stream position), as the engine's are.  The engine's HALO rule: on a
    buffer that does not end at EOF, a match of the chain, or the chain exit,
    that reaches the readable end raises UGPU_HALO."""

    def __init__(self, opc, data, fail_fix=False):
        from oracle_lib import OracleDfa
        self.d = OracleDfa(opc)
        self.data = data
        self.fail_fix = fail_fix
        self.t = None

    def _chain(self, entry, hi, rend, eof):
        from ugrep_amd._lib import UGPU_HALO, UgpuError
        _, _, _, lst = self.d.find(self.data, start=entry, want_list=True)
        sel = [m for m in lst if m[0] < hi]
        ex = self.d.chain_exit(self.data, entry, hi)
        if not eof and (ex >= rend or any(m[0] + m[1] >= rend for m in sel)):
            raise UgpuError(UGPU_HALO, "match runs past the readable end")
        cnt = len(sel)
        dg = sum(31 * m[0] + m[1] for m in sel) & M64
        dc = sum((m[0] + 1) * m[2] for m in sel) & M64
        return cnt, dg, dc, ex

    def scan(self, ptr, lo, hi, rend, eof, bias, stream=0):
        cnt, dg, dc, ex = self._chain(bias + lo, bias + hi, bias + rend, eof)
        self.t = _T(count=cnt, digest=dg, dcap=dc, entry=lo, exit=ex - bias)

    def totals(self):
        return self.t

    def chain_fix(self, ptr, lo, hi, rend, eof, bias, old, new, stream=0):
        if self.fail_fix:
            from ugrep_amd._lib import UGPU_DEVICE, UgpuError
            raise UgpuError(UGPU_DEVICE, "injected failure")
        c0, d0, k0, e0 = self._chain(bias + old, bias + hi, bias + rend, eof)
        c1, d1, k1, e1 = self._chain(bias + new, bias + hi, bias + rend, eof)
        return _T(count=(c1 - c0) & M64, digest=(d1 - d0) & M64, dcap=(k1 - k0) & M64, entry=new,
                  exit=M64 if e1 == e0 else e1 - bias)


def _worker(rank, world, port, opc, halo, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ugrep_amd.dist import Shard, shard_bounds, stitch
        data = _stream_bytes()
        lo, hi, _, _ = shard_bounds(data.size, world, rank, halo)
        fetched = []

        def fetch(a, z):
            fetched.append(z - a)
            return torch.from_numpy(np.concatenate([data[a:z], np.zeros(16, np.uint8)]))

        sc = OracleScanner(opc, data, fail_fix=(rank == fail_rank))
        sh = Shard(sc, fetch, lo, hi, data.size, halo)
        rec = sh.scan()
        try:
            out = stitch(rec, sh.fix)
        except Exception as e:  # noqa: BLE001
            q.put((rank, {"raised": type(e).__name__}))
            return
        # the OFFSETS pass's true-entry re-scan (bench.py step): same buffer, no HALO left
        cnt = sh.scan(out["entries"][rank])["count"] if out["entries"][rank] != lo else out["counts"][rank]
        q.put((rank, {"out": out, "grown": sh.grown, "read_end": sh.read_end, "fetched": fetched, "cnt": cnt}))
    finally:
        dist.destroy_process_group()


def _run(world, opc, halo, fail_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, opc, halo, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.fixture(scope="module")
def opc():
    import ugrep_amd
    return ugrep_amd.compile_regex("xa|ab+|qx")


def test_fix_grows_the_halo(opc):
    from oracle_lib import OracleDfa
    data = _stream_bytes()
    res = _run(3, opc, 64 << 10)
    cnt, dg, dc, lst = OracleDfa(opc).find(data, want_list=True)
    assert any(m[0] == 4 * MIB + 1 and m[1] == 6 * MIB + 1 for m in lst)  # (the 6 MiB "ab+" match)
    for r in range(3):
        o = res[r]["out"]
        assert (o["count"], o["digest"], o["dcap"]) == (cnt, dg, dc), r
    assert res[0]["grown"] == 0
    assert res[1]["grown"] >= 1 and res[1]["read_end"] > 10 * MIB + 2  # (grown by the chain fix)
    assert res[1]["out"]["fixes"] == 2  # (rank 1 re-entered after "qx", rank 2 after the 6 MiB match)
    # per-shard true counts (records re-scan) add up to the whole stream's
    assert sum(res[r]["cnt"] for r in range(3)) == cnt


def test_failed_fix_raises_on_every_rank(opc):
    res = _run(3, opc, 64 << 10, fail_rank=1)
    assert res[1] == {"raised": "UgpuError"}
    assert res[0] == {"raised": "ShardError"} and res[2] == {"raised": "ShardError"}
