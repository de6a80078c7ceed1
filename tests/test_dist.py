"""CPU (gloo, world_size 2 and 3): the shard-stitch protocol of ugrep_amd.dist.

Each rank 'scans' its shard with the oracle restatement (test infrastructure
standing in for the GPU scanner) and stitches through torch.distributed; the
stitched totals must equal one sequential scan, for cut points that split
matches and for a chain that never re-synchronises."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, opc, data, halo, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle_lib import OracleDfa
        from ugrep_amd.dist import shard_bounds, stitch
        d = OracleDfa(opc)
        lo, hi, read_end, eof = shard_bounds(len(data), world, rank, halo)
        view = data[:read_end]
        # speculative scan of [lo, hi) entered at lo: matches starting in [lo, hi)
        cnt, dg, dc, lst = d.find(view[:read_end], start=lo, want_list=True)
        sel = [m for m in lst if m[0] < hi]
        # chain restricted to starts < hi: recompute totals on the selection
        cnt = len(sel)
        dg = sum(m[0] * 31 + m[1] for m in sel) & ((1 << 64) - 1)
        dc = sum((m[0] + 1) * m[2] for m in sel) & ((1 << 64) - 1)
        ex = d.chain_exit(view, lo, hi)

        def fix_fn(old, new):
            _, _, _, l2 = d.find(view, start=new, want_list=True)
            s2 = [m for m in l2 if m[0] < hi]
            ex2 = d.chain_exit(view, new, hi)
            return dict(count=(len(s2) - cnt) & ((1 << 64) - 1),
                        digest=(sum(m[0] * 31 + m[1] for m in s2) - dg) & ((1 << 64) - 1),
                        dcap=(sum((m[0] + 1) * m[2] for m in s2) - dc) & ((1 << 64) - 1),
                        exit=ex2 if ex2 != ex else None)

        out = stitch(dict(entry=lo, exit=ex, count=cnt, digest=dg, dcap=dc), fix_fn)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(world, opc, data, halo=1 << 16):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, opc, data, halo, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs = [o for _, o in sorted(res)]
    assert all(o == outs[0] for o in outs)
    return outs[0]


@pytest.mark.parametrize("world", [2, 3])
def test_stitch_identifiers(patterns, world):
    from oracle_lib import OracleDfa, gen
    data = gen(3, 21, 0, 300007)  # shard cuts land inside identifiers
    opc = patterns["c3_ident"]["opc"]
    out = _run(world, opc, data)
    cnt, dg, dc, _ = OracleDfa(opc).find(data)
    assert (out["count"], out["digest"], out["dcap"]) == (cnt, dg, dc)


def test_stitch_nonsynchronising(patterns):
    from oracle_lib import OracleDfa
    data = np.full(200001, ord("a"), np.uint8)
    data[0] = ord("b")
    opc = patterns["aa"]["opc"]
    out = _run(2, opc, data, halo=16)
    cnt, dg, dc, _ = OracleDfa(opc).find(data)
    assert (out["count"], out["digest"], out["dcap"]) == (cnt, dg, dc)
    assert out["fixes"] == 1


def _gather_worker(rank, world, port, recs, dst, q, no_cap=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from ugrep_amd.dist import gather_offsets
        mine = np.asarray(recs[rank], dtype=np.int64).reshape(-1, 3)
        out = gather_offsets(torch.from_numpy(mine[:, 0].copy()), torch.from_numpy(mine[:, 1].astype(np.int32)),
                             None if no_cap else torch.from_numpy(mine[:, 2].astype(np.int32)), dst=dst)
        q.put((rank, None if out is None else [None if t is None else t.tolist() for t in out]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dst,no_cap", [(2, None, False), (3, None, False), (3, 1, False), (3, None, True)])
def test_gather_offsets(patterns, world, dst, no_cap):
    """Per-shard records of the true chain, exchanged, equal one sequential scan's
    list (no_cap: 12-byte records, one accept index)."""
    from oracle_lib import OracleDfa, gen
    from ugrep_amd.dist import shard_bounds
    data = gen(3, 5, 0, 50021)
    opc = patterns["c3_ident"]["opc"]
    _, _, _, lst = OracleDfa(opc).find(data, want_list=True)
    recs = []
    for r in range(world):
        lo, hi, _, _ = shard_bounds(len(data), world, r, 0)
        recs.append([m for m in lst if lo <= m[0] < hi])
    recs[1] = []  # an empty shard on the way
    want = [m for r in recs for m in r]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, recs, dst, q, no_cap)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        if dst is not None and r != dst:
            assert res[r] is None
            continue
        s, ln, cp = res[r]
        if no_cap:
            assert cp is None
            assert [list(t) for t in zip(s, ln)] == [m[:2] for m in want]
        else:
            assert [list(t) for t in zip(s, ln, cp)] == [list(m) for m in want]
