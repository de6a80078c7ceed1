"""CPU (gloo, world_size 8): the driver's 8-GPU layout rehearsed with one
process per rank.  The stream is cut into 8 shards, every
cut inside a match (C3 identifiers, and one 3 MiB identifier that runs past its
shard's 64 KiB halo, so that rank's scan grows the halo); ugrep_amd.dist.Shard
+ stitch() resolve the true chain, the OFFSETS records stay on their ranks and
only their sums travel (dist.verify_sharded), and a failing owner makes every
rank raise instead of leaving the others blocked in a collective.

Each rank's scanner is the CPU stand-in of tests/test_dist_halo.py (the
engine's interface and HALO rule on the oracle restatement)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dist_halo import OracleScanner, _free_port

WORLD = 8
MIB = 1 << 20


def _stream_bytes():
    """8 MiB of the C3 corpus with every 1 MiB cut inside an identifier, and a
    3 MiB identifier from 2.5 MiB on (across the cuts at 3 and 4 MiB)."""
    from oracle_lib import gen
    n = 8 * MIB
    data = gen(3, 71, 0, n)
    for r in range(1, WORLD):
        c = r * MIB
        data[c - 5:c + 5] = np.frombuffer(b"identifier", np.uint8)
    data[5 * MIB // 2 - 1] = ord(" ")
    data[5 * MIB // 2:11 * MIB // 2] = ord("x")
    data[11 * MIB // 2] = ord(" ")
    return data


def _worker(rank, world, port, opc, halo, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle_lib import OracleDfa
        from ugrep_amd.dist import Shard, shard_bounds, stitch, verify_sharded
        data = _stream_bytes()
        lo, hi, _, _ = shard_bounds(data.size, world, rank, halo)

        def fetch(a, z):
            return torch.from_numpy(np.concatenate([data[a:z], np.zeros(16, np.uint8)]))

        sc = OracleScanner(opc, data, fail_fix=(rank == fail_rank))
        sh = Shard(sc, fetch, lo, hi, data.size, halo)
        rec = sh.scan()
        try:
            out = stitch(rec, sh.fix)
        except Exception as e:  # noqa: BLE001
            q.put((rank, {"raised": type(e).__name__}))
            return
        # this rank's true records: its chain from the true entry, starts < hi
        ent = out["entries"][rank]
        lst = [] if ent >= hi else [m for m in OracleDfa(opc).find(data, start=ent, want_list=True)[3] if m[0] < hi]
        st = torch.tensor([m[0] for m in lst], dtype=torch.int64)
        ln = torch.tensor([m[1] for m in lst], dtype=torch.int32)
        cp = torch.tensor([m[2] for m in lst], dtype=torch.int32)
        ver = verify_sharded(st, ln, cp, out)
        q.put((rank, {"out": out, "grown": sh.grown, "ver": ver, "n": len(lst)}))
    finally:
        dist.destroy_process_group()


def _run(opc, halo, fail_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, opc, halo, fail_rank, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.fixture(scope="module")
def opc():
    import ugrep_amd
    return ugrep_amd.compile_regex("[A-Za-z_][A-Za-z0-9_]*|[0-9]+")


def test_world8_stitch_halo_and_sharded_records(opc):
    from oracle_lib import OracleDfa
    data = _stream_bytes()
    cnt, dg, dc, lst = OracleDfa(opc).find(data, want_list=True)
    assert any(m[0] == 5 * MIB // 2 and m[1] == 3 * MIB for m in lst)  # (the 3 MiB identifier)
    res = _run(opc, 64 << 10)
    for r in range(WORLD):
        o = res[r]["out"]
        assert (o["count"], o["digest"], o["dcap"]) == (cnt, dg, dc), r
        assert res[r]["ver"]["ok"] and res[r]["ver"]["count"] == cnt, (r, res[r]["ver"])
    # every cut lies inside a match: every rank after the first was re-entered
    assert res[0]["out"]["fixes"] == WORLD - 1
    # the rank whose shard ends inside the 3 MiB identifier grew its halo
    assert res[2]["grown"] >= 1
    assert sum(res[r]["n"] for r in range(WORLD)) == cnt
    # ranks 3 and 4 lie inside the long match: no records of their own
    assert res[3]["n"] == 0 and res[4]["n"] == 0


def test_world8_failing_owner(opc):
    res = _run(opc, 64 << 10, fail_rank=5)
    assert res[5] == {"raised": "UgpuError"}
    for r in range(WORLD):
        if r != 5:
            assert res[r] == {"raised": "ShardError"}, r
