"""Multi-GPU sharding of one logical buffer.

One process per GPU.  Rank r scans the contiguous shard [r*S, (r+1)*S) of the
stream (plus a read-only halo past its end so that a match crossing the shard
end can finish), speculating that the FIND chain enters at its shard start.
The ranks then exchange one small record each (all_gather over RCCL/xGMI):

    (entry, exit, count, digest, dcap)

and resolve the true chain left to right: rank r's speculative entry is
correct iff exit(r-1) == entry(r).  Otherwise rank r re-enters its shard at
exit(r-1) (ugpu_chain_fix, a lock-step merge of the two chains that normally
ends within a few bytes) and broadcasts the correction.  For patterns that
cannot match '\\n' and newline-aligned shards no correction is ever needed;
arbitrary cut points are handled exactly.

The reference has no counterpart (one buffer is always scanned by one thread,
src/ugrep.cpp:4118-4480); this is new design.  The protocol is pure host logic
over torch.distributed, tested with gloo on CPU (tests/test_dist.py).
"""
import numpy as np
import torch
import torch.distributed as dist

MASK64 = (1 << 64) - 1


def _to_i64(v):
    return int(np.array([v & MASK64], dtype=np.uint64).view(np.int64)[0])


def _to_u64(v):
    return int(np.array([v], dtype=np.int64).view(np.uint64)[0])


def stitch(rec, fix_fn, device="cpu", group=None):
    """Resolve shard records into exact totals.

    rec    : dict(entry, exit, count, digest, dcap) of this rank's shard, positions global.
    fix_fn : fix_fn(old_entry, new_entry) -> dict(count, digest, dcap, exit) correction for
             THIS rank's shard (exit None if unchanged); only called on the rank that owns it.
    Returns dict(count, digest, dcap, exit, fixes) identical on every rank.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    keys = ("entry", "exit", "count", "digest", "dcap")
    mine = torch.tensor([_to_i64(rec[k]) for k in keys], dtype=torch.int64, device=device)
    allrec = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allrec, mine, group=group)
    recs = [dict(zip(keys, (_to_u64(int(x)) for x in t.cpu().tolist()))) for t in allrec]
    fixes = 0
    prev_exit = recs[0]["exit"]
    for r in range(1, world):
        if prev_exit != recs[r]["entry"]:
            fixes += 1
            buf = torch.zeros(5, dtype=torch.int64, device=device)
            if rank == r:
                d = fix_fn(recs[r]["entry"], prev_exit)
                ex = d.get("exit")
                buf = torch.tensor([_to_i64(d["count"]), _to_i64(d["digest"]), _to_i64(d["dcap"]),
                                    1 if ex is not None else 0, _to_i64(ex if ex is not None else 0)],
                                   dtype=torch.int64, device=device)
            dist.broadcast(buf, src=r, group=group)
            v = [_to_u64(int(x)) for x in buf.cpu().tolist()]
            recs[r]["count"] = (recs[r]["count"] + v[0]) & MASK64
            recs[r]["digest"] = (recs[r]["digest"] + v[1]) & MASK64
            recs[r]["dcap"] = (recs[r]["dcap"] + v[2]) & MASK64
            recs[r]["entry"] = prev_exit
            if v[3]:
                recs[r]["exit"] = v[4]
        prev_exit = recs[r]["exit"]
    out = dict(count=0, digest=0, dcap=0, exit=prev_exit, fixes=fixes)
    for r in recs:
        out["count"] = (out["count"] + r["count"]) & MASK64
        out["digest"] = (out["digest"] + r["digest"]) & MASK64
        out["dcap"] = (out["dcap"] + r["dcap"]) & MASK64
    return out


def shard_bounds(total, world, rank, halo):
    """[lo, hi) of rank's shard, its readable end, and whether that is the stream end."""
    per = total // world
    lo = rank * per
    hi = total if rank == world - 1 else lo + per
    read_end = min(total, hi + halo)
    return lo, hi, read_end, read_end == total
