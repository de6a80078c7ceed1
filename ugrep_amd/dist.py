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


KEYS = ("entry", "exit", "count", "digest", "dcap")


class ShardError(RuntimeError):
    """Raised on every rank when one rank's shard correction failed."""


def resolve(recs, fix):
    """Resolve per-shard chain records, left to right, into exact totals.

    recs : list of dict(entry, exit, count, digest, dcap), one per shard in
           stream order, positions global, each scanned speculatively from
           its shard start (entry).
    fix  : fix(r, old_entry, new_entry) -> dict(count, digest, dcap, exit) with
           the correction for shard r re-entered at new_entry (exit None when
           unchanged: the two chains met inside the shard).
    Shard r's speculative entry is right iff exit(r-1) == entry(r); otherwise r
    is re-entered at exit(r-1), and a changed exit carries the correction on
    to r+1.  Returns dict(count, digest, dcap, exit, fixes, entries, counts).
    This is the whole protocol; stitch() runs it over torch.distributed and the
    tests drive it in-process as well.
    """
    recs = [dict(r) for r in recs]
    fixes = 0
    prev_exit = recs[0]["exit"]
    for r in range(1, len(recs)):
        if prev_exit != recs[r]["entry"]:
            fixes += 1
            d = fix(r, recs[r]["entry"], prev_exit)
            recs[r]["count"] = (recs[r]["count"] + d["count"]) & MASK64
            recs[r]["digest"] = (recs[r]["digest"] + d["digest"]) & MASK64
            recs[r]["dcap"] = (recs[r]["dcap"] + d["dcap"]) & MASK64
            recs[r]["entry"] = prev_exit
            if d.get("exit") is not None:
                recs[r]["exit"] = d["exit"]
        prev_exit = recs[r]["exit"]
    out = dict(count=0, digest=0, dcap=0, exit=prev_exit, fixes=fixes,
               entries=[r["entry"] for r in recs], counts=[r["count"] for r in recs])
    for r in recs:
        out["count"] = (out["count"] + r["count"]) & MASK64
        out["digest"] = (out["digest"] + r["digest"]) & MASK64
        out["dcap"] = (out["dcap"] + r["dcap"]) & MASK64
    return out


def stitch(rec, fix_fn, device="cpu", group=None):
    """Resolve shard records into exact totals across ranks (one all_gather).

    rec    : dict(entry, exit, count, digest, dcap) of this rank's shard, positions global.
    fix_fn : fix_fn(old_entry, new_entry) -> dict(count, digest, dcap, exit) correction for
             THIS rank's shard (exit None if unchanged); only called on the rank that owns it,
             whose result is broadcast to the others.
    Returns resolve()'s dict, identical on every rank; entries[r] / counts[r] are
    shard r's true chain entry and match count (a rank whose entry moved re-scans
    from it to materialise its records).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = torch.tensor([_to_i64(rec[k]) for k in KEYS], dtype=torch.int64, device=device)
    allrec = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allrec, mine, group=group)
    recs = [dict(zip(KEYS, (_to_u64(int(x)) for x in t.cpu().tolist()))) for t in allrec]

    def fix(r, old, new):
        # [count, digest, dcap, exit known, exit, failed]: the owner's failure
        # travels in the same broadcast, so that no rank is left blocked in a
        # collective when fix_fn raises; every rank then raises
        buf = torch.zeros(6, dtype=torch.int64, device=device)
        err = None
        if rank == r:
            try:
                d = fix_fn(old, new)
                ex = d.get("exit")
                buf = torch.tensor([_to_i64(d["count"]), _to_i64(d["digest"]), _to_i64(d["dcap"]),
                                    1 if ex is not None else 0, _to_i64(ex if ex is not None else 0), 0],
                                   dtype=torch.int64, device=device)
            except Exception as e:  # noqa: BLE001 - re-raised below, after the broadcast
                err = e
                buf[5] = 1
        # owner ranks r are visited in the same order on every rank
        dist.broadcast(buf, src=r, group=group)
        v = [_to_u64(int(x)) for x in buf.cpu().tolist()]
        if v[5]:
            if err is not None:
                raise err
            raise ShardError("rank %d failed to re-enter its shard at %d (see that rank's error)" % (r, new))
        return dict(count=v[0], digest=v[1], dcap=v[2], exit=v[4] if v[3] else None)

    return resolve(recs, fix)


class Shard:
    """One rank's shard [lo, hi) of a total-byte stream, in its own buffer
    [lo, read_end), with every engine call that can meet UGPU_HALO retried on
    a grown halo.

    A match longer than the halo makes a scan fail with UGPU_HALO,
    and so does ugpu_chain_fix when the TRUE chain (re-entered at the previous
    shard's exit) walks into a match the speculative chain never saw.  Both
    are handled here, on the owner rank, before any collective: the halo is
    doubled, the shard fetched again, and the call repeated, up to the stream
    end (where no match can run past).  fetch(lo, read_end) -> a uint8 CUDA
    tensor holding the stream's bytes [lo, read_end) (with the 16 bytes of
    padding the engine may read past them).  After a grown halo, .buf /
    .ptr / .read_end name the new buffer: callers read them per call."""

    def __init__(self, scanner, fetch, lo, hi, total, halo=1 << 20, stream=0):
        self.sc, self.fetch, self.lo, self.hi, self.total = scanner, fetch, lo, hi, total
        self.halo = max(int(halo), 1)
        self.stream = stream
        self.grown = 0
        self._load()

    def _load(self):
        self.read_end = min(self.total, self.hi + self.halo)
        self.eof = self.read_end == self.total
        self.buf = None  # (release the old buffer before fetching the larger one)
        self.buf = self.fetch(self.lo, self.read_end)
        self.ptr = self.buf.data_ptr()

    def _retry(self, call):
        from ._lib import UGPU_HALO, UgpuError
        while True:
            try:
                return call()
            except UgpuError as err:
                if err.code != UGPU_HALO or self.eof:
                    raise
                self.halo *= 2
                self.grown += 1
                self._load()

    def scan(self, entry=None):
        """Scan [max(entry, lo), hi) (entry None: lo; an entry at or past hi
        scans nothing: the previous shard's last match covers this shard);
        returns stitch()'s record, positions global."""
        e = self.lo if entry is None else min(max(entry, self.lo), self.hi)

        def go():
            self.sc.scan(self.ptr, e - self.lo, self.hi - self.lo, self.read_end - self.lo, self.eof, self.lo,
                         self.stream)
            return self.sc.totals()
        t = self._retry(go)
        return dict(entry=t.entry + self.lo, exit=t.exit + self.lo, count=t.count, digest=t.digest, dcap=t.dcap)

    def fix(self, old, new):
        """stitch()'s fix_fn: the correction for this shard re-entered at new
        instead of old (ugpu_chain_fix)."""
        def go():
            return self.sc.chain_fix(self.ptr, 0, self.hi - self.lo, self.read_end - self.lo, self.eof, self.lo,
                                     old - self.lo, new - self.lo, self.stream)
        t = self._retry(go)
        return dict(count=t.count, digest=t.digest, dcap=t.dcap,
                    exit=None if t.exit == MASK64 else t.exit + self.lo)


def scan_shard(scanner, fetch, lo, hi, total, halo=1 << 20, entry=None, stream=0):
    """Scan shard [lo, hi) of a total-byte stream from `entry` (default lo),
    growing the readable halo when a match runs past it (Shard).  Returns
    (record, buffer, read_end): the record in stitch()'s form with global
    positions, and the buffer and readable end the record was scanned on
    (fix_fn and the OFFSETS pass must use the same)."""
    sh = Shard(scanner, fetch, lo, hi, total, halo, stream)
    rec = sh.scan(entry)
    return rec, sh.buf, sh.read_end


def shard_bounds(total, world, rank, halo):
    """[lo, hi) of rank's shard, its readable end, and whether that is the stream end."""
    per = total // world
    lo = rank * per
    hi = total if rank == world - 1 else lo + per
    read_end = min(total, hi + halo)
    return lo, hi, read_end, read_end == total


def record_sums(start, length, cap=None):
    """(count, digest, dcap) of match records as u64 sums: digest = sum(31 start
    + len), dcap = sum((start + 1) cap) (0 when cap is None: 12-byte records)."""
    n = int(start.numel())
    if n == 0:
        return 0, 0, 0
    s64 = start.to(torch.int64)
    dg = int((s64 * 31 + length.to(torch.int64)).sum().item()) & MASK64  # (int64 sums wrap as u64)
    dc = int(((s64 + 1) * cap.to(torch.int64)).sum().item()) & MASK64 if cap is not None else 0
    return n, dg, dc


def verify_sharded(start, length, cap, totals, device="cpu", group=None):
    """OFFSETS without moving records: every rank keeps its own
    shard's records and only their sums travel -- one all_gather of 3 x u64
    per rank instead of the records themselves (8 x 15 GB for dense tables at
    8 ranks).  start / length / cap: this rank's records in chain order;
    totals: stitch()'s result.  Returns dict(count, digest, dcap, ok) with the
    sums over all ranks; ok when count and digest (and dcap, when cap is given
    on every rank) equal the stitched totals.  Identical on every rank."""
    world = dist.get_world_size(group)
    n, dg, dc = record_sums(start, length, cap)
    mine = torch.tensor([_to_i64(n), _to_i64(dg), _to_i64(dc), 1 if cap is not None else 0], dtype=torch.int64,
                        device=device)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    vals = [[_to_u64(int(x)) for x in t.cpu().tolist()] for t in parts]
    out = dict(count=sum(v[0] for v in vals) & MASK64, digest=sum(v[1] for v in vals) & MASK64,
               dcap=sum(v[2] for v in vals) & MASK64)
    ok = out["count"] == totals["count"] and out["digest"] == totals["digest"]
    if all(v[3] for v in vals):
        ok = ok and out["dcap"] == totals["dcap"]
    out["ok"] = ok
    return out


def gather_offsets(start, length, cap, group=None, dst=None, concat=True):
    """Exchange the final match records of every shard.

    start (int64, global byte offsets), length and cap (int32) are this rank's
    records in chain order, on the collective's device.  The records are
    packed 16 B each ((start, len << 32 | cap)) -- 12 B (start, len) when cap is
    None (tables with one accept index) -- padded to the largest shard's
    count and exchanged with one all_gather (dst None: every rank gets the
    whole list) or one gather to rank dst (others get None); the result is the
    concatenation in rank order, which is global chain order because shards
    are contiguous and ordered.  RCCL has no all_gatherv; padding costs at most
    (world - 1) x the count spread, and the counts travel first in one
    8-byte all_gather.  concat=False returns the per-rank parts as lists
    (start, len, cap per rank, views into the received buffers) instead of
    one concatenation, which would double the receiver's record memory.

    Memory: a receiver holds world x max(count) x (12 or 16) B.
    Dense tables at 8 x 16 GiB (C3: ~1.25 G records per shard, 12 B) make that
    ~120 GB at the root -- which is why the bench gathers to one root
    (dst=0) and never all-gathers records: an all_gather would put those
    120 GB on every rank.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = start.device
    n = torch.tensor([start.numel()], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    counts = [int(x.item()) for x in ns]
    m = max(max(counts), 1)
    k = counts[rank]
    if cap is None:
        pack = torch.zeros((m, 3), dtype=torch.int32, device=dev)
        if k:
            pack[:k, 0:2] = start[:k].to(torch.int64).contiguous().view(torch.int32).view(k, 2)
            pack[:k, 2] = length[:k].to(torch.int32)
    else:
        pack = torch.zeros((m, 2), dtype=torch.int64, device=dev)
        if k:
            pack[:k, 0] = start[:k].to(torch.int64)
            pack[:k, 1] = (length[:k].to(torch.int64) << 32) | (cap[:k].to(torch.int64) & 0xFFFFFFFF)
    if dst is None:
        parts = [torch.empty_like(pack) for _ in range(world)]
        dist.all_gather(parts, pack, group=group)
    else:
        parts = [torch.empty_like(pack) for _ in range(world)] if rank == dst else None
        dist.gather(pack, parts, dst=dst, group=group)
        if rank != dst:
            return None
    if not concat:
        ps = [parts[r][:counts[r]] for r in range(world)]
        if cap is None:
            return ([p[:, 0:2].contiguous().view(torch.int64).reshape(-1) for p in ps], [p[:, 2] for p in ps], None)
        return ([p[:, 0] for p in ps], [(p[:, 1] >> 32).to(torch.int32) for p in ps],
                [(p[:, 1] & 0xFFFFFFFF).to(torch.int32) for p in ps])
    allp = torch.cat([parts[r][:counts[r]] for r in range(world)])
    if cap is None:
        st = allp[:, 0:2].contiguous().view(torch.int64).reshape(-1)
        return st, allp[:, 2].clone(), None
    return allp[:, 0].clone(), (allp[:, 1] >> 32).to(torch.int32), (allp[:, 1] & 0xFFFFFFFF).to(torch.int32)
