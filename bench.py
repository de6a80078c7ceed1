#!/usr/bin/env python3
"""Benchmark of the FIND hot path (BASELINE.json metric: GB/s scanned + matches/s).

One step = one whole-buffer FIND pass (scan kernel + stitch kernel, match count
and digests) over this GPU's resident 16 GiB shard of a synthetic stream.  With
N GPUs (torchrun, one process per GPU, RCCL), rank r owns shard r of one logical
stream of N x 16 GiB (weak scaling) and the shard chains are stitched with one
all_gather per step (ugrep_amd/dist.py).  Inputs are generated on the device
before timing; H2D copies are not part of any timed number.

Default workload = BASELINE configs[1]: C2 'foo|bar|baz' over 16 GiB synthetic
ASCII words on 1 MI355X.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# the engine (libugrep_amd.so) is loaded by main() after the launcher decision,
# so that a parent that only starts the rank processes never loads HIP code
ugrep_amd = gather_offsets = Shard = shard_bounds = stitch = None

METRIC = "GB/s scanned + matches/s, 16 GiB synthetic buffer, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)

CONFIGS = {
    # name: (pattern key, ugrep mode/regex, corpus kind, default bytes per GPU, description)
    "c1": ("c1_lorem", "F", "lorem", 0, 64 << 20, "-F 'lorem' over tests/lorem.utf8.txt tiled to 64 MiB"),
    "c2": ("c2_foobarbaz", "re", "foo|bar|baz", 1, 16 << 30,
           "3-literal alternation 'foo|bar|baz' over 16 GiB synthetic ASCII words"),
    "c2p": ("c2_foobarbaz", "re", "foo|bar|baz", 2, 16 << 30,
            "'foo|bar|baz' over 16 GiB planted known-answer corpus"),
    "c3": ("c3_ident", "re", "[A-Za-z_][A-Za-z0-9_]*", 3, 16 << 30,
           "identifier ERE over 16 GiB synthetic source-code corpus"),
    "c4": ("c4_word", "re", r"\w+", 4, 8 << 30, "Unicode \\w+ over 8 GiB synthetic UTF-8 words"),
    # C5's whole stream: 128 GiB in total, cut into one shard per rank (strong
    # scaling; with --gpus 8 each rank scans 16 GiB, as the weak-scaling c2 line)
    "c5": ("c2_foobarbaz", "re", "foo|bar|baz", 1, 128 << 30,
           "'foo|bar|baz' over one 128 GiB synthetic ASCII stream, sharded across the ranks"),
}
STRONG = {"c5"}  # configs whose size is the whole job's, not per GPU


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def _harness(exe, mode, rx, spec, threads, reps):
    out = subprocess.run([exe, "bench", mode, rx, spec, str(threads), str(reps)], capture_output=True,
                         timeout=900, check=True).stdout.decode()
    return json.loads(out.strip().splitlines()[-1])


def _spec(kind, sample):
    if kind == 0:
        return "file:%s:%d" % (os.path.join(REPO, "tests", "golden", "lorem.utf8.txt"), sample)
    return "gen:%d:1:0:%d" % (kind, sample)


def cpu_baseline(cfg, sample, threads, rx_override=None, word=False):
    """The reference CPU matcher on a bounded sample of the same corpus.

    `value` is the reference AVX2 path (oracle/_ref/ref_harness_avx2: libreflex
    compiled from the reference sources with -DHAVE_AVX2, BASELINE.json's
    "reference AVX2 CPU path") on all `threads` host cores, newline-split shards
    sharing one Pattern as ugrep's workers do (src/ugrep.cpp:4206).  Also
    reported: the same build on 1 core (on a smaller sample), and the
    AVX512BW-dispatching build on all cores.  Returns (baseline dict, the
    reference's count/digest/dcap of the whole sample) -- the latter is compared
    with the GPU scan of the same bytes.  Falls back to the oracle restatement
    ("port") when the reference build is absent."""
    pkey, mode, rx, kind, _, _ = CONFIGS[cfg]
    if rx_override is not None:
        mode, rx, pkey = "re", rx_override, None
    if word:
        mode += "W"  # (the harness's Matcher option W, ugrep -w)
    avx2 = os.path.join(REPO, "oracle", "_ref", "ref_harness_avx2")
    avx512 = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if os.path.exists(avx2):
        try:
            j = _harness(avx2, mode, rx, _spec(kind, sample), threads, 3)
            one_sample = min(sample, 1 << 30 if info_dense(cfg) else sample)
            j1 = _harness(avx2, mode, rx, _spec(kind, one_sample), 1, 2)
            out = dict(value=round(j["bytes"] / j["seconds"] / 1e9, 3), unit="GB/s", cores=threads, kind="reference",
                       build="AVX2 (-DHAVE_AVX2)",
                       sample="%d MiB of the same corpus (seed 1, bytes [0, %d)), reference libreflex Matcher::find() "
                              "loop, newline-split across %d threads (one GPU's share of the node's cores) sharing "
                              "one Pattern, best of 3; %d matches" % (sample >> 20, sample, threads, j["count"]),
                       one_core={"value": round(j1["bytes"] / j1["seconds"] / 1e9, 3), "unit": "GB/s",
                                 "sample_bytes": one_sample, "best_of": 2},
                       host_cpus_visible=len(os.sched_getaffinity(0)))
            if os.path.exists(avx512):
                j5 = _harness(avx512, mode, rx, _spec(kind, sample), threads, 3)
                out["avx512bw_build"] = {"value": round(j5["bytes"] / j5["seconds"] / 1e9, 3), "unit": "GB/s",
                                         "cores": threads}
            return out, (j["count"], j["digest"], j["dcap"])
        except Exception as e:  # pragma: no cover - diagnostic path
            log("reference harness failed (%s); using the oracle restatement" % e)
    if pkey is None or word:
        return None, None  # (no reference build: the restatement leg covers the BASELINE patterns only)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_lib import OracleDfa, gen as host_gen
    with open(os.path.join(REPO, "ugrep_amd", "data", "config_patterns.json")) as f:
        opc = json.load(f)[pkey]["opc"]
    buf = host_gen(kind, 1, 0, sample) if kind else np.frombuffer(
        (open(os.path.join(REPO, "tests", "golden", "lorem.utf8.txt"), "rb").read() * (sample // 9419 + 1))[:sample],
        np.uint8)
    d = OracleDfa(opc)
    best = 1e30
    for _ in range(2):
        t0 = time.perf_counter()
        d.find_mt(buf, threads)
        best = min(best, time.perf_counter() - t0)
    return dict(value=round(sample / best / 1e9, 3), unit="GB/s", cores=threads, kind="port",
                sample="%d MiB, oracle restatement (dense-table walker), %d threads" % (sample >> 20, threads)), None


def info_dense(cfg):
    """Configs the reference walks byte by byte (no SIMD prefilter): ~0.2 GB/s per core."""
    return cfg in ("c3", "c4")


def gpu_reference_check(pat, buf, sample, want, sptr):
    """Scan the cpu_baseline sample [0, sample) of this GPU's buffer as one whole
    buffer (EOF at its end, as the reference harness sees it) and compare
    count/digest/dcap with the reference's."""
    sc = ugrep_amd.Scanner(pat)
    sc.scan(buf.data_ptr(), 0, sample, sample, True, 0, sptr)
    t = sc.totals()
    got = (t.count, t.digest, t.dcap)
    return {"equal": got == tuple(want), "bytes": sample, "gpu": list(got), "reference": list(want),
            "fields": ["count", "digest", "dcap"]}


KERNELS = {0: "sparse_kernel", 1: "dense_kernel", 2: "xi_kernel", 3: "xg_kernel", 4: "wfind_kernel", 5: "xc_kernel",
           6: "xu_kernel"}  # (6: xc_kernel's U mode, code-point run tables)


def measured_traffic(cfg, nbytes, kernel):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/traffic.json, written from tools/profile.sh runs:
    FETCH_SIZE x 1024 x 2 on gfx950), when it was taken on this config and size."""
    try:
        with open(os.path.join(REPO, "profiles", "traffic.json")) as f:
            t = json.load(f).get(cfg)
    except (OSError, ValueError):
        return None
    if not t or t.get("algorithmic_bytes_per_launch") != nbytes or kernel not in t.get("kernel", ""):
        return None
    return t


def verify_whole(args, kind, total, pat, res, rank, dev, sptr):
    """Scan the whole logical stream [0, total) as one buffer on this GPU and
    compare count/digest/dcap with the stitched multi-shard result."""
    whole = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    if kind == 0:
        data = open(os.path.join(REPO, "tests", "golden", "lorem.utf8.txt"), "rb").read()
        tile = np.frombuffer(data, np.uint8)
        whole[:total].copy_(torch.from_numpy(tile[np.arange(total, dtype=np.int64) % tile.size]))
    else:
        ugrep_amd.gen(kind, 1, 0, whole.data_ptr(), total, sptr)
    sc = ugrep_amd.Scanner(pat)
    sc.scan(whole.data_ptr(), 0, total, total, True, 0, sptr)
    t = sc.totals()
    ok = (t.count, t.digest, t.dcap) == (res["count"], res["digest"], res["dcap"])
    log("verify: whole-stream count %d digest %d dcap %d; stitched %d %d %d -> %s"
        % (t.count, t.digest, t.dcap, res["count"], res["digest"], res["dcap"], "OK" if ok else "MISMATCH"))
    del whole
    torch.cuda.empty_cache()
    return ok


def pcie_inclusive(pat, buf, nbytes, dev, reps=3):
    """Host-buffer rate: ugpu_find_all on a pinned host copy of the first `nbytes`
    (hipMalloc + H2D + scan + fix + free per call). Never `value`:
    the boundary's device-resident entry point is what `value` measures."""
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.copy_(buf[:nbytes])
    torch.cuda.synchronize(dev)
    want = ugrep_amd.find_all(pat, buf[:nbytes], offsets=False)  # same bytes, device-resident
    best = float("inf")
    got = None
    for _ in range(reps):
        t0 = time.perf_counter()
        got = ugrep_amd.find_all(pat, host, offsets=False)
        best = min(best, time.perf_counter() - t0)
    ok = (got.count, got.digest, got.dcap) == (want.count, want.digest, want.dcap)
    del host
    return {"value": round(nbytes / best / 1e9, 2), "unit": "GB/s", "sample_bytes": nbytes,
            "path": "ugpu_find_all on a pinned host buffer (hipMalloc + H2D + scan + fix), best of %d" % reps,
            "equals_device_resident": ok}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): start N
    rank processes with torch.distributed.run (one per GPU, rendezvous on
    127.0.0.1) and exit with its status.  This process never touches the GPU
    (only `import torch`, which initialises nothing), and it starts the ranks
    as children -- it does not exec."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    log("launching %d ranks: %s" % (n, " ".join(cmd[1:])))
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def launch_check(backend):
    """--launch-check: the rank bring-up alone (process group, one all_gather of
    every rank's identity, barrier), no GPU work; rank 0 prints one JSON line.
    The CPU test of the launcher runs this with UGPU_BENCH_BACKEND=gloo."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist.init_process_group(backend, rank=rank, world_size=world)
    mine = torch.tensor([rank, local, os.getpid()], dtype=torch.int64)
    allr = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    dist.barrier()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "backend": backend,
                          "ranks": [dict(rank=int(t[0]), local_rank=int(t[1]), pid=int(t[2])) for t in allr]}),
              flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--bytes", type=int, default=0, help="bytes per GPU (default: the config's size)")
    ap.add_argument("--halo", type=int, default=1 << 20, help="readable bytes past a shard end")
    ap.add_argument("--cpu-sample-mib", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pcie-sample-mib", type=int, default=2048,
                    help="host-buffer sample for the PCIe-inclusive leg (0 = skip)")
    ap.add_argument("--offsets-exchange", choices=("auto", "gather", "sharded"), default="auto",
                    help="N>1 --offsets: gather the records to rank 0 (SURVEY 8e step 4), keep them on their ranks "
                         "and exchange only their sums (dist.verify_sharded), or auto: gather when all records "
                         "fit in %d GiB at the root, else sharded (dense tables at 8 ranks: ~120 GB)" % 8)
    ap.add_argument("--offsets", action="store_true",
                    help="each step also materialises the match records (start, len, accept) in HBM and, "
                         "for N > 1, all-gathers them to every rank (SURVEY.md §8e step 4)")
    ap.add_argument("--offsets-pipeline", choices=("auto", "on", "off"), default="auto",
                    help="N=1 --offsets: two scanners on two streams, so that one batch's record expansion "
                         "overlaps the next batch's COUNT pass (auto: on)")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 also scans the whole logical stream alone and checks the stitched totals")
    ap.add_argument("--compile", action="store_true",
                    help="tables from the native regex compiler (ugpu_compile) instead of the reference's "
                         "dumped opcode words")
    ap.add_argument("--word", action="store_true",
                    help="Matcher option W (ugrep -w) on the same pattern (not a BASELINE config)")
    ap.add_argument("--regex", default=None,
                    help="another pattern (ERE, compiled by ugpu_compile) over the config's corpus, e.g. "
                         "word boundaries '\\bfoo\\b' (not a BASELINE config)")
    ap.add_argument("--launch-check", action="store_true",
                    help="bring the ranks up (process group, all_gather, barrier) and report them; no GPU work")
    args = ap.parse_args()

    # rehearsal knobs for a one-GPU box: UGPU_BENCH_BACKEND=gloo puts every rank
    # on UGPU_BENCH_DEVICE (default 0) and stitches over gloo on the host
    backend = os.environ.get("UGPU_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: start one rank per GPU ourselves (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_check:
        launch_check(backend)
        return
    global ugrep_amd, gather_offsets, Shard, shard_bounds, stitch
    import ugrep_amd as _u
    from ugrep_amd import dist as _d
    ugrep_amd, gather_offsets, Shard, shard_bounds, stitch = (_u, _d.gather_offsets, _d.Shard, _d.shard_bounds,
                                                             _d.stitch)
    verify_sharded = _d.verify_sharded

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    if backend != "nccl":
        local = int(os.environ.get("UGPU_BENCH_DEVICE", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    xdev = dev if backend == "nccl" else torch.device("cpu")
    # UGPU_BENCH_PG=1: the process group and the stitch / gather collectives
    # also for one rank (rehearses the RCCL path on a one-GPU box)
    pg = world > 1 or os.environ.get("UGPU_BENCH_PG") == "1"
    if pg:
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    pkey, mode, rx, kind, size, desc = CONFIGS[args.config]
    per_gpu = args.bytes or size
    if args.config in STRONG and not args.bytes:
        per_gpu = size // world
    total = per_gpu * world
    lo, hi, _, _ = shard_bounds(total, world, rank, args.halo)
    with open(os.path.join(REPO, "ugrep_amd", "data", "config_patterns.json")) as f:
        opc = json.load(f)[pkey]["opc"]
    if args.regex is not None:
        rx, mode = args.regex, "re"
        opc = ugrep_amd.compile_regex(rx)
        desc = "'%s'%s over the corpus of %s (%s)" % (rx, " -w" if args.word else "", args.config, desc)
    elif args.compile:
        opc = ugrep_amd.compile_regex(rx, fixed=(mode == "F"))
    pat = ugrep_amd.Pattern(opc, word=args.word)
    info = pat.info()

    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def fetch(a, z):
        """The synthetic stream's bytes [a, z) in a fresh device buffer."""
        t = torch.empty(z - a + 16, dtype=torch.uint8, device=dev)
        if kind == 0:
            data = open(os.path.join(REPO, "tests", "golden", "lorem.utf8.txt"), "rb").read()
            tile = np.frombuffer(data, np.uint8)
            idx = (np.arange(a, z, dtype=np.int64) % tile.size)
            t[:z - a].copy_(torch.from_numpy(tile[idx]))
        else:
            ugrep_amd.gen(kind, 1, a, t.data_ptr(), z - a, sptr)
        torch.cuda.synchronize(dev)
        return t

    sc = ugrep_amd.Scanner(pat, records=args.offsets)
    if args.offsets:
        sc.stage(True)  # single-pass OFFSETS (prefiltered tables): the COUNT pass stages the records
    # one scan before the timed steps: a match longer than the halo grows it
    # (dist.Shard), so the steps run on a shard that holds its matches; the
    # chain fix and the true-entry re-scan grow it the same way, on the owner
    # rank before any collective (a failure there is broadcast by stitch and
    # every rank exits non-zero)
    shard = Shard(sc, fetch, lo, hi, total, args.halo, stream=sptr)
    shard.scan()
    buf = shard.buf
    log("rank %d: shard [%d, %d) read_end %d, pattern %s: %s" % (rank, lo, hi, shard.read_end, rx, info))
    kms = []

    recs_dev = {}  # --offsets: device record arrays, grown outside the timed steps when possible

    # 12-byte records (start, len) when every match has the same accept index
    # (C3, C4); 16 bytes with the accept index otherwise (C2: 3)
    one_accept = bool(info["shape"] & ugrep_amd._lib.SHAPE_ONE_ACCEPT)

    rec_bytes = 12 if one_accept else 16
    gather_limit = 8 << 30  # record bytes at the root that --offsets-exchange auto still gathers

    def records(count, total_count=None, lane=None):
        sc_, sptr_, rd = (sc, sptr, recs_dev) if lane is None else lane
        if rd.get("cap", -1) < count:
            cap = count + count // 8 + 1024
            rd.update(cap=cap, start=torch.empty(cap, dtype=torch.int64, device=dev),
                      len=torch.empty(cap, dtype=torch.int32, device=dev),
                      acc=None if one_accept else torch.empty(cap, dtype=torch.int32, device=dev))
        acc = rd["acc"]
        sc_.offsets(rd["start"].data_ptr(), rd["len"].data_ptr(), 0 if acc is None else acc.data_ptr(),
                    count, sptr_)
        st, ln = rd["start"][:count], rd["len"][:count]
        ac = None if acc is None else acc[:count]
        if pg:
            ex = args.offsets_exchange
            if ex == "auto":
                ex = "gather" if (total_count or 0) * rec_bytes <= gather_limit else "sharded"
            if ex == "sharded":
                # records stay on their ranks; their sums travel (one all_gather of
                # 4 x 8 B per rank) and are checked against the stitched totals
                return ([st], [ln], [ac], "sharded")
            # to rank 0 only, as per-rank parts (dist.gather_offsets: an
            # all_gather of dense tables' records would not fit at 8 ranks)
            g = gather_offsets(st.to(xdev), ln.to(xdev), None if ac is None else ac.to(xdev), dst=0, concat=False)
            return (([st], [ln], [ac]) if g is None else g) + ("gather",)  # (ranks > 0: their own)
        return [st], [ln], [ac], "local"

    def step():
        rec = shard.scan()
        kms.append(sc.kernel_ms())
        if pg:
            rec = stitch(rec, shard.fix, device=xdev)
        if args.offsets:
            count = rec["count"] if not pg else None
            if pg and rec["entries"][rank] != lo:  # chain re-entered this shard: re-scan from there
                # (an entry at or past hi: the previous shard's last match covers this whole shard)
                count = shard.scan(rec["entries"][rank])["count"]
            elif pg:
                count = rec["counts"][rank]
            rec["records"] = records(count, rec["count"])
            if rec["records"][3] == "sharded":
                sts, lns, acs, _ = rec["records"]
                # (the sums are taken where the records are; only they move)
                rec["verify"] = verify_sharded(sts[0], lns[0], acs[0], rec, device=xdev)
        return rec

    # N=1 --offsets, pipelined: batch i+1's COUNT pass is issued on the other
    # scanner's stream before batch i's records are written, so the record
    # expansion (write-bound) overlaps the next COUNT (read-bound); every
    # batch still gets its whole COUNT and all of its records, into its own
    # record arrays (two sets, alternating)
    pipe = args.offsets and not pg and args.offsets_pipeline != "off"
    if pipe:
        sc2 = ugrep_amd.Scanner(pat, records=True)
        sc2.stage(True)
        stream2 = torch.cuda.Stream(dev)
        lanes = [(sc, sptr, recs_dev), (sc2, stream2.cuda_stream, {})]
        sc2.scan(shard.ptr, 0, shard.hi - shard.lo, shard.read_end - shard.lo, shard.eof, shard.lo, lanes[1][1])
        sc2.totals()  # (its buffers sized outside the timed steps)

        def issue(i):
            s_, p_, _ = lanes[i % 2]
            s_.scan(shard.ptr, 0, shard.hi - shard.lo, shard.read_end - shard.lo, shard.eof, shard.lo, p_)

        def run_pipe(n):
            issue(0)
            out_ = None
            for i in range(n):
                s_ = lanes[i % 2][0]
                t = s_.totals()
                if i + 1 < n:
                    issue(i + 1)  # the next batch's COUNT, on the other stream
                kms.append(s_.kernel_ms())
                out_ = dict(entry=t.entry + shard.lo, exit=t.exit + shard.lo, count=t.count, digest=t.digest,
                            dcap=t.dcap)
                out_["records"] = records(t.count, t.count, lane=lanes[i % 2])
            return out_

    if pipe:
        res = run_pipe(max(2, args.warmup))  # (both record sets sized before the timed steps)
    for _ in range(0 if pipe else args.warmup):
        res = step()
    kms.clear()
    if pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if pipe:
        res = run_pipe(args.steps)
    for _ in range(0 if pipe else args.steps):
        res = step()
    torch.cuda.synchronize(dev)
    if pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if pg:
        e = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    pcie = None
    buf = shard.buf  # (a grown halo replaced it)
    if rank == 0 and world == 1 and args.pcie_sample_mib > 0:
        pcie = pcie_inclusive(pat, buf, min(args.pcie_sample_mib << 20, hi - lo), dev)
    cpu_leg = (None, None)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # value: the reference on one GPU's share of the node's cores (the
        # visible CPUs / 8 GPUs of an MI355X node, at least 16); also reported:
        # the same on every visible core (os.sched_getaffinity shows the whole
        # machine; capped at 256 threads)
        visible = len(os.sched_getaffinity(0))
        threads = int(os.environ.get("UGPU_BENCH_CPU_THREADS", "0")) or max(16, visible // 8)
        threads = min(threads, visible)
        sample = min(args.cpu_sample_mib << 20, per_gpu)
        log("cpu baseline: %d MiB, %d threads (per-GPU share of %d visible CPUs)" % (sample >> 20, threads, visible))
        base, ref = cpu_baseline(args.config, sample, threads, args.regex, args.word)
        allc = min(visible, 256)
        if base is not None and base.get("kind") == "reference" and allc > threads:
            try:
                pkey_, mode_, rx_, kind_, _, _ = CONFIGS[args.config]
                if args.regex is not None:
                    mode_, rx_ = "re", args.regex
                ja = _harness(os.path.join(REPO, "oracle", "_ref", "ref_harness_avx2"), mode_ + ("W" if args.word else ""),
                              rx_, _spec(kind_, sample), allc, 2)
                base["all_cores"] = {"value": round(ja["bytes"] / ja["seconds"] / 1e9, 3), "unit": "GB/s",
                                     "cores": allc, "best_of": 2}
            except Exception as e:  # pragma: no cover - diagnostic path
                log("all-cores reference leg failed: %s" % e)
        chk = None
        if ref is not None:  # the same bytes on the GPU, compared with the reference
            chk = gpu_reference_check(pat, buf, sample, ref, sptr)
            log("reference parity on [0, %d): %s" % (sample, chk))
        cpu_leg = (base, chk)
    verified = None
    if args.verify:
        del buf
        shard.buf = None
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        if pg:
            dist.barrier()  # every shard buffer is released before rank 0 allocates the whole stream
        verified = verify_whole(args, kind, total, pat, res, rank, dev, sptr) if rank == 0 else None
        if pg:
            dist.barrier()

    k_avg = float(np.mean(kms)) if kms else float("nan")
    rank_kms = [k_avg]
    if pg:  # every rank's own scan-kernel time (HIP events), reported by rank 0
        mine = torch.tensor([k_avg], dtype=torch.float64, device=xdev)
        allk = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allk, mine)
        rank_kms = [round(float(t.item()), 4) for t in allk]
    achieved = (hi - lo) / (k_avg * 1e-3) / 1e9
    value = total * args.steps / elapsed / 1e9
    matches_per_s = res["count"] * args.steps / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.config in STRONG else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": desc, "config": args.config, "pattern": rx, "bytes_per_gpu": per_gpu,
                   "total_bytes": total, "corpus_kind": kind, "parallelism": "shard%d" % world,
                   "tables": "compiled" if (args.compile or args.regex is not None) else "reference", "word": args.word, "dfa_states": info["states"], "dfa_row": info["row"], "prefilter_ppm": info["prefilter_ppm"]},
        "matches": res["count"],
        "matches_per_s": round(matches_per_s, 1),
        "digest": res["digest"],
        "roofline": {"bound": "hbm", "kernel": KERNELS[info["kernel"]],
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel_ms": round(k_avg, 4), "algorithmic_bytes_per_launch": hi - lo},
        "rank_kernel_ms": rank_kms,
    }
    if pcie is not None:
        out["pcie_inclusive"] = pcie
    if verified is not None:
        out["verified_whole_stream"] = verified
    if args.offsets:
        sts, lns, _, how = res["records"]
        m64 = (1 << 64) - 1
        if how == "sharded":
            ver = res["verify"]
            out["offsets"] = {"records": ver["count"], "bytes_per_record": rec_bytes,
                              "gathered_to": "none: records stay on their ranks, their sums are all-gathered "
                                             "(dist.verify_sharded)",
                              "digest_matches_totals": bool(ver["ok"])}
        else:
            nrec = sum(int(s_.numel()) for s_ in sts)
            dg = sum(int((s_ * 31 + l_.to(torch.int64)).sum().item()) for s_, l_ in zip(sts, lns)) & m64  # (wraps as u64)
            out["offsets"] = {"records": nrec, "bytes_per_record": rec_bytes,
                              "gathered_to": "rank 0 (per-rank parts)" if pg else "local",
                              "digest_matches_totals": nrec == res["count"] and dg == res["digest"],
                              "pipelined": bool(pipe)}
        if shard.grown:
            out["offsets"]["halo_grown"] = shard.grown
    # (the committed PMC traffic is per BASELINE config and pattern)
    tr = None if (args.regex is not None or args.word) else measured_traffic(args.config, hi - lo,
                                                                             KERNELS[info["kernel"]])
    if tr and tr.get("kernel_ms") and abs(tr["kernel_ms"] - k_avg) > 0.05 * k_avg:
        # the counters were taken on a run whose kernel time differs from this one's
        log("traffic.json %s: kernel %.4f ms there, %.4f ms here: not used" % (args.config, tr["kernel_ms"], k_avg))
        out["roofline"]["traffic_note"] = "profiles/traffic.json entry not used: kernel time %.4f ms there vs %.4f ms" \
            % (tr["kernel_ms"], k_avg)
        tr = None
    if tr:
        out["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
        out["roofline"]["traffic_source"] = tr["source"]
        out["roofline"]["traffic_kernel_ms"] = tr.get("kernel_ms")
    if cpu_leg[0] is not None:
        out["cpu_baseline"] = cpu_leg[0]
        if cpu_leg[1] is not None:
            out["parity_vs_reference"] = cpu_leg[1]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
