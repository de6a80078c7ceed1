#!/usr/bin/env python3
"""ugrep itself, CPU against drop-in GPU: `ugrep -co -J16 PATTERN files...` of
the reference build (oracle/_ref/ugrep) and of the drop-in build
(oracle/_ref/ugrep_gpu: reflex::GpuMatcher at ugrep's construction sites) over
the same files, 16 worker threads (one GPU's share of the node's cores), with
the adapter's default policy.  ugrep reads files through input() (memory maps
are off unless --mmap, src/ugrep.hpp:43-44), so each input reaches the GPU as a
stream of chunks (ugpu_stream_feed); with --mmap a whole buffer
(ugpu_find_records).  Either way the bytes cross PCIe.
Prints one JSON line per config: wall seconds (best of --reps), GB/s, whether
the outputs are identical, and how the adapter dispatched (matchers, GPU scans,
FIND calls answered by the GPU and by the CPU matcher, and why).

    python tools/bench_ugrep.py [--files 32] [--mib 128] [--workers 16] [--reps 3]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

# -co: count every match (the FIND chain), not matching lines (plain -c stops
# at a line's first match, src/ugrep.cpp:10536-10565)
CONFIGS = [("c2", "foo|bar|baz", 1), ("c2_gpu", "foo|bar|baz", 1), ("c3", "[A-Za-z_][A-Za-z0-9_]*", 3), ("c4", r"\w+", 4),
           # loop-needle tables on the C2 corpus, -co and -cow
           ("c2_ing", "[a-z]+ing", 1), ("c2_ing_gpu", "[a-z]+ing", 1), ("c2_wing_gpu", "[a-z]+ing", 1, ["-w"]),
           # option W without a selective prefilter (sparse_kernel, DfaPlan::wsparse) on the C3 corpus
           ("c3_wazAZ", "[A-Za-z]+", 3, ["-w"])]


def stats(stderr):
    agg = dict(matchers=0, gpu_matchers=0, scans=0, gpu_finds=0, cpu_finds=0, cpu_why={}, read_ms_max=0.0,
               feed_ms_max=0.0)
    for ln in stderr.decode(errors="replace").splitlines():
        if not ln.startswith("[ugpu-adapter] scans="):
            continue
        kv = dict(f.split("=", 1) for f in ln.split()[1:])
        agg["matchers"] += 1
        agg["scans"] += int(kv["scans"])
        agg["gpu_finds"] += int(kv["gpu_finds"])
        agg["cpu_finds"] += int(kv["cpu_finds"])
        if int(kv["scans"]):
            agg["gpu_matchers"] += 1
        # (per matcher: time in its stream's reads and in ugpu_stream_feed)
        for k in ("read_ms", "feed_ms"):
            if k in kv:
                agg[k + "_max"] = max(agg[k + "_max"], float(kv[k]))
        if kv["cpu_why"] != "-":
            for w in kv["cpu_why"].split(","):
                k, v = w.split(":")
                agg["cpu_why"][k] = agg["cpu_why"].get(k, 0) + int(v)
    return agg


def run(exe, args, env, reps):
    best, out, err = 1e30, None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = subprocess.run([exe] + args, env=env, capture_output=True, timeout=1200)
        dt = time.perf_counter() - t0
        if r.returncode not in (0, 1):
            raise RuntimeError("%s failed: %s" % (exe, r.stderr.decode(errors="replace")[-500:]))
        if dt < best:
            best, out, err = dt, r.stdout, r.stderr
    return best, out, err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=32)
    ap.add_argument("--mib", type=int, default=128)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--configs", default="c2,c2_gpu,c3,c4")
    a = ap.parse_args()
    from oracle_lib import gen
    ref = os.path.join(REPO, "oracle", "_ref", "ugrep")
    gpu = os.path.join(REPO, "oracle", "_ref", "ugrep_gpu")
    n = a.mib << 20
    # process start-up: one small file, forced onto the GPU (HIP runtime and
    # device init, table upload, pinned pool), against the CPU build
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        p = os.path.join(d, "small.txt")
        gen(1, 1, 0, 1 << 16).tofile(p)
        env = dict(os.environ, UGPU_ADAPTER_MIN_BYTES="0", UGPU_ADAPTER_STATS="1", UGPU_ADAPTER_WARM="0")
        t_cpu, o_cpu, _ = run(ref, ["-co", "foo|bar|baz", p], env, a.reps)
        t_gpu, o_gpu, e_gpu = run(gpu, ["-co", "foo|bar|baz", p], env, a.reps)
        print(json.dumps({"config": "startup", "bytes": 1 << 16, "cpu_s": round(t_cpu, 4), "gpu_s": round(t_gpu, 4),
                          "outputs_equal": o_cpu == o_gpu, "adapter": stats(e_gpu)}), flush=True)
    for cfg in CONFIGS:
        name, rx, kind = cfg[:3]
        flags = cfg[3] if len(cfg) > 3 else []
        if name not in a.configs.split(","):
            continue
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
            files = []
            for k in range(a.files):
                p = os.path.join(d, "%s_%03d.txt" % (name, k))
                gen(kind, 1, k * n, n).tofile(p)
                files.append(p)
            args = ["-co", "-J%d" % a.workers] + flags + [rx] + files
            env = dict(os.environ)
            env.pop("UGPU_ADAPTER_SPARSE_MAX", None)
            env.pop("UGPU_ADAPTER_MIN_BYTES", None)
            t_cpu, o_cpu, _ = run(ref, args, env, a.reps)
            # c2_gpu: the prefiltered table forced onto the GPU -- the device
            # warmed up before the first input (UGPU_ADAPTER_WARM=0), the device
            # queue at its default 2 slots; by default (c2) such a table stays
            # on the workers' cores until a dense table has warmed the device
            genv = dict(env, UGPU_ADAPTER_STATS="1")
            if name.endswith("_gpu"):
                genv["UGPU_ADAPTER_WARM"] = "0"
            t_gpu, o_gpu, e_gpu = run(gpu, args, genv, a.reps)
            total = a.files * n
            # -J: files finish in any order
            s_cpu, s_gpu = sorted(o_cpu.splitlines()), sorted(o_gpu.splitlines())
            diff = [(x.decode(), y.decode()) for x, y in zip(s_cpu, s_gpu) if x != y][:4]
            print(json.dumps({"config": name, "pattern": rx, "flags": flags, "files": a.files, "bytes": total,
                              "workers": a.workers, "cpu_s": round(t_cpu, 4), "gpu_s": round(t_gpu, 4),
                              "cpu_gbps": round(total / t_cpu / 1e9, 2), "gpu_gbps": round(total / t_gpu / 1e9, 2),
                              "speedup": round(t_cpu / t_gpu, 2), "outputs_equal": s_cpu == s_gpu, "diff": diff,
                              "adapter": stats(e_gpu)}), flush=True)


if __name__ == "__main__":
    main()
