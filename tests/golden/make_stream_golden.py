#!/usr/bin/env python3
"""Regenerate tests/golden/streams.json (build container only): the REFERENCE
matcher's count, digest = sum(start*31+len) and dcap = sum((start+1)*cap) over
long prefixes of the benchmark corpora, to pin multi-shard (C5) and full-size
parity on the GPU box, where the reference cannot run.

Each entry is one whole buffer: reflex::Matcher m(pattern); m.buffer(buf, n+1);
while (m.find()) ... over bytes [0, n) of the oracle/gen.h corpus `kind` with
seed 1 (oracle/_ref/ref_harness "find", libreflex compiled from
/root/reference/lib by oracle/Makefile).  The GPU tests cut the same bytes into
shards at arbitrary offsets and stitch them (tests/test_c5.py).

Usage: make -C oracle ref && python tests/golden/make_stream_golden.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")

# name -> (pattern key in patterns.json, mode, regex, corpus kind, bytes)
STREAMS = {
    "c2_512m": ("c2_foobarbaz", "re", "foo|bar|baz", 1, 512 << 20),
    "c3_256m": ("c3_ident", "re", "[A-Za-z_][A-Za-z0-9_]*", 3, 256 << 20),
    "c4_128m": ("c4_word", "re", r"\w+", 4, 128 << 20),
}


def main():
    out = {}
    for name, (pkey, mode, rx, kind, n) in STREAMS.items():
        r = subprocess.run([HARNESS, "find", mode, rx, "gen:%d:1:0:%d" % (kind, n)], capture_output=True,
                           check=True, text=True).stdout.split()
        out[name] = dict(pattern=pkey, regex=rx, kind=kind, seed=1, bytes=n, count=int(r[0]), digest=int(r[1]),
                         dcap=int(r[2]))
        print(name, out[name])
    with open(os.path.join(HERE, "streams.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
