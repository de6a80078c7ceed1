#!/usr/bin/env python3
"""Generate tests/golden/utf8.json: reflex::isutf8 results of the REFERENCE
(lib/simd.cpp:169-421, compiled from /root/reference by oracle/Makefile into
oracle/_ref/ref_harness and ref_harness_avx2) on hand-made and seeded inputs.

Run in the build container (the reference does not travel):
    make -C oracle ref && python tests/golden/make_utf8_golden.py

The inputs are placed at every offset around the reference's 16/32-byte SIMD
block boundaries and at its SIMD/scalar split, so that each of its code paths
(ASCII prescan, p/q/r block check, end backtrack, scalar tail) decides some of
them.  Both builds must agree; the fixture stores their common answer.
"""
import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")


def ref_isutf8(specs, harness):
    out = subprocess.run([os.path.join(REF, harness), "isutf8"], input="\n".join(specs) + "\n",
                         capture_output=True, text=True, check=True).stdout.split()
    assert len(out) == len(specs)
    return [o == "1" for o in out]


SEQS = {
    "ascii": [b"a", b"Z", b"~", b"\x01", b"\x7f", b"\n"],
    "two": [b"\xc2\x80", b"\xc3\xa9", b"\xdf\xbf"],
    "three": [b"\xe0\xa0\x80", b"\xe2\x82\xac", b"\xef\xbf\xbf", b"\xed\xa0\x80", b"\xe0\x80\x80"],
    "four": [b"\xf0\x90\x80\x80", b"\xf4\x8f\xbf\xbf", b"\xf0\x80\x80\x80", b"\xf4\x90\x80\x80"],
    "bad": [b"\x00", b"\x80", b"\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xf5\x80\x80\x80", b"\xff", b"\xfe",
            b"\xc3", b"\xe2\x82", b"\xf0\x90\x80", b"\xc3\xc3", b"\xe2a\xac", b"\xc3\xa9\xa9"],
}


def cases():
    out = [b""]
    out += [bytes([b]) for b in range(256)]
    out += [bytes([a, b]) for a in (0x00, 0x41, 0x80, 0xc1, 0xc2, 0xdf, 0xe0, 0xef, 0xf0, 0xf4, 0xf5, 0xff)
            for b in (0x00, 0x41, 0x7f, 0x80, 0xbf, 0xc0, 0xc2, 0xe0, 0xf0, 0xff)]
    # one sequence at every offset of a 72-byte ASCII line (16/32/64-byte blocks)
    for kind, seqs in SEQS.items():
        for s in seqs:
            for off in range(0, 72 - len(s) + 1, 1 if kind == "bad" else 3):
                out.append(b"x" * off + s + b"y" * (72 - off - len(s)))
    # cut-off sequences at the end of buffers of lengths around 16/32/48/64
    for n in (15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 96, 97):
        for s in SEQS["two"] + SEQS["three"] + SEQS["four"]:
            for cut in range(1, len(s) + 1):
                body = b"q" * max(0, n - cut) + s[:cut]
                out.append(body)
                out.append("é".encode() * (n // 2) + s[:cut])
    # NUL in otherwise ASCII / UTF-8 buffers
    for n in (16, 33, 70, 130):
        for z in (0, 1, 15, 16, 31, 32, n - 1):
            if z < n:
                b = bytearray(b"k" * n)
                b[z] = 0
                out.append(bytes(b))
                u = bytearray(("ж" * n).encode()[:2 * n])
                u[2 * z if 2 * z < len(u) else z] = 0
                out.append(bytes(u))
    # seeded random token streams, some corrupted
    rng = random.Random(20251016)
    toks = SEQS["ascii"] + SEQS["two"] + SEQS["three"] + SEQS["four"]
    for i in range(900):
        n = rng.choice([5, 17, 40, 70, 130, 300])
        b = bytearray()
        while len(b) < n:
            b += rng.choice(toks)
        if i % 3:
            k = rng.randrange(len(b))
            b[k] = rng.randrange(256)
        if i % 7 == 0:
            b = b[:rng.randrange(len(b) + 1)]
        out.append(bytes(b))
    return out


def main():
    if not os.path.exists(os.path.join(REF, "ref_harness")):
        sys.exit("build the reference harness first: make -C oracle ref")
    cs = cases()
    specs = ["hex:" + c.hex() if c else "hex:" for c in cs]
    r512 = ref_isutf8(specs, "ref_harness")
    r2 = ref_isutf8(specs, "ref_harness_avx2")
    assert r512 == r2, "reference builds disagree"
    files = [
        {"type": "file", "name": "lorem.utf8.txt"},
        {"type": "file", "name": "Hello.java"},
        {"type": "gen", "kind": 4, "seed": 1, "off": 0, "len": 1 << 20},
        {"type": "gen", "kind": 3, "seed": 1, "off": 0, "len": 1 << 20},
        {"type": "gen", "kind": 1, "seed": 1, "off": 0, "len": 1 << 20},
    ]
    fspecs = []
    for f in files:
        if f["type"] == "file":
            fspecs.append("file:%s" % os.path.join(HERE, f["name"]))
        else:
            fspecs.append("gen:%d:%d:%d:%d" % (f["kind"], f["seed"], f["off"], f["len"]))
    f512 = ref_isutf8(fspecs, "ref_harness")
    assert f512 == ref_isutf8(fspecs, "ref_harness_avx2")
    for f, r in zip(files, f512):
        f["isutf8"] = r
    doc = {"source": "reflex::isutf8 of the reference (oracle/_ref/ref_harness isutf8), AVX512BW and AVX2 builds agree",
           "cases": [[c.hex(), r] for c, r in zip(cs, r512)], "inputs": files}
    with open(os.path.join(HERE, "utf8.json"), "w") as fh:
        json.dump(doc, fh, separators=(",", ":"))
    print("%d cases (%d valid), %d inputs" % (len(cs), sum(r512), len(files)))


if __name__ == "__main__":
    main()
