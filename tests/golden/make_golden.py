#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ (run in the build container only).

The expected outputs come from the REFERENCE matcher itself: oracle/_ref/ref_harness
links libreflex compiled from /root/reference/lib (see oracle/Makefile).  The
reference cannot travel to the GPU box, so its outputs are committed here as data:

  patterns.json  opcode words (Pattern::opc_) + scalar fields per pattern, exactly
                 what a caller passes through the C-ABI (include/ugpu.h).
  cases.json     (pattern, input) -> count, digest = sum(start*31+len),
                 dcap = sum((start+1)*cap), and the full (start,len,cap) list for
                 small cases.
  refgold.json   match offsets parsed from the reference's OWN golden outputs
                 (/root/reference/tests/out/*.out, produced by tests/verify.sh),
                 which pin ref_harness and the oracle restatement.

Usage: make -C oracle ref && python tests/golden/make_golden.py
"""
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
REFTESTS = "/root/reference/tests"

# name -> (mode, regex).  mode: re/F = ugrep default (Unicode), reU/FU = ugrep -U.
PATTERNS = {
    "c1_lorem": ("F", "lorem"),
    "c2_foobarbaz": ("re", "foo|bar|baz"),
    "c3_ident": ("re", "[A-Za-z_][A-Za-z0-9_]*"),
    "c4_word": ("re", r"\w+"),
    "hello": ("reU", "Hello"),
    "hello_wnhS": ("reU", r"\w+[\n\h]+\S+"),
    "astar_b": ("re", "a*b"),
    "fo_foo_foob": ("re", "fo|foo|foob"),
    "aa": ("re", "aa"),
    "abab_c": ("re", "(ab)+c"),
    "x_digits_y": ("re", "x[0-9]{2,4}y"),
    "digits": ("re", "[0-9]+"),
    "the_then": ("re", "the|then|there|these"),
    "float": ("re", r"\d+\.\d+"),
    "nonspace": ("re", r"[^ \t]+"),
    "dot": ("re", "."),
    "a_dot_c": ("re", "a.c"),
    "e_acute": ("re", "é+"),
    "five_chars": ("re", "q|w|x|y|z"),
    "long_alt": ("re", "internationalization|international|intern"),
    "lorem_ascii": ("FU", "lorem"),
    "nomatch": ("reU", "nomatch"),
    "wide_class": ("re", r"[\p{Greek}\p{Cyrillic}]+"),
    "s_plus": ("re", r"\S+"),
    # unsupported on the GPU path (anchors, word boundaries, lookahead): must be rejected
    "anchor_bol": ("re", "^foo"),
    "anchor_eol": ("re", "foo$"),
    "word_boundary": ("re", r"\bfoo\b"),
    "lookahead": ("re", "foo(?=bar)"),
}

EDGE_INPUTS = {
    "empty": b"",
    "one_a": b"a",
    "survey_probe": b"9abc x_1 2a foofoo barbaz fo\nobar",
    "fofoo": b"fofoo foob foobar fo",
    "aab_chain": b"b" + b"a" * 5001 + b"\nab aaab aab\n",
    "hello_world": b"Hello World\nHello\nhello HELLO\n",
    "utf8_mix": "héllo wörld € 你好 ok éé é\n中文 Ελληνικά Кириллица x12y x1234y x12345y\n".encode(),
    "digits_float": b"3.14 2. .5 10.01 7\n1234567890\n",
    "intern": b"internationalization internationa intern internal international\n",
    "abab": b"ababc abc ababab ababababc c\n",
    "binaryish": bytes(range(256)) * 3,
    "newlines": b"\n\n\nfoo\n\nbar\n",
}

GEN_KINDS = {"words": 1, "planted": 2, "code": 3, "utf8": 4}


def dump(mode, rx):
    out = subprocess.check_output([HARNESS, "dump", mode, rx])
    return json.loads(out)


def find(mode, rx, spec, want_list):
    args = [HARNESS, "find", mode, rx, spec] + (["list"] if want_list else [])
    out = subprocess.check_output(args).decode().split("\n")
    count, digest, dcap = (int(x) for x in out[0].split())
    lst = [[int(v) for v in ln.split()] for ln in out[1:] if ln.strip()]
    return count, digest, dcap, lst


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle ref")
    pats = {}
    for name, (mode, rx) in PATTERNS.items():
        j = dump(mode, rx)
        j.update(mode=mode, regex=rx)
        pats[name] = j
    cases = []
    # small edge inputs x every pattern: full match lists
    for iname, data in EDGE_INPUTS.items():
        spec = "hex:" + data.hex()
        for pname, (mode, rx) in PATTERNS.items():
            c, d, dc, lst = find(mode, rx, spec, True)
            cases.append(dict(pattern=pname, input=dict(type="hex", name=iname, hex=data.hex()),
                              count=c, digest=d, dcap=dc, matches=lst))
    # reference data fixtures
    for fname in ("lorem.utf8.txt", "Hello.java"):
        spec = "file:" + os.path.join(HERE, fname)
        for pname, (mode, rx) in PATTERNS.items():
            c, d, dc, lst = find(mode, rx, spec, True)
            cases.append(dict(pattern=pname, input=dict(type="file", name=fname),
                              count=c, digest=d, dcap=dc, matches=lst if c <= 5000 else None))
    # generator slices (64 KiB at an odd offset, full lists for the config patterns)
    for gname, kind in GEN_KINDS.items():
        for off, ln, lists in ((1000003, 65536, True), (0, 1 << 20, False)):
            spec = "gen:%d:%d:%d:%d" % (kind, 12345, off, ln)
            for pname in ("c2_foobarbaz", "c3_ident", "c4_word", "c1_lorem", "digits", "fo_foo_foob",
                          "the_then", "s_plus", "aa", "astar_b"):
                mode, rx = PATTERNS[pname]
                c, d, dc, lst = find(mode, rx, spec, lists)
                cases.append(dict(pattern=pname, input=dict(type="gen", kind=kind, seed=12345, off=off, len=ln),
                                  count=c, digest=d, dcap=dc, matches=lst if lists else None))
    # config-sized digests (64 MiB): the C1 anchor and one per generated corpus
    big = [("c1_lorem", "file:" + os.path.join(HERE, "lorem.utf8.txt") + ":67108864",
            dict(type="file", name="lorem.utf8.txt", total=67108864))]
    for pname, kind in (("c2_foobarbaz", 1), ("c2_foobarbaz", 2), ("c3_ident", 3), ("c4_word", 4)):
        big.append((pname, "gen:%d:%d:%d:%d" % (kind, 1, 0, 1 << 26),
                    dict(type="gen", kind=kind, seed=1, off=0, len=1 << 26)))
    for pname, spec, inp in big:
        mode, rx = PATTERNS[pname]
        c, d, dc, _ = find(mode, rx, spec, False)
        cases.append(dict(pattern=pname, input=inp, count=c, digest=d, dcap=dc, matches=None, big=True))

    with open(os.path.join(HERE, "patterns.json"), "w") as f:
        json.dump(pats, f, indent=1)
    # the benchmark configs' compiled tables, shipped with the package as the
    # precompiled-pattern artifact a caller hands over the C ABI (bench.py)
    cfg = {k: pats[k] for k in ("c1_lorem", "c2_foobarbaz", "c3_ident", "c4_word")}
    os.makedirs(os.path.join(REPO, "ugrep_amd", "data"), exist_ok=True)
    with open(os.path.join(REPO, "ugrep_amd", "data", "config_patterns.json"), "w") as f:
        json.dump(cfg, f)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(cases, f)

    write_refgold()
    print("patterns", len(pats), "cases", len(cases))


def write_refgold():
    """The reference's own goldens (tests/verify.sh:262-271): -U -ounkbT gives
    line, column and byte offset of every match; -c the matching-line count."""
    refgold = {}
    strip = re.compile(r"\x1b\[[0-9;]*[mK]")
    for pname, fn in (("hello", "Hello_Hello-ounkbT.out"), ("hello_wnhS", "Hello_wnhS-ounkbT.out")):
        offs, lines = [], []
        for ln in open(os.path.join(REFTESTS, "out", fn), encoding="latin-1"):
            ln = strip.sub("", ln)
            m = re.match(r"Hello\.java:\s*(\d+):\s*\d+:\s*(\d+):", ln)
            if m:
                lines.append(int(m.group(1)))
                offs.append(int(m.group(2)))
        refgold[pname] = dict(file="Hello.java", source="tests/out/" + fn, starts=offs, lines=lines)
    for ln in open(os.path.join(REFTESTS, "out", "Hello_Hello-c.out"), encoding="latin-1"):
        m = re.match(r"Hello\.java:(\d+)", strip.sub("", ln))
        if m:
            refgold["hello"]["c_count"] = int(m.group(1))
            refgold["hello"]["c_source"] = "tests/out/Hello_Hello-c.out"
    cnt = open(os.path.join(REFTESTS, "out", "lorem.utf8-iwco.out"), encoding="latin-1").read()
    refgold["lorem_iwco_count"] = int(strip.sub("", cnt).strip())
    with open(os.path.join(HERE, "refgold.json"), "w") as f:
        json.dump(refgold, f, indent=1)


if __name__ == "__main__":
    import sys
    if sys.argv[1:] == ["--refgold-only"]:
        write_refgold()
    else:
        main()
