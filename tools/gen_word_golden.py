#!/usr/bin/env python3
"""Generate tests/golden/word_cases.json: reference match lists for ugrep -w
(Matcher option W, src/ugrep.cpp:8616-8618; lib/matcher.cpp:76, :107, :142,
:208, :664; include/reflex/matcher.h:1194-1237).

Each case is (pattern, -F?, input spec) with the reference's full
(start, len, accept) list from oracle/_ref/ref_harness find reW|FW (libreflex
compiled from /root/reference), plus the reference's opcode words so the GPU
box needs no regex compiler.  Inputs: a hand-made edge-case text (ASCII and
UTF-8 word boundaries, '_', digits, invalid UTF-8, a match at BOB/EOF) and
64 KiB slices of the synthetic corpora.  Build container only; the output is
data, committed.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")

EDGE = ("foo xfoo foo_ foo. éfoo fooé foo\n"
        "_foo foo_bar 1foo foo1 (foo) ¿foo? «foo» foo-bar foo\tfoo\n"
        "lorem Lorem loremipsum ipsum_lorem lorem,lorem ñlorem loremñ €lorem lorem€\n"
        "int x_1 = 42; αβγ δ ε, word_ends here. ab12 12ab a_b é_é\n"
        "日本語 テキスト foo日本 日本foo 中foo中 ǅfoo fooǅ\n").encode("utf-8") + \
    b"foo\x80foo \x80foo foo\x80 \xc3foo foo\xc3 \xe2\x82foo foo\xe2\x82\xacfoo \xf0\x9f\x98\x80foo foo"

CASES = [
    ("re", "foo"), ("re", "foo|bar|baz"), ("re", "lorem"), ("F", "lorem"), ("F", "foo"),
    ("re", r"\w+"), ("re", "[A-Za-z_][A-Za-z0-9_]*"), ("re", r"\d+"), ("re", "[a-z]+"),
    ("re", "foo|foo_bar"), ("re", "ab|ab12|a"), ("re", r"\W+"), ("re", "é\\w*"), ("re", "日本"),
    ("re", "x_1|x"), ("re", r"[a-z]+\d*"), ("re", "o+"), ("re", "foo.?"),
]


def ref(mode, rx, spec):
    out = subprocess.run([HARNESS, "find", mode + "W", rx, spec, "list"], capture_output=True, check=True)
    lines = out.stdout.decode().split("\n")
    cnt, dg, dc = (int(v) for v in lines[0].split())
    lst = [[int(v) for v in ln.split()] for ln in lines[1:] if ln.strip()]
    assert len(lst) == cnt
    return cnt, dg, dc, lst


def dump(mode, rx):
    out = subprocess.run([HARNESS, "dump", mode, rx], capture_output=True, check=True)
    return json.loads(out.stdout)["opc"]


def main():
    tmp = os.path.join(REPO, "tests", "golden", "word_edge.txt")
    with open(tmp, "wb") as f:
        f.write(EDGE)
    inputs = [("edge", "file:%s:0" % tmp, None)]
    for kind in (1, 3, 4):
        inputs.append(("gen%d" % kind, "gen:%d:5:0:65536" % kind, (kind, 5, 0, 65536)))
    cases = []
    for mode, rx in CASES:
        opc = dump(mode, rx)
        for name, spec, g in inputs:
            cnt, dg, dc, lst = ref(mode, rx, spec)
            cases.append(dict(mode=mode, pattern=rx, input=name, gen=g, opc=opc, count=cnt, digest=dg, dcap=dc,
                              list=lst if cnt <= 4000 else None))
    with open(os.path.join(REPO, "tests", "golden", "word_cases.json"), "w") as f:
        json.dump(cases, f)
    print("%d cases" % len(cases), file=sys.stderr)


if __name__ == "__main__":
    main()
