#!/usr/bin/env python3
"""Generate tests/golden/lookahead_compile.json: the reference's tables and
FIND results for lookahead patterns, to pin the native compiler's lookahead
(ugpu_compile, Parser::lookahead_group in ugrep_amd/csrc/regex_compile.cpp)
against lib/pattern.cpp:1331-1359 / :2374-2419 / :2953-2964.

Per pattern: the converted regex (what ugrep hands its Pattern), the
reference's opcode words (null when the reference throws regex_error), and
the reference Matcher's FIND over an edge text (count, digest, dcap and the
match list), all from the reference harness (oracle/_ref/ref_harness: libreflex
compiled from /root/reference).  Includes the shapes the compiler refuses
(nested and adjacent lookaheads, anchors), so the test can check that a
refusal is the only other outcome.

Build container only; the output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

EDGE = (b"xy x y xyz yx abc ab ac abd aab abab abbc a\nfoobar foo bar foobarbaz fooqux foobarqux bazqux\n"
        b"dolor sit amet, consectetur. 3.14 42 7.x 1.2.3\nprintf(x); f(1)(2) g (3)\ncaf\xc3\xa9x \xc3\xa9x x\xc3\xa9 "
        b"\xe4\xb8\xad\xc3\xa9\nsinging sing ring rings bring\naaab aab ab b\n")

PATTERNS = [
    ("reU", r"(?=x)y"), ("reU", r"(?=x)"), ("reU", r"(?=xy)x"), ("reU", r"a(?=b)c"), ("reU", r"a(?=b*)"),
    ("reU", r"a(?=b?)c"), ("reU", r"(a(?=b))+"), ("reU", r"x(?=y)|y(?=x)"), ("reU", r"foo(?=bar)|foo"),
    ("reU", r"foo|foo(?=bar)"), ("reU", r"(foo(?=bar)|baz)qux"), ("reU", r"a(?=b|c)|a(?=d)"),
    ("reU", r"a{2}(?=b)"), ("reU", r"(a(?=b)){2}"), ("reU", r"a(?=b)b"), ("reU", r"[a-z]+(?=ing)"),
    ("reU", r"\d+(?=\.\d)"), ("reU", r"ab(?=c)|a(?=bc)"), ("reU", r"[a-z]+(?=,)|[a-z]+(?=\.)"),
    ("reU", r"a*(?=b)"), ("reU", r"(?:dolor|sit)(?= )"), ("reU", r"\w+(?=\()|\w+(?= \()"),
    ("re", r"caf(?=é)"), ("re", r"\w(?=é)"), ("re", r"é(?=x)"), ("re", r"[a-z]+(?=ing|s\b)"),
    ("reU", r"(?i)FOO(?=bar)"), ("reU", r"x(?=y)z|xy|x"),
    # refused by the native compiler (the reference merges these lookahead ranges)
    ("reU", r"a(?=b(?=c))"), ("reU", r"a(?=b)(?=c)"),
    # refused: lookahead with anchors / word boundaries
    ("reU", r"^a(?=b)"), ("reU", r"a(?=b)$"), ("reU", r"\ba(?=b)"),
]


def run(args):
    r = subprocess.run([HARNESS] + args, capture_output=True)
    if r.returncode:
        return None
    return r.stdout.decode()


def main():
    cases = []
    spec = "hex:" + EDGE.hex()
    for mode, rx in PATTERNS:
        d = run(["dump", mode, rx])
        if d is None:
            cases.append(dict(pattern=rx, mode=mode, opc=None))
            continue
        dd = json.loads(d)
        out = run(["find", mode, rx, spec, "list"])
        lines = out.strip().split("\n")
        cnt, dg, dc = (int(x) for x in lines[0].split())
        lst = [[int(v) for v in ln.split()] for ln in lines[1:]]
        cases.append(dict(pattern=rx, mode=mode, opc=dd["opc"], conv=dd["conv_hex"], count=cnt, digest=dg, dcap=dc,
                          list=lst))
    out = os.path.join(GOLDEN, "lookahead_compile.json")
    with open(out, "w") as f:
        json.dump(dict(edge_hex=EDGE.hex(), cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
