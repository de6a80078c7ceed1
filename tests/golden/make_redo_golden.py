#!/usr/bin/env python3
"""Generate tests/golden/redo_cases.json: reference results for negative
patterns (ugrep -N PATTERN wraps it as (?^PATTERN), src/ugrep.cpp:6487,
src/cnf.cpp:503; the Pattern marks the DFA states that hold a negated accept
REDO, lib/pattern.cpp:2358-2363 and :2945-2947; the FIND loop steps over a
match whose last accept is REDO, lib/matcher.cpp:151-156, :218-225,
:732-738), from the reference harness (oracle/_ref/ref_harness: libreflex
compiled from /root/reference).

Each case: the converted pattern's opcode words and regex (what the drop-in
adapter compiles, UGPU_RX_REFLEX), and per input the reference Matcher's
count/digest/dcap, plus the full match list for the small inputs.  Patterns
in ugrep's -N form: the negative alternatives first, then the positive ones.

Build container only; the output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

EDGE = (b"foo foobar fox food foo\nxfoo fo foofoo bar barn ba baz bazaar\n"
        b"ab a b aab abb abab xy xyy x y yy xyxy 123 a1 1a foo1 42x\n"
        b"lorem ipsum dolor sit amet, dolorem sitis dolor-sit\n"
        b"caf\xc3\xa9 foo\xc3\xa9 \xc3\xa9foo \xe4\xb8\xad\xe6\x96\x87 foo\xe4\xb8\xad\n\nlast foo")

PATTERNS = [
    # (mode, regex): re = Unicode (ugrep's default), reU = -U (bytes)
    ("reU", r"(?^foo)|f\w+"),
    ("re", r"(?^foo)|f\w+"),
    ("reU", r"(?^fo+)|(?^bar)|f\w+|b\w+"),
    ("reU", r"(?^ba[rz])|[a-z]+"),
    ("reU", r"(?^foo)|bar|baz"),
    ("reU", r"(?^foo)|foo\w*"),
    ("re", r"(?^lorem)|\w+"),
    ("reU", r"(?^dolor)|(?^sit)|[a-z]+"),
    ("reU", r"(?^[0-9]+)|\w+"),
    ("reU", r"(?^a+)|b+"),
    ("reU", r"(?^ab)|a|b"),
    ("reU", r"(?^xy+)|x|y+"),
    ("reU", r"(?^dolor)|dolor\w*|sit"),
    ("reU", r"f\w+|(?^foo)"),
]


def inputs():
    # (name, spec, with the full match list)
    out = [("edge", "hex:" + EDGE.hex(), True), ("Hello.java", "file:" + os.path.join(GOLDEN, "verify", "Hello.java"), True),
           ("lorem.utf8.txt", "file:" + os.path.join(GOLDEN, "verify", "lorem.utf8.txt"), False)]
    for kind in (1, 3, 4):
        out.append(("gen%d_256k" % kind, "gen:%d:5:0:262144" % kind, False))
    return out


def run(args):
    r = subprocess.run([HARNESS] + args, capture_output=True)
    if r.returncode:
        return None
    return r.stdout.decode()


def main(word=False):
    """word: ugrep -w -N (Matcher option W, harness mode suffix "W"), written
    to redo_w_cases.json"""
    cases = []
    ins = inputs()
    for mode, rx in PATTERNS:
        if word:
            mode += "W"
        d = run(["dump", mode.rstrip("W"), rx])
        if d is None:
            print("skip (reference refuses): %s" % rx, file=sys.stderr)
            continue
        dd = json.loads(d)
        res = []
        for name, spec, full in ins:
            out = run(["find", mode, rx, spec] + (["list"] if full else []))
            if out is None:
                continue
            lines = out.strip().split("\n")
            cnt, dg, dc = (int(x) for x in lines[0].split())
            lst = [[int(v) for v in ln.split()] for ln in lines[1:]] if full else None
            res.append(dict(input=name, count=cnt, digest=dg, dcap=dc, list=lst))
        cases.append(dict(pattern=rx, mode=mode, opc=dd["opc"], conv=dd["conv_hex"], results=res))
    meta = dict(edge_hex=EDGE.hex(), inputs=[dict(name=n, spec=s.replace(REPO + "/", "")) for n, s, _ in ins])
    out = os.path.join(GOLDEN, "redo_w_cases.json" if word else "redo_cases.json")
    with open(out, "w") as f:
        json.dump(dict(meta=meta, cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main(word="--word" in sys.argv[1:])
