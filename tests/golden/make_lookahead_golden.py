#!/usr/bin/env python3
"""Generate tests/golden/lookahead_cases.json: reference results for patterns
with lookahead (X(?=Y): the Pattern marks the DFA states where Y starts with
HEAD la and the states where it completes with TAIL la, lib/pattern.cpp:
2953-2964; the FIND walk records the HEAD position and a TAIL moves the match
end back to it, lib/matcher.cpp:157-175, :226-237), from the reference harness
(oracle/_ref/ref_harness: libreflex compiled from /root/reference).

Each case: the converted pattern's opcode words and regex, and per input the
reference Matcher's count/digest/dcap, plus the full match list for the small
inputs.  Inputs: an edge text, tests/golden/verify/Hello.java and the C1-C4
corpora (256 KiB slices).

Build container only; the output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

EDGE = (b"foobar fooba foo bar barfoo fobar foofoobar\nab a b aab abb abab a1 ab1 abc1 1a\n"
        b"xyz xyb xy xyzxyz x yz\nprintf(\"%d\", x); int main(void) { return f(1)(2); }\n"
        b"word. word, words; wordy end.\ncaf\xc3\xa9 foo\xc3\xa9 \xc3\xa9foo \xe4\xb8\xad\xe6\x96\x87 foo\xe4\xb8\xad\n"
        b"12px 3em 4 5px6 77pt p12x\n\nlast foobar")

PATTERNS = [
    # (mode, regex): re = Unicode (ugrep's default), reU = -U (bytes)
    ("reU", r"foo(?=bar)"),
    ("re", r"foo(?=bar)"),
    ("reU", r"fo+(?=ba)|bar"),
    ("reU", r"a(?=b)|ab"),
    ("reU", r"[a-z]+(?=[0-9])"),
    ("reU", r"x(?=y)z|xy"),
    ("reU", r"[0-9]+(?=px|em)"),
    ("reU", r"\w+(?=\()"),
    ("re", r"\w+(?=\()"),
    ("reU", r"word(?=[.,;])|end"),
    ("reU", r"(foo|bar)(?=bar|foo)"),
    ("reU", r"[a-z]+(?=[0-9])|[0-9]+(?=[a-z])"),
    ("reU", r"a(?=b)"),
    ("reU", r"[a-z](?=[a-z]{2})"),
    ("re", r"\w+(?=\s)"),
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


# option W only (ugrep -w): at_we is tested where the TAKE happens, before
# TAIL moves the match end back
W_PATTERNS = [("reU", r"[a-z]+(?= [a-z]+)"), ("reU", r"\w+(?=,)"), ("re", r"\w+(?=\.)"), ("reU", r"in(?=c|t)")]


def main(word=False):
    """word: Matcher option W (harness mode suffix "W"), written to
    lookahead_w_cases.json"""
    cases = []
    ins = inputs()
    for mode, rx in PATTERNS + (W_PATTERNS if word else []):
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
    out = os.path.join(GOLDEN, "lookahead_w_cases.json" if word else "lookahead_cases.json")
    with open(out, "w") as f:
        json.dump(dict(meta=meta, cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main(word="--word" in sys.argv[1:])
