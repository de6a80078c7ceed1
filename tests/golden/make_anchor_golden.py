#!/usr/bin/env python3
"""Generate tests/golden/anchor_cases.json: reference results for line anchors
(^ and $, META_BOL / META_EOL edges) and for option N (ugrep -Y; also -x,
src/ugrep.cpp:8381-8386), from the reference harness (oracle/_ref/ref_harness:
libreflex compiled from /root/reference, reflex::Matcher(pat, input, "N")).

Each case: the ugrep-converted pattern's opcode words (as ugpu_dfa_create gets
them), and per input the reference's count/digest/dcap (plus the full match
list for inputs up to 64 KiB) with the Matcher's match predictor switched off
(harness mode suffix "P": every position is a FIND candidate, which leaves the
DFA semantics of lib/matcher.cpp:125-546 -- what the engine implements), and,
where it differs, "run": the same Matcher as ugrep runs it (predictor on).  The
two differ where the reference's predictor rejects a position the DFA matches
at through a meta edge: anchored patterns without option N (ugrep sets N for
every pattern that starts with ^ or ends with $, src/cnf.hpp:201-206, and for
-x) and interior anchors such as "a$|ab".  Patterns: ugrep -x wrappers ^(?:P)$
(src/cnf.hpp:167-185), ^P, P$, ^$, mixed alternatives, empty-matching patterns;
inputs: a hand-made text with empty lines, CR LF, lone CR, a last line without
a newline and leading newlines, the reference's CLI inputs, and corpus slices.

Build container only; the output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

EDGE = (b"\nfoo\nbar\n\nxfoo\r\nbaar\r\n\r\nfoo bar\nfoo\rbar\nHello\n  \n\t\nab12\nAB\nfoofoo\n"
        b"caf\xc3\xa9\n\xc3\xa9t\xc3\xa9 foo\nbaz\r\n\nlast foo")

PATTERNS = [
    # ugrep -x wrappers (CNF::anchor), plain and with alternations / empty-matching bodies
    "^(?:foo|ba+r)$", "^(?:Hello)$", "^(?:foo)$", "^(?:\\w+)$", "^(?:.*)$", "^(?:a*)$", "^(?:[a-z ]*)$",
    "^(?:\\s*)$", "^(?:\\w+ \\w+)$", "^(?:foo|)$", "^(?:[^\\n]*r)$", "^(?:café|été foo)$",
    # line anchors alone and mixed
    "^$", "^", "$", "^foo", "foo$", "^\\w+", "\\w+$", "^[A-Z]", "[0-9]+$", "^a|b", "a$|ab", "^foo|bar$",
    "^(foo|bar)+", "(foo|bar)+$", "^.", ".$", "^ *", " *$", "^\\s*$",
    # empty-matching patterns without anchors (option N)
    "a*", "x?", "\\w*", "(foo)?", "o*",
    # interior anchors (ugrep runs these without N unless -Y)
    "(^foo)", "(bar$)", "a$|ab", "x|^y", "(^|,)foo", "foo($|,)",
]
MODES = ["re", "reN", "reU", "reUN"]


def inputs():
    # (name, spec, with the full match list)
    out = [("edge", "hex:" + EDGE.hex(), True), ("Hello.java", "file:" + os.path.join(GOLDEN, "verify", "Hello.java"), True),
           ("lorem.utf8.txt", "file:" + os.path.join(GOLDEN, "verify", "lorem.utf8.txt"), False)]
    for kind in (1, 3, 4):
        out.append(("gen%d_256k" % kind, "gen:%d:5:0:262144" % kind, False))
        out.append(("gen%d_4m" % kind, "gen:%d:6:0:4194304" % kind, False))
    return out


def run(args):
    r = subprocess.run([HARNESS] + args, capture_output=True)
    if r.returncode:
        return None
    return r.stdout.decode()


def main():
    cases = []
    ins = inputs()
    for rx in PATTERNS:
        for mode in MODES:
            base = mode.rstrip("N")
            d = run(["dump", base, rx])
            if d is None:
                continue
            dd = json.loads(d)
            opc = dd["opc"]
            res = []
            for name, spec, full in ins:
                out = run(["find", mode + "P", rx, spec] + (["list"] if full else []))
                ran = run(["find", mode, rx, spec])
                if out is None or ran is None:
                    continue
                lines = out.strip().split("\n")
                cnt, dg, dc = (int(x) for x in lines[0].split())
                lst = [[int(v) for v in ln.split()] for ln in lines[1:]] if full else None
                r = [int(x) for x in ran.strip().split("\n")[0].split()]
                res.append(dict(input=name, count=cnt, digest=dg, dcap=dc, list=lst,
                                run=None if r == [cnt, dg, dc] else r))
            # conv: the regex the Pattern holds ((?m) + Matcher::convert output),
            # what the drop-in adapter hands to ugpu_compile(UGPU_RX_REFLEX)
            cases.append(dict(pattern=rx, mode=mode, nul=mode.endswith("N"), opc=opc, conv=dd["conv_hex"], results=res))
    meta = dict(edge_hex=EDGE.hex(), inputs=[dict(name=n, spec=s.replace(REPO + "/", "")) for n, s, _ in ins])
    out = os.path.join(GOLDEN, "anchor_cases.json")
    with open(out, "w") as f:
        json.dump(dict(meta=meta, cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
