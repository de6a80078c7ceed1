#!/usr/bin/env python3
"""Generate tests/golden/wordb_cases.json: reference results for the word
boundary meta edges \\b \\B \\< \\> (META_WBB .. META_EWE,
include/reflex/pattern.h:933-940; tested by lib/matcher.cpp:317-404 through
include/reflex/matcher.h:1194-1319), from the reference harness
(oracle/_ref/ref_harness: libreflex compiled from /root/reference).

Each case: the ugrep-converted pattern's opcode words (as ugpu_dfa_create gets
them; RE/flex moves begin-of-match assertions to the accept side, so \\bfoo\\b
ends in META_WBE -> META_WBB -> TAKE) and per input the reference's
count/digest/dcap (plus the full match list for small inputs) with the
Matcher's match predictor switched off (harness mode suffix "P": the DFA
semantics the engine implements), and, where it differs, "run": the Matcher
as ugrep runs it.  The two differ where the Pattern's predictor rejects
positions the DFA matches at (\\w+\\b and x\\b|xy print nothing in the
reference CLI); the drop-in adapter keeps those patterns on the CPU matcher
(integration/reflex_gpu_matcher.h predictor_exact).  Inputs: a hand-made
text with every boundary kind next to ASCII, '_', digits, UTF-8 word and
non-word characters, invalid UTF-8, CR LF and a last line without newline;
the reference's CLI inputs; corpus slices.

Build container only; the output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

EDGE = (b"foo bar foo_bar foo-bar foobar barfoo foo\nfoo\r\nx_foo foo1 1foo (foo) [foo]\n"
        b"caf\xc3\xa9 \xc3\xa9t\xc3\xa9 foo\xc3\xa9 \xc3\xa9foo x\xc3\xa9 \xc3\xa9x na\xc3\xafve \xe2\x82\xac5 5\xe2\x82\xac\n"
        b"\xce\xb1\xce\xb2\xce\xb3 foo \xe4\xb8\xad\xe6\x96\x87 foo\xe4\xb8\xad x\xf0\x9f\x98\x80x\n"
        b"bad \xc3( \xc3 x\xc3a x\xa9 \xa9x \xff foo\xc3\n  the them other the\tthe, the.\n"
        b"__ _x_ x__ 12 3.4 a1b2 ab AB Ab\n\nlast foo")

PATTERNS = [
    # at both ends, at one end, each kind
    r"\bfoo\b", r"\bfoo", r"foo\b", r"\<foo", r"foo\>", r"\<foo\>", r"\Bfoo", r"foo\B", r"\Boo\B",
    r"\>foo", r"foo\<", r"\bx", r"x\b", r"\Bx", r"x\B", r"\<x", r"x\>", r"\bthe\b", r"\Bthe",
    # classes, Unicode, alternation, fixed repeats
    r"\b\w\w\b", r"\b[a-z]{3}\b", r"\b\d\b", r"\b\d+\.\d+\b", r"\bé", r"é\b", r"\bété\b", r"\b\p{L}\b",
    r"\b[^a-z ]\b", r"\b_", r"_\b", r"\b\s", r"\s\b", r"\bfoo\b|\bbar\b", r"\<(foo|bar)\>", r"\bfoo|bar",
    r"\bdolor\b|\bdolore\b", r"\b(foo|foobar)\b", r"\bfo\b|\bfoo\b", r"\bLorem\b", r"\bHello\b",
    # loops before the assertion (the predictor rejects matches here)
    r"\w+\b", r"\b\w+\b", r"\<\w+\>", r"\b[a-z]+\b", r"x\b|xy", r"foo.\b", r"\b.\b", r"[a-z]+\B",
    # an assertion between consumed bytes (its meta target consumes: the engine refuses)
    r"a\Bb", r"foo\b bar",
    # with line anchors
    r"^foo\b", r"\bfoo$", r"^\<\w\w\>$",
    # assertions alone
    r"\b", r"\B", r"\<", r"\>",
    # alternatives ending at the same byte under different assertions: the
    # accept is the first meta edge that holds in descending META code, not
    # the lowest satisfied index (^ab|ab$ with both: 2)
    r"\bé|é\b|\Bx\B", r"\bab|ab\b", r"ab\>|ab|\bab", r"\bab\b|ab\b", r"^ab|ab$", r"^ab$|ab$", r"\bfoo\b|foo",
    r"\<the|the\>|\Bthe",
    # the adapter rule's boundary: finite alternations whose
    # branches share a prefix under different boundary kinds, and \b after a
    # fixed repeat of classes -- finite, so the rule sends them to the GPU
    r"\bfoo\b|\bfoo\B", r"\bab\b|\Bab", r"foo\>|foob\b", r"\<fo|\<foo\>", r"\b(a|ab|abc)\b",
    r"(foo|fo)\b", r"\b\w{3}\b", r"\b[a-z]{2}\d\b", r"\<\w{2}\>", r"\b\d{2,3}\b", r"\b.{2}\b",
    r"\bx\w\b", r"\b[[:alpha:]]{3}\b|\bfoo",
]
MODES = ["re", "reN", "reU"]


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
            cases.append(dict(pattern=rx, mode=mode, nul=mode.endswith("N"), opc=dd["opc"], conv=dd["conv_hex"],
                              pred=dict(len=dd["len"], min=dd["min"], pin=dd["pin"], lbk=dd["lbk"]), results=res))
    meta = dict(edge_hex=EDGE.hex(), inputs=[dict(name=n, spec=s.replace(REPO + "/", "")) for n, s, _ in ins])
    out = os.path.join(GOLDEN, "wordb_cases.json")
    with open(out, "w") as f:
        json.dump(dict(meta=meta, cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
