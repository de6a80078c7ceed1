#!/usr/bin/env python3
"""Generate tests/golden/asgroup_cases.json: reference results for patterns
whose line anchors or word boundaries sit inside a group at the start or the
end of a top-level alternative -- (^|,)foo, foo($|,), (\\bfoo|bar) -- from the
reference harness (oracle/_ref/ref_harness: libreflex compiled from
/root/reference).  The native compiler distributes such a group over its
alternative (ugrep_amd/csrc/regex_compile.cpp rx_assertion_groups); the
fixtures pin that the reference matches the same.

Each case: the pattern, the ugrep-converted regex (as the drop-in adapter
compiles it), and per input the reference's count/digest/dcap and match list
with the Matcher's match predictor off (harness mode "reP": the DFA semantics
the engine implements) and, where different, as ugrep runs it ("run").
Patterns the reference rejects are left out.  Build container only; the
output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

EDGE = (b"foo,foo ,foo\nfoo;foo bar\n,bar foo,\nthe the,the\nthem the\n id;id ,id\nid\n"
        b"x_foo foo1 (foo) [foo],foo\r\nfoo\r\nbarfoo foobar bar,bar;bar\n"
        b"caf\xc3\xa9,foo \xc3\xa9foo foo\xc3\xa9 ,\xc3\xa9t\xc3\xa9\n  the\tthe, the.\nlast foo")

PATTERNS = [
    r"(^|,)foo", r"(,|^)foo", r"(?:^|,)foo", r"(^|[,;])(foo|bar)", r"foo($|,)", r"foo(,|$)", r"(^| )the( |$)",
    r"(^|\s)foo(\s|$)", r"((^|,)foo|bar)", r"((^|,)foo|bar)(,|$)", r"(^|;)id\b", r"(?:^|[,;])id\b",
    r"(\bfoo|bar)", r"(foo|\bbar)", r"(\<foo|,bar)", r"(foo\>|bar,)", r"(\bfoo|\bbar)\b", r"(x|\bthe)",
    r"(\Bfoo|;id)", r"(foo|^bar)", r"(^|,)foo|bar", r"the|(^|,)id", r"(^|,)[a-z]+", r"(\b[a-z]+|,)",
    r"(,|\<)[a-z]+(\>|,)", r"(\bfoo|\bbar)(,|\b)",
    # on the reference's CLI inputs (lorem: ", consectetur", ". Sed")
    r"(^|, )[a-z]+", r"(\bdolor|amet,)", r"(^|\. )[A-Z][a-z]+", r"[a-z]+(,|\.|$)", r"(^|\s)(public|class)\b",
]


def inputs():
    return [("edge", "hex:" + EDGE.hex(), True),
            ("lorem.utf8.txt", "file:" + os.path.join(GOLDEN, "verify", "lorem.utf8.txt"), True),
            ("Hello.java", "file:" + os.path.join(GOLDEN, "verify", "Hello.java"), True)]


def run(args):
    r = subprocess.run([HARNESS] + args, capture_output=True)
    if r.returncode:
        return None
    return r.stdout.decode()


def main():
    cases = []
    ins = inputs()
    for rx in PATTERNS:
        d = run(["dump", "re", rx])
        if d is None:
            print("reference rejects", rx, file=sys.stderr)
            continue
        dd = json.loads(d)
        res = []
        for name, spec, full in ins:
            out = run(["find", "reP", rx, spec, "list"])
            ran = run(["find", "re", rx, spec])
            lines = out.strip().split("\n")
            cnt, dg, dc = (int(x) for x in lines[0].split())
            lst = [[int(v) for v in ln.split()] for ln in lines[1:]]
            r = [int(x) for x in ran.strip().split("\n")[0].split()]
            res.append(dict(input=name, count=cnt, digest=dg, dcap=dc, list=lst, run=None if r == [cnt, dg, dc] else r))
        cases.append(dict(pattern=rx, conv=dd["conv_hex"], results=res))
    meta = dict(edge_hex=EDGE.hex(), inputs=[dict(name=n, spec=s.replace(REPO + "/", "")) for n, s, _ in ins])
    out = os.path.join(GOLDEN, "asgroup_cases.json")
    with open(out, "w") as f:
        json.dump(dict(meta=meta, cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
