#!/usr/bin/env python3
"""Generate tests/golden/verify_cases.json: a subset of the reference's own CLI
test suite (tests/verify.sh) with the SHA-256 and size of each expected output
file (tests/out/*.out), so the drop-in ugrep build (oracle/_ref/ugrep_gpu:
ugrep's sources with reflex::GpuMatcher at its Matcher construction sites) can
be checked on the GPU box byte for byte against the reference's goldens without
committing 13 MB of outputs.  Inputs are the suite's own files, copied to
tests/golden/verify/.

Cases (each as the suite runs it, UG = ugrep --color=always --sort):
  verify.sh:262-279  for PAT in '' Hello '\\w+[\\n\\h]+\\S+' '\\S\\n\\S' nomatch,
                     OUT '' only, every OPS: UG -U $OPS "$PAT" $FILES
  verify.sh:300-335  -Iw -Ix -F -Fw -Fx -G -Gw -Gx per PAT
  verify.sh:186-203  -iwco -f lorem over the UTF-8/16/32 and (stdin patterns,
                     --encoding=LATIN1) Latin-1 files, for '' -F -G
  verify.sh:354-365  --bool queries (several matchers per query, :8920)
Build container only (reads /root/reference/tests/out); the output is data."""
import hashlib
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = "/root/reference/tests/out"
FILES = ["Hello.bat", "Hello.class", "Hello.java", "Hello.pdf", "Hello.sh", "Hello.txt", "empty.txt", "emptyline.txt"]
UG = ["--color=always", "--sort"]


def fn(prefix, pat, keep="[:alnum:]_"):
    allowed = re.compile(r"[A-Za-z0-9_]" if keep == "[:alnum:]_" else r"[A-Za-z0-9_\-]")
    return "".join(c for c in prefix + pat if allowed.match(c))


def main():
    cases = []

    def add(args, out, stdin=None):  # stdin: name of an input file piped in
        path = os.path.join(OUT, out)
        if not os.path.exists(path):
            return
        data = open(path, "rb").read()
        cases.append({"args": UG + args, "stdin": stdin, "expect": out,
                      "sha256": hashlib.sha256(data).hexdigest(), "size": len(data)})

    for pat in ["", "Hello", r"\w+[\n\h]+\S+", r"\S\n\S", "nomatch"]:
        f = fn("Hello_", pat)
        for ops in ["", "-l", "-lv", "-c", "-co", "-cv", "-n", "-nkbT", "-unkbT", "-o", "-on", "-onkbT", "-ounkbT",
                    "-v", "-nv", "-C2", "-nC2", "-vC2", "-nvC2", "-onC10", "-y", "-ny", "-vy", "-nvy"]:
            add(["-U"] + ([ops] if ops else []) + [pat] + FILES, f + ops + ".out")
        for ops in ["-Iw", "-Ix", "-F", "-Fw", "-Fx"]:
            add(["-U", ops, pat] + FILES, f + ops + ".out")
        gpat = r"\w\+[\n\h]\+\S\+" if pat == r"\w+[\n\h]+\S+" else pat
        for ops in ["-G", "-Gw", "-Gx"]:
            add(["-U", ops, gpat] + FILES, f + ops + ".out")
    for ops in ["", "-F", "-G"]:
        for name in ["lorem.utf8.txt", "lorem.utf16.txt", "lorem.utf32.txt"]:
            add(([ops] if ops else []) + ["-iwco", "-f", "lorem", name], "lorem.utf8%s-iwco.out" % ops)
        add(([ops] if ops else []) + ["-iwco", "--encoding=LATIN1", "-f", "-", "lorem.latin1.txt"],
            "lorem.latin1%s-iwco.out" % ops, stdin="lorem")
    for pat in ["", "Hello World", "Hello -World", "Hello -bin", "bin -Hello", "bin -greeting", "Hello -World|greeting",
                "Hello -bin|greeting", "Hello -(greeting|World)", '"a Hello" greeting']:
        f = fn("Hello_", pat, keep="[:alnum:]_-")
        for ops in ["", "-l", "-c", "-co", "-o", "-C2", "-y", "--json"]:
            add(["-U", "--bool"] + ([ops] if ops else []) + [pat] + FILES, f + "--bool" + ops + ".out")
    dst = os.path.join(REPO, "tests", "golden", "verify_cases.json")
    with open(dst, "w") as fo:
        json.dump({"source": "tests/verify.sh + tests/out/*.out of the reference (sha256 of each expected output)",
                   "env": {"GREP_COLORS": "cx=hb:ms=hug:mc=ib+W:fn=h35:ln=32h:cn=1;32:bn=1;32:se=+36"},  # verify.sh:116
                   "files": FILES, "cases": cases}, fo, indent=0)
    print("%d cases -> %s" % (len(cases), dst))


if __name__ == "__main__":
    main()
