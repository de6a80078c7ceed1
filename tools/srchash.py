"""Source hash of the engine library (ugrep_amd/csrc/* and include/ugpu.h, in
C-locale name order): the Makefile embeds it in libugrep_amd.so
(ugpu_build_id), and ugrep_amd/_lib.py warns when the library loaded was not
built from the sources beside it."""
import hashlib
import os
import sys


def srchash(repo):
    h = hashlib.sha256()
    csrc = os.path.join(repo, "ugrep_amd", "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith((".hip", ".hpp", ".cpp", ".inc", ".h")))
    files.append(os.path.join(repo, "include", "ugpu.h"))
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(srchash(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
