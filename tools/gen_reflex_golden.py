#!/usr/bin/env python3
"""Generate tests/golden/reflex_cases.npz: for every case of compile_cases.npz
(same patterns and modes), the regex the reference Pattern holds after ugrep's
conversion -- Pattern::operator[](0), its public accessor
(include/reflex/pattern.h:302) -- and the reference's opcode words.  This is
what the drop-in adapter compiles with ugpu_compile(..., UGPU_RX_REFLEX)
(integration/reflex_gpu_matcher.h), so tests/test_compile.py can pin that mode
to the reference tables without reading any private Pattern member.

Build container only (oracle/_ref/ref_harness, libreflex compiled from
/root/reference); the output is data, committed."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
EXTRA = [("re", "x(?i)ab|cd"), ("re", "(?i)a(?-i)b"), ("re", "a(?i:b)c"), ("i", "[^a-z]+"), ("F", "a\\Q.E"),
         ("re", r"[\x00-\x1f]+"), ("re", r"\\\[\]"), ("re", "(a|b)*c{2,3}"), ("W", r"\w+"), ("i", "(?:x|Y)z")]


def main():
    z = np.load(os.path.join(REPO, "tests", "golden", "compile_cases.npz"))
    cases = [(str(m), p.decode("utf-8")) for m, p in zip(z["modes"], z["patterns"])] + EXTRA
    modes, convs, offs, words = [], [], [0], []
    for mode, rx in cases:
        hmode, hrx = {"re": ("re", rx), "F": ("F", rx), "i": ("re", "(?i)" + rx), "W": ("re", rx)}[mode]
        r = subprocess.run([HARNESS, "dump", hmode, hrx], capture_output=True)
        if r.returncode:
            continue  # the reference rejects it: nothing to convert
        j = json.loads(r.stdout)
        if len(j["opc"]) > 40000:
            continue
        modes.append(mode)
        convs.append(bytes.fromhex(j["conv_hex"]))
        words.extend(j["opc"])
        offs.append(len(words))
    out = os.path.join(REPO, "tests", "golden", "reflex_cases.npz")
    roffs = np.cumsum([0] + [len(c) for c in convs]).astype(np.int64)
    np.savez_compressed(out, modes=np.array(modes), regex=np.frombuffer(b"".join(convs), np.uint8),
                        roffsets=roffs, offsets=np.array(offs, np.int64), words=np.array(words, np.uint32))
    print("%d cases, %d words -> %s (%d bytes)" % (len(convs), len(words), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
