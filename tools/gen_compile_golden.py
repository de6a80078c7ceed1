#!/usr/bin/env python3
"""Generate tests/golden/compile_cases.npz: reference opcode tables for the
regex compiler's parity tests (tests/test_compile.py).

For each case (pattern, mode) the reference Pattern is built by
oracle/_ref/ref_harness dump (libreflex compiled from /root/reference, the
conversion ugrep applies: Matcher::convert("(?m)"+rx, notnewline|unicode),
src/ugrep.cpp:8574-8590; -F quotes with \\Q..\\E, -i prefixes (?i)).  Stored:
the opcode words, or an empty table when the reference rejects the pattern
(regex_error).  Build container only (needs the reference build); the
output is data, committed.  Cases: a hand list of constructs and edge cases,
plus seeded random patterns over a grammar of the supported syntax.
"""
import json
import os
import random
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")

HAND = [
    # BASELINE configs
    ("re", "foo|bar|baz"), ("re", "[A-Za-z_][A-Za-z0-9_]*"), ("re", r"\w+"), ("F", "lorem"), ("re", "lorem"),
    # dot forms (convert.cpp:2118-2160) and newline handling
    ("re", "a.b"), ("re", ".*x"), ("re", ".+"), ("re", ".."), ("re", "x.?y"), ("re", "\\n"), ("re", "[\\n]"),
    # accept indices of top-level alternatives
    ("re", "a|a"), ("re", "a|ab|a."), ("re", "a|b|"), ("re", "x*"), ("re", ""), ("re", "(foo|bar)|baz"),
    # classes
    ("re", r"\s"), ("re", r"\S"), ("re", r"\W"), ("re", r"\D"), ("re", r"\H"), ("re", r"\h+"), ("re", r"\d+\.\d*"),
    ("re", r"[^\w]"), ("re", "[^a]"), ("re", r"[\W]"), ("re", r"[\S]"), ("re", r"[\D]"), ("re", r"[\H]"),
    ("re", r"[\W\d]"), ("re", r"[^\W]"), ("re", r"[^\S]"), ("re", r"[a\W]"), ("re", r"x[\S]y"),
    ("re", "[]a]"), ("re", "[a-]"), ("re", r"[\x00-\x7f]"), ("re", r"[^\x00-\x7f]"), ("re", "[α-ω]+"),
    # literals and escapes
    ("re", "é+"), ("re", r"\xff"), ("re", r"\x{20AC}"), ("re", r"\x{1F600}+"), ("re", "a\\tb"), ("re", r"a\.b\+"),
    ("re", r"\/"), ("re", "😀|€|ж"), ("re", r"\0101"), ("re", "a}"), ("re", "]"), ("re", "a]b"),
    # repeats and groups
    ("re", "a{2,4}"), ("re", "a{3}"), ("re", "a{2,}"), ("re", "x{0}"), ("re", "x{0,0}y"), ("re", "(ab|c)+d?"),
    ("re", "(?:x|y)z"), ("re", "a**"), ("re", r"(\w+\s*){2,3}"), ("re", "(é|ab){1,3}c"),
    # -F quoting (src/cnf.hpp:147-165)
    ("F", "a.b*c"), ("F", "(x|y)"), ("F", "[é]"), ("F", "\\E\\Q"), ("F", ""),
    # -i (ASCII letters)
    ("i", "lorem"), ("i", "k"), ("i", "s"), ("i", "[a-z]+"), ("i", "foo|BAR"), ("i", r"\w+x"),
    # -i over Unicode (case_fold.inc; (?i) leaves \x{..} escapes unfolded)
    ("i", "é"), ("i", "ж"), ("i", "straße"), ("i", "ÉCOLE"), ("i", "[à-ÿ]+"), ("i", "[é]"), ("i", r"\x{e9}"),
    ("i", r"[\x{e9}]"), ("i", r"\x41"), ("i", "Ωμέγα"), ("i", "ǅ"), ("i", "ſ"), ("i", "K"), ("i", "ß"), ("i", "İ"),
    ("i", "ı"), ("i", "[α-ω]"), ("i", r"\p{Greek}"), ("i", "[^é]"), ("i", "Ⓐ"), ("i", "ⅰ"), ("i", r"\W"),
    ("i", r"\p{L}"), ("i", r"\p{Latin}+"), ("i", r"\P{L}"), ("i", r"[\p{Greek}a]"), ("i", "[[:lower:]]"),
    ("i", "[[:alpha:]]+"), ("i", "Straße|ΣΊΣΥΦΟΣ|Привет"),
    # \p{..} classes and POSIX brackets (Unicode tables, lib/unicode.cpp)
    ("re", r"\p{L}"), ("re", r"\p{Lu}+"), ("re", r"\P{L}"), ("re", r"[\p{L}]"), ("re", r"[\P{L}]"),
    ("re", r"[^\p{L}]"), ("re", r"\p{Greek}+"), ("re", r"\p{Han}"), ("re", r"\pL"), ("re", r"\PL"),
    ("re", r"\p{Letter}"), ("re", r"\p{Zs}"), ("re", r"\P{Cc}"), ("re", r"[\P{Cc}]"), ("re", r"\P{Space}"),
    ("re", r"[\P{Zs}]"), ("re", r"[x\P{Lu}]"), ("re", r"\p{L}\p{M}*"), ("re", r"[\p{Han}\p{Hiragana}\p{Katakana}]+"),
    ("re", r"\p{Lu}\p{Ll}+"), ("re", "[[:alpha:]_][[:alnum:]_]*"), ("re", "[[:upper:]]"),
    ("re", "[[:digit:][:space:]]"), ("re", "[[:punct:]]+"), ("re", "[[:xdigit:]]"), ("re", "[[:ascii:]]"),
    ("re", "[[:cntrl:]]"), ("re", "[[:print:]]"), ("re", "[[:graph:]]"), ("re", "[[:word:]]"), ("re", "[[:blank:]]"),
    ("re", "[[:lower:]]"), ("re", r"\p{Common}"), ("re", r"\P{Greek}"), ("re", r"\p{Nd}+|\p{Sc}"),
    ("re", r"\p{Cyrillic}+"), ("re", r"\p{Arabic}\p{Mn}*"),
    # syntax errors (reference throws regex_error)
    ("re", "(|a)"), ("re", "()"), ("re", "{"), ("re", "a{"), ("re", "a{,3}"), ("re", "(a|)"), ("re", "|a"),
    ("re", "[a-z"), ("re", "(a"), ("re", "a)"),
]

ATOMS = ['a', 'b', 'c', 'é', 'ж', '€', '😀', '.', r'\w', r'\d', r'\s', r'\W', r'\S', r'\D', r'\h', r'\H', '[abc]',
         '[^a]', '[a-cé]', r'[^\w]', r'[\d\s]', '[α-ω]', r'\.', r'\x41', 'x', '\t', r'[\W]', '[^ж-я]', '[0-9]',
         r'\x{10000}', r'[\x{80}-\x{7ff}]', r'[^\x{800}-\x{ffff}]', r'\p{L}', r'\P{Lu}', r'[\p{Greek}x]',
         '[[:alpha:]]', r'\p{Nd}']


def random_pattern(rng, d=0):
    r = rng.random()
    if d > 3 or r < 0.35:
        return rng.choice(ATOMS)
    if r < 0.55:
        return random_pattern(rng, d + 1) + random_pattern(rng, d + 1)
    if r < 0.65:
        return '(' + random_pattern(rng, d + 1) + '|' + random_pattern(rng, d + 1) + ')'
    if r < 0.85:
        return '(' + random_pattern(rng, d + 1) + ')' + rng.choice(['*', '+', '?', '{2}', '{1,3}', '{0,2}', '{2,}'])
    return rng.choice(ATOMS) + rng.choice(['*', '+', '?'])


def ref_opc(mode, rx):
    hmode, hrx = {"re": ("re", rx), "F": ("F", rx), "i": ("re", "(?i)" + rx)}[mode]
    r = subprocess.run([HARNESS, "dump", hmode, hrx], capture_output=True)
    return None if r.returncode else json.loads(r.stdout)["opc"]


def main():
    cases = list(HAND)
    rng = random.Random(20261016)
    while len(cases) < len(HAND) + 160:
        rx = random_pattern(rng)
        if rng.random() < 0.3:
            rx += '|' + random_pattern(rng, 1)
        cases.append(("i" if rng.random() < 0.25 else "re", rx))
    modes, pats, offs, words = [], [], [0], []
    for mode, rx in cases:
        opc = ref_opc(mode, rx)
        if opc is not None and len(opc) > 40000:
            continue  # keep the fixture small
        modes.append(mode)
        pats.append(rx)
        words.extend(opc or [])
        offs.append(len(words))
    out = os.path.join(REPO, "tests", "golden", "compile_cases.npz")
    np.savez_compressed(out, modes=np.array(modes), patterns=np.array([p.encode("utf-8") for p in pats], dtype=object)
                        .astype(np.bytes_), offsets=np.array(offs, np.int64), words=np.array(words, np.uint32))
    print("%d cases, %d words -> %s (%d bytes)" % (len(pats), len(words), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
