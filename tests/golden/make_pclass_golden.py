#!/usr/bin/env python3
"""Generate tests/golden/pclass_cases.json: the reference's tables for
\\p{NAME} classes the native compiler learned in round 6 (every name the
reference's range[] tables define, lib/language_scripts.cpp, lib/unicode.cpp;
ranges measured by tools/gen_unicode_ranges.py).

Per name: the converted regex (what ugrep hands its Pattern) and the
reference's opcode words for \\p{NAME}+ in Unicode mode, from the reference
harness (oracle/_ref/ref_harness: libreflex compiled from /root/reference).
A sample of scripts, identifier classes and the aliases, kept small: the
large classes' tables run to hundreds of KiB.

Build container only; the output is data, committed."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
GOLDEN = os.path.join(REPO, "tests", "golden")

NAMES = ["Adlam", "Ahom", "Avestan", "Balinese", "Bopomofo", "Braille", "Cherokee", "Coptic", "Deseret", "Glagolitic",
         "Gothic", "Gujarati", "Gurmukhi", "Kannada", "Khmer", "Lao", "Malayalam", "Mongolian", "Myanmar", "Ogham",
         "Runic", "Sinhala", "Syriac", "Tagalog", "Telugu", "Thaana", "Tibetan", "Tifinagh", "Vai", "Yi", "Tangut",
         "Inherited", "JavaIdentifierStart", "CsIdentifierStart", "PythonIdentifierStart", "IdentifierIgnorable",
         "d", "l", "s", "u", "w"]


# Matcher::convert pastes a class in as its UTF-8 regex text, grouped only when
# that has alternatives: these classes are one byte sequence with leading single
# bytes, so a quantifier binds to the sequence's last atom (\p{Ogham}+ is
# \xe1\x9a[\x80-\x9c]+); every such name the reference defines, and other quantifiers
QUIRK = ["Braille", "Buhid", "Dogra", "Elbasan", "Elymaic", "Hanunoo", "Line_Separator", "Lycian", "Mahajani",
         "Makasar", "Meroitic_Hieroglyphs", "Nag_Mundari", "Ogham", "Ol_Chiki", "Old_North_Arabian", "Old_Permic",
         "Old_Sogdian", "Old_South_Arabian", "Palmyrene", "Paragraph_Separator", "Pau_Cin_Hau", "Phags_Pa", "Shavian",
         "Syloti_Nagri", "Thaana", "Toto", "Zl", "Zp"]
MORE = [r"\p{Ogham}{2}", r"\p{Zl}*x", r"\p{Braille}?y", r"x\p{Thaana}{2,3}", r"(\p{Ogham})+", r"[\p{Ogham}]+",
        r"\p{Ogham}|\p{Thaana}+", r"\p{Zp}{1,2}\p{Ogham}*"]


def main():
    cases = []
    pats = [(n, r"\p{%s}+" % n) for n in NAMES + [q for q in QUIRK if q not in NAMES]] + [(None, r) for r in MORE]
    for name, rx in pats:
        r = subprocess.run([HARNESS, "dump", "re", rx], capture_output=True)
        if r.returncode:
            cases.append(dict(name=name, pattern=rx, opc=None))
            continue
        d = json.loads(r.stdout)
        cases.append(dict(name=name, pattern=rx, conv=d["conv_hex"], opc=d["opc"]))
    out = os.path.join(GOLDEN, "pclass_cases.json")
    with open(out, "w") as f:
        json.dump(dict(cases=cases), f, separators=(",", ":"))
    print("%d cases -> %s (%d bytes)" % (len(cases), out, os.path.getsize(out)), file=sys.stderr)


if __name__ == "__main__":
    main()
