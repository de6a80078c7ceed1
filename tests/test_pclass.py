"""\\p{NAME} in the native compiler (missing 4: "the rarer \\p{...}
scripts" were refused, so the drop-in adapter left such patterns on the CPU).

Since round 6 the compiler knows every name the reference's range[] tables
define (lib/language_scripts.cpp, lib/unicode.cpp): all scripts, the
identifier classes, Unicode / Non_ASCII_Unicode, C / Other and the one-letter
aliases, with ranges measured on the reference matcher
(tools/gen_unicode_ranges.py -> ugrep_amd/csrc/unicode_ranges.inc).

Parity: tests/golden/pclass_cases.json (tests/golden/make_pclass_golden.py,
oracle/_ref/ref_harness) holds the reference's tables of \\p{NAME}+ for 66
names and 8 other quantified forms; the compiled table must be
language-equivalent to each (ugrep's own converted regex compiled with
UGPU_RX_REFLEX, as the adapter does, and the ERE form).  The ERE form
reproduces a quirk of Matcher::convert: a class whose UTF-8 encoding is one
byte sequence with leading single bytes is pasted in ungrouped, so a quantifier
binds to its last atom (\\p{Ogham}+ is \\xe1\\x9a[\\x80-\\x9c]+, which also
matches invalid UTF-8 such as E1 9A 80 80): 28 names have that shape."""
import json
import os

import pytest

from oracle_lib import GOLDEN

with open(os.path.join(GOLDEN, "pclass_cases.json")) as _f:
    CASES = json.load(_f)["cases"]


def test_fixture():
    assert len(CASES) >= 70 and all(c["opc"] for c in CASES)


def test_compiled_classes_equal_reference():
    import ugrep_amd as U
    from ugrep_amd.matcher import host_equivalent
    for c in CASES:
        conv = bytes.fromhex(c["conv"])
        assert host_equivalent(U.compile_regex(conv, reflex=True), c["opc"]), c["name"]
        assert host_equivalent(U.compile_regex(c["pattern"]), c["opc"]), c["name"]


@pytest.mark.parametrize("name", ["Tangut", "Linear_B", "Egyptian_Hieroglyphs", "Old_Italic", "Nko", "SignWriting",
                                  "UnicodeIdentifierPart", "Non_ASCII_Unicode", "Unicode", "Other"])
def test_more_names_compile(name):
    import ugrep_amd as U
    U.compile_regex(r"\p{%s}+" % name)
    U.compile_regex(r"[\p{%s}x]" % name)
    if name != "Unicode":  # (\P{Unicode} is empty: the reference refuses it)
        U.compile_regex(r"\P{%s}" % name)


def test_unknown_name_still_refused():
    import ugrep_amd as U
    with pytest.raises((U.Unsupported, U.UgpuError)):
        U.compile_regex(r"\p{NoSuchScript}")
