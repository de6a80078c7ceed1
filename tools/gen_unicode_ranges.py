#!/usr/bin/env python3
"""Generate ugrep_amd/csrc/unicode_ranges.inc: the code point ranges of the
Unicode classes \\w (Word), \\d (Nd) and \\s (Space) as the reference defines
them in Unicode mode (include/reflex/unicode.h, lib/unicode.cpp:96,
lib/language_scripts.cpp:11317 "Word").

The reference's Unicode version differs from this image's unicodedata (13.0)
and regex (17.0) modules, so the ranges are measured on the reference matcher
itself: every Unicode scalar value (minus '\\n') is encoded as UTF-8 on a line
of its own and scanned with the reference's compiled DFA for the class
(oracle/_ref/ref_harness dump, build container only); a code point is in the
class iff the class matches exactly its encoding.  The output is data (ranges),
committed; this script runs only where /root/reference is present.
"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from oracle_lib import OracleDfa  # noqa: E402

HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")


def ref_opc(rx):
    out = subprocess.run([HARNESS, "dump", "re", rx], capture_output=True, check=True).stdout
    return json.loads(out)["opc"]


def members(rx):
    cps = [c for c in range(0x110000) if not 0xD800 <= c < 0xE000 and c != 10]
    parts, where, pos = [], {}, 0
    for c in cps:
        b = chr(c).encode("utf-8")
        where[(pos, len(b))] = c
        parts.append(b + b"\n")
        pos += len(b) + 1
    buf = np.frombuffer(b"".join(parts), np.uint8)
    _, _, _, lst = OracleDfa(ref_opc(rx)).find(buf, want_list=True)
    return sorted(where[(s, ln)] for s, ln, _ in lst if (s, ln) in where)


def ranges(cps):
    out = []
    for c in cps:
        if out and out[-1][1] + 1 == c:
            out[-1][1] = c
        else:
            out.append([c, c])
    return out


# \p{NAME} classes (lib/unicode.cpp, lib/language_scripts.cpp): general
# categories, their long names, common scripts and the POSIX-style names that
# [[:name:]] brackets also use (lib/posix.cpp, pattern.cpp posix_class[])
CATEGORIES = ["L", "Lu", "Ll", "Lt", "Lm", "Lo", "M", "Mn", "Mc", "Me", "N", "Nd", "Nl", "No", "P", "Pd", "Ps",
              "Pe", "Pi", "Pf", "Pc", "Po", "S", "Sm", "Sc", "Sk", "So", "Z", "Zs", "Zl", "Zp", "Cc", "Cf"]
LONG = {"Letter": "L", "Mark": "M", "Number": "N", "Punctuation": "P", "Symbol": "S", "Separator": "Z",
        "Lowercase_Letter": "Ll", "Uppercase_Letter": "Lu", "Titlecase_Letter": "Lt", "Modifier_Letter": "Lm",
        "Other_Letter": "Lo", "Non_Spacing_Mark": "Mn", "Spacing_Combining_Mark": "Mc", "Enclosing_Mark": "Me",
        "Space_Separator": "Zs", "Line_Separator": "Zl", "Paragraph_Separator": "Zp", "Math_Symbol": "Sm",
        "Currency_Symbol": "Sc", "Modifier_Symbol": "Sk", "Other_Symbol": "So", "Decimal_Digit_Number": "Nd",
        "Letter_Number": "Nl", "Other_Number": "No", "Dash_Punctuation": "Pd", "Open_Punctuation": "Ps",
        "Close_Punctuation": "Pe", "Initial_Punctuation": "Pi", "Final_Punctuation": "Pf",
        "Connector_Punctuation": "Pc", "Other_Punctuation": "Po", "Control": "Cc", "Format": "Cf"}
SCRIPTS = ["Latin", "Greek", "Cyrillic", "Armenian", "Hebrew", "Arabic", "Devanagari", "Bengali", "Tamil", "Thai",
           "Georgian", "Hangul", "Hiragana", "Katakana", "Han", "Ethiopic", "Common"]
# (round 6) every other name the reference's \\p{NAME} accepts (lib/language_scripts.cpp,
# lib/unicode.cpp range[...]): the remaining scripts, the identifier classes
# (Java/C#/Python/Unicode identifier parts and starts), Unicode,
# Non_ASCII_Unicode, C / Other and the one-letter aliases
MORE = ["Adlam", "Ahom", "Anatolian_Hieroglyphs", "Avestan", "Balinese", "Bamum", "Bassa_Vah", "Batak",
        "Bhaiksuki", "Bopomofo", "Brahmi", "Braille", "Buginese", "Buhid", "C", "Canadian_Aboriginal", "Carian",
        "Caucasian_Albanian", "Chakma", "Cham", "Cherokee", "Chorasmian", "Coptic", "CsIdentifierPart",
        "CsIdentifierStart", "Cuneiform", "Cypriot", "Cypro_Minoan", "Deseret", "Dives_Akuru", "Dogra", "Duployan",
        "Egyptian_Hieroglyphs", "Elbasan", "Elymaic", "Glagolitic", "Gothic", "Grantha", "Gujarati",
        "Gunjala_Gondi", "Gurmukhi", "Hanifi_Rohingya", "Hanunoo", "Hatran", "IdentifierIgnorable",
        "Imperial_Aramaic", "Inherited", "Inscriptional_Pahlavi", "Inscriptional_Parthian", "JavaIdentifierPart",
        "JavaIdentifierStart", "Javanese", "Kaithi", "Kannada", "Kawi", "Kayah_Li", "Kharoshthi",
        "Khitan_Small_Script", "Khmer", "Khojki", "Khudawadi", "Lao", "Lepcha", "Limbu", "Linear_A", "Linear_B",
        "Lisu", "Lycian", "Lydian", "Mahajani", "Makasar", "Malayalam", "Mandaic", "Manichaean", "Marchen",
        "Masaram_Gondi", "Medefaidrin", "Meetei_Mayek", "Mende_Kikakui", "Meroitic_Cursive",
        "Meroitic_Hieroglyphs", "Miao", "Modi", "Mongolian", "Mro", "Multani", "Myanmar", "Nabataean",
        "Nag_Mundari", "Nandinagari", "New_Tai_Lue", "Newa", "Nko", "Non_ASCII_Unicode", "Nushu",
        "Nyiakeng_Puachue_Hmong", "Ogham", "Ol_Chiki", "Old_Hungarian", "Old_Italic", "Old_North_Arabian",
        "Old_Permic", "Old_Persian", "Old_Sogdian", "Old_South_Arabian", "Old_Turkic", "Old_Uyghur", "Oriya",
        "Osage", "Osmanya", "Other", "Pahawh_Hmong", "Palmyrene", "Pau_Cin_Hau", "Phags_Pa", "Phoenician",
        "Psalter_Pahlavi", "PythonIdentifierPart", "PythonIdentifierStart", "Rejang", "Runic", "Samaritan",
        "Saurashtra", "Sharada", "Shavian", "Siddham", "SignWriting", "Sinhala", "Sogdian", "Sora_Sompeng",
        "Soyombo", "Sundanese", "Syloti_Nagri", "Syriac", "Tagalog", "Tagbanwa", "Tai_Le", "Tai_Tham", "Tai_Viet",
        "Takri", "Tangsa", "Tangut", "Telugu", "Thaana", "Tibetan", "Tifinagh", "Tirhuta", "Toto", "Ugaritic",
        "Unicode", "UnicodeIdentifierPart", "UnicodeIdentifierStart", "Vai", "Vithkuqi", "Wancho", "Warang_Citi",
        "Yezidi", "Yi", "Zanabazar_Square", "d", "l", "s", "u", "w"]
POSIX = ["ASCII", "Space", "XDigit", "Cntrl", "Print", "Alnum", "Alpha", "Blank", "Digit", "Graph", "Lower",
         "Punct", "Upper", "Word"]


def has_newline(rx):
    """'\\n' is a member when the start state's transition on 0x0A accepts."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from dfa_equiv import _parse_opc
    nxt, caps = _parse_opc(ref_opc(rx))
    return bool(caps[nxt[1][10]])


def emit(lines, cname, cps, nl):
    r = ranges(sorted(set(cps) | ({10} if nl else set())))
    lines.append("static const uint32_t %s[][2] = {" % cname)
    for i in range(0, len(r), 6):
        lines.append("  " + " ".join("{0x%X, 0x%X}," % (a, b) for a, b in r[i:i + 6]))
    lines.append("};")
    lines.append("")
    return len(r)


def main():
    lines = ["// GENERATED by tools/gen_unicode_ranges.py -- do not edit.",
             "// Unicode class ranges as the reference defines them (see the script's docstring).", ""]
    for name, rx in (("word", r"\w"), ("digit", r"\d"), ("space", r"\s")):
        n = emit(lines, "k_%s_ranges" % name, members(rx), False)
        print("%s: %d ranges" % (name, n), file=sys.stderr)
    reg = []
    pnl = {}
    for name in CATEGORIES + SCRIPTS + POSIX + MORE:
        rx = r"\p{%s}" % name
        cname = "k_p_%s" % name
        try:
            cps, nl = members(rx), has_newline(rx)
        except subprocess.CalledProcessError:
            print("\\p{%s}: the reference refuses it, skipped" % name, file=sys.stderr)
            continue
        n = emit(lines, cname, cps, nl)
        try:
            pnl[cname] = int(has_newline(r"\P{%s}" % name))  # '\n' in the complement \P{NAME}
        except subprocess.CalledProcessError:  # (\P{Unicode}: an empty class, which the reference refuses)
            pnl[cname] = 0
        reg.append((name, cname))
        print("\\p{%s}: %d ranges" % (name, n), file=sys.stderr)
    for long, short in LONG.items():
        reg.append((long, "k_p_%s" % short))
    lines.append("typedef struct UClass { const char *name; const uint32_t (*ranges)[2]; unsigned n; int pnl; } UClass;")
    lines.append("static const UClass k_pclasses[] = {")
    for name, cname in reg:
        lines.append("  {\"%s\", %s, sizeof(%s) / sizeof(%s[0]), %d}," % (name, cname, cname, cname, pnl[cname]))
    lines.append("};")
    lines.append("")
    with open(os.path.join(REPO, "ugrep_amd", "csrc", "unicode_ranges.inc"), "w") as f:
        f.write("\n".join(lines))


if __name__ == "__main__":
    main()
