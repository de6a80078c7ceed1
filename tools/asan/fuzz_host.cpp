// fuzz_host.cpp -- sanitizer harness for the host half (libugpu_host.so:
// the regex compiler, the table builders, the plan).  Built with
// -fsanitize=address,undefined from the same sources (tools/asan/Makefile).
//
// N random patterns from the grammar ugpu_compile supports (literals, classes
// and their negations, \w \d \s \b \< \> ^ $, escapes, groups, alternation,
// the quantifiers ? * + {m,n}, (?^...) negative alternatives, (?=...)
// lookaheads, \p{NAME} classes of one byte sequence), each with
// random flags (-F, -i, RE/flex mode), plus byte-level mutations of them
// (truncations, random bytes, unbalanced brackets: malformed input must fail
// cleanly).  Every pattern that compiles is run through every host entry
// point that takes opcode words: the plan with and without option W / N, the
// dense tables, the context accepts, the prefilter, the transducers, the xc /
// xu tables, the dominated-restart bits and table equivalence.  A sanitizer
// report aborts the run (halt_on_error); the harness itself checks the
// documented contracts (UGPU_OK / UGPU_UNSUPPORTED / UGPU_INVAL only).
#include "ugpu.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

namespace {

std::mt19937_64 rng;

uint32_t rnd(uint32_t n) { return (uint32_t)(rng() % n); }

// (ASCII atoms most of the time: the Unicode classes make large DFAs, and
// the sanitized subset construction is slow on those)
const char* kAtoms[] = {"a", "b", "foo", "x", "[a-z]", "[^a-z]", "[A-Za-z_]", "[0-9]", "\\d", "\\s", ".", "\\.",
                        "\\\\", "[[:digit:]]", "\\x41", "\\n", "\\t", "[-a]", "[a-]", "[]a]", "[^]a]", "\\bfoo",
                        "\\<x", "y\\>", "\\Bz", "^", "$", "ing", "ed", " "};
const char* kWide[] = {"\\w", "\\W", "\\S", "[[:alpha:]]", "\\p{L}", "\\p{Greek}", "é", "€", "中", "[à-ÿ]",
                       "\\p{Ogham}", "\\p{Zl}", "\\p{Braille}", "\\p{Thaana}", "\\p{Tangut}"};

std::string gen(int depth)
{
  std::string s;
  const int n = 1 + (int)rnd(3);
  for (int i = 0; i < n; ++i) {
    const uint32_t k = rnd(depth > 0 ? 10 : 7);
    if (k < 6) {
      s += rnd(12) == 0 ? kWide[rnd(sizeof(kWide) / sizeof(kWide[0]))] : kAtoms[rnd(sizeof(kAtoms) / sizeof(kAtoms[0]))];
    } else if (k < 7) {
      // (round 6: groups with assertions at their alternatives' ends, which
      // the compiler distributes over the alternative)
      switch (rnd(4)) {
        case 0: s += "(^|" + gen(depth - 1) + ")"; break;
        case 1: s += "(" + gen(depth - 1) + "|$)"; break;
        case 2: s += "(\\b" + gen(depth - 1) + "|" + gen(depth - 1) + ")"; break;
        default: s += "(" + gen(depth - 1) + ")";
      }
    } else if (k < 8) {
      s += "(" + gen(depth - 1) + "|" + gen(depth - 1) + ")";
    } else if (k < 9) {
      // (round 6: lookahead groups too)
      s += (rnd(3) == 0 ? "(?=" : "(?:") + gen(depth - 1) + ")";
    } else {
      s += gen(depth - 1) + "|" + gen(depth - 1);
    }
    switch (rnd(9)) {
      case 0: s += "*"; break;
      case 1: s += "+"; break;
      case 2: s += "?"; break;
      case 3: s += "{" + std::to_string(rnd(3)) + "," + std::to_string(2 + rnd(2)) + "}"; break;
      case 4: s += "{" + std::to_string(1 + rnd(2)) + "}"; break;
      default: break;
    }
  }
  if (rnd(25) == 0) s = "(?^" + s + ")|" + gen(0);
  return s;
}

std::string mutate(std::string s)
{
  switch (rnd(6)) {
    case 0: if (!s.empty()) s.resize(rnd((uint32_t)s.size())); break;
    case 1: s.insert(s.begin() + rnd((uint32_t)s.size() + 1), (char)rnd(256)); break;
    case 2: s += "[" ; break;
    case 3: s += "("; break;
    case 4: s = ")" + s; break;
    default:
      for (auto& c : s)
        if (rnd(8) == 0) c = (char)rnd(256);
  }
  return s;
}

int calls = 0, compiled = 0, planned = 0, unsupported = 0;

void check(int rc, const char* what, const std::string& rx)
{
  ++calls;
  if (rc != UGPU_OK && rc != UGPU_UNSUPPORTED && rc != UGPU_INVAL) {
    std::fprintf(stderr, "%s: unexpected status %d for /%s/\n", what, rc, rx.c_str());
    std::abort();
  }
  if (rc != UGPU_OK && !ugpu_last_error()) {
    std::fprintf(stderr, "%s: no error string\n", what);
    std::abort();
  }
}

void exercise(const std::string& rx, uint32_t flags, const uint32_t* prev, uint32_t nprev)
{
  uint32_t* opc = nullptr;
  uint32_t nop = 0;
  const int rc = ugpu_compile(rx.data(), rx.size(), flags, &opc, &nop);
  if (rc != UGPU_OK) {
    if (rc != UGPU_INVAL && rc != UGPU_UNSUPPORTED) {
      std::fprintf(stderr, "ugpu_compile: status %d for /%s/\n", rc, rx.c_str());
      std::abort();
    }
    if (!ugpu_compile_error()) std::abort();
    if (rc == UGPU_UNSUPPORTED) ++unsupported;
    return;
  }
  ++compiled;
  for (uint32_t pf : {0u, (uint32_t)UGPU_PAT_WORD, (uint32_t)UGPU_PAT_EMPTY}) {
    ugpu_dfa_info info;
    const int r = ugpu_dfa_plan_host(opc, nop, pf, &info);
    check(r, "plan", rx);
    if (r == UGPU_OK) ++planned;
  }
  ugpu_dfa_info info;
  int r = ugpu_tables_build_host(opc, nop, &info, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr);
  check(r, "tables", rx);
  if (r == UGPU_OK) {
    std::vector<uint16_t> trans((size_t)info.states * info.row);
    std::vector<uint8_t> cls(256);
    std::vector<uint32_t> caps(info.states);
    uint32_t start = 0, accb = 0;
    if (info.format != 2) {
      check(ugpu_tables_build_host(opc, nop, &info, trans.data(), (uint32_t)trans.size(), cls.data(), caps.data(),
                                   (uint32_t)caps.size(), &start, &accb),
            "tables2", rx);
      // a too-small buffer must be refused, not written past
      if (trans.size() > 1) {
        const int r2 = ugpu_tables_build_host(opc, nop, &info, trans.data(), (uint32_t)trans.size() - 1, cls.data(),
                                              caps.data(), (uint32_t)caps.size(), &start, &accb);
        if (r2 == UGPU_OK) {
          std::fprintf(stderr, "tables: short buffer accepted for /%s/\n", rx.c_str());
          std::abort();
        }
      }
    }
    std::vector<uint32_t> acap((size_t)info.states * 64);
    int an = 0, sa = 0;
    check(ugpu_tables_context_host(opc, nop, acap.data(), (uint32_t)acap.size(), &an, &sa), "context", rx);
    uint8_t ft[20];
    int en = 0;
    check(ugpu_tables_prefilter_host(opc, nop, ft, &en), "prefilter", rx);
    int ok = 0;
    if (info.format != 2) {
      std::vector<uint16_t> xt(trans.size());
      check(ugpu_tables_transducer_host(opc, nop, xt.data(), (uint32_t)xt.size(), &ok), "transducer", rx);
      uint8_t sync[256];
      check(ugpu_tables_gap_host(opc, nop, xt.data(), (uint32_t)xt.size(), sync, &ok), "gap", rx);
      uint32_t rows = 0;
      uint8_t sb = 0;
      check(ugpu_tables_immediate_host(opc, nop, nullptr, 0, &rows, &sb, &ok), "immediate", rx);
      std::vector<uint8_t> xid((size_t)rows * 256 + 1);
      check(ugpu_tables_immediate_host(opc, nop, xid.data(), (uint32_t)xid.size(), &rows, &sb, &ok), "immediate2",
            rx);
    }
    uint8_t xc[256];
    check(ugpu_tables_xc_host(opc, nop, xc, &ok), "xc", rx);
    std::vector<uint8_t> xu(256 + 64 * 256 + 256);
    std::vector<uint32_t> bm3(2048);
    check(ugpu_tables_xu_host(opc, nop, xu.data(), bm3.data(), &ok), "xu", rx);
    uint32_t nd = 0;
    int all = 0;
    check(ugpu_tables_dom_host(opc, nop, nullptr, 0, &nd, &all), "dom", rx);
    std::vector<uint32_t> dom(nd + 1);
    check(ugpu_tables_dom_host(opc, nop, dom.data(), (uint32_t)dom.size(), &nd, nullptr), "dom2", rx);
    if (prev) {
      int eq = 0;
      check(ugpu_tables_equivalent_host(opc, nop, prev, nprev, &eq), "equivalent", rx);
    }
  } else {
    ++unsupported;
  }
  ugpu_opc_free(opc);
}

}  // namespace

int main(int argc, char** argv)
{
  const int n = argc > 1 ? std::atoi(argv[1]) : 10000;
  rng.seed(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 6);
  uint32_t* prev = nullptr;
  uint32_t nprev = 0;
  ugpu_compile("[a-z]+", 6, 0, &prev, &nprev);
  for (int i = 0; i < n; ++i) {
    std::string rx = gen(2);
    if (rnd(4) == 0) rx = mutate(rx);
    const uint32_t fl = rnd(3) == 0 ? (uint32_t)UGPU_RX_ICASE : 0u;
    const uint32_t flags = fl | (rnd(8) == 0 ? (uint32_t)UGPU_RX_FIXED : 0u) | (rnd(6) == 0 ? (uint32_t)UGPU_RX_REFLEX : 0u);
    if (std::getenv("FUZZ_VERBOSE")) std::fprintf(stderr, "%d /%s/ %u\n", i, rx.c_str(), flags);
    exercise(rx, flags, prev, nprev);
    if (i % 2000 == 0) std::fprintf(stderr, "fuzz_host: %d patterns\n", i);
  }
  // malformed opcode words straight into the table builders
  for (int i = 0; i < 2000; ++i) {
    std::vector<uint32_t> w(1 + rnd(40));
    for (auto& x : w) x = rnd(4) == 0 ? 0x00ffffffu : (uint32_t)rng();
    ugpu_dfa_info info;
    const int r = ugpu_dfa_plan_host(w.data(), (uint32_t)w.size(), 0, &info);
    check(r, "plan(random words)", "<words>");
    uint8_t ft[20];
    int en = 0;
    check(ugpu_tables_prefilter_host(w.data(), (uint32_t)w.size(), ft, &en), "prefilter(random words)", "<words>");
  }
  ugpu_opc_free(prev);
  std::printf("fuzz_host: %d patterns, %d compiled, %d planned, %d unsupported, %d checked calls\n", n, compiled,
              planned, unsupported, calls);
  return 0;
}
