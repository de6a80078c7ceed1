// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE, in-container only.
//
// Drives the REFERENCE RE/flex matcher (compiled from /root/reference/lib by
// oracle/Makefile into oracle/_ref/) the way ugrep does, to pin the oracle
// restatement and to generate golden fixtures.  Nothing here is product code.
//
//   pattern build  : "(?m)" + regex, reflex::Matcher::convert(.., notnewline|unicode),
//                    Pattern(conv, "r")          -- src/ugrep.cpp:8574-8604, :8849
//   -F quoting     : \Q...\E with \E escaped     -- src/cnf.hpp:147-165
//   search loop    : m.buffer(buf, n+1); while (m.find()) ...   -- src/ugrep.cpp:3939, :10544
//
// Usage:
//   ref_harness dump  re|F PATTERN
//   ref_harness find  re|F PATTERN INPUT [list]
//   ref_harness bench re|F PATTERN INPUT THREADS REPS
// INPUT = file:PATH[:TOTAL_BYTES]  (file tiled/truncated to TOTAL_BYTES)
//       | gen:KIND:SEED:OFF:LEN    (oracle/gen.h corpus slice)
//       | hex:HEXBYTES

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include <thread>
#include <chrono>
#include <algorithm>
#include <map>
#include <set>
#include <bitset>
#include <list>
#include <iostream>
#include <sstream>
#include <fstream>
#include <cstring>
#include <cstddef>
#include <utility>

// Introspection of Pattern's private tables (probe-only).
#define private public
#define protected public
#include <reflex/matcher.h>
#include <reflex/simd.h>
#undef private
#undef protected

#include "gen.h"

static std::string build_regex(const std::string& mode, const std::string& rx)
{
  // modes: re / F (Unicode, ugrep default) and reU / FU (-U: ASCII/binary, no unicode flag)
  bool ascii = mode == "reU" || mode == "FU";
  std::string regex = rx;
  if (mode == "F" || mode == "FU")
  {
    // CNF::quote (src/cnf.hpp:147-165)
    if (!regex.empty())
    {
      size_t from = 0, to;
      while ((to = regex.find("\\E", from)) != std::string::npos)
      {
        regex.insert(to + 2, "\\\\E\\Q");
        from = to + 7;
      }
      regex.insert(0, "\\Q").append("\\E");
    }
  }
  regex.insert(0, "(?m)");
  reflex::convert_flag_type flags = reflex::convert_flag::notnewline;
  if (!ascii)
    flags |= reflex::convert_flag::unicode;
  return reflex::Matcher::convert(regex, flags);
}

static std::vector<char> load_input(const std::string& spec)
{
  std::vector<char> buf;
  if (spec.compare(0, 5, "file:") == 0)
  {
    std::string rest = spec.substr(5);
    size_t total = 0;
    size_t c = rest.rfind(':');
    if (c != std::string::npos && c > 0 && rest.find_first_not_of("0123456789", c + 1) == std::string::npos)
    {
      total = strtoull(rest.c_str() + c + 1, NULL, 10);
      rest = rest.substr(0, c);
    }
    std::ifstream f(rest.c_str(), std::ios::binary);
    std::vector<char> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (total == 0)
      total = data.size();
    buf.resize(total);
    for (size_t i = 0; i < total; ++i)
      buf[i] = data[i % data.size()];
  }
  else if (spec.compare(0, 4, "gen:") == 0)
  {
    int kind; unsigned long long seed, off, len;
    if (sscanf(spec.c_str() + 4, "%d:%llu:%llu:%llu", &kind, &seed, &off, &len) != 4)
    {
      fprintf(stderr, "bad gen spec\n");
      exit(2);
    }
    buf.resize(len);
    gen_fill(kind, seed, off, reinterpret_cast<uint8_t*>(buf.data()), len);
  }
  else if (spec.compare(0, 4, "hex:") == 0)
  {
    std::string h = spec.substr(4);
    for (size_t i = 0; i + 1 < h.size(); i += 2)
      buf.push_back(static_cast<char>(strtoul(h.substr(i, 2).c_str(), NULL, 16)));
  }
  else
  {
    fprintf(stderr, "bad input spec\n");
    exit(2);
  }
  buf.push_back('\0'); // ugrep passes size+1 (src/ugrep.cpp:3939)
  return buf;
}

struct Tally
{
  uint64_t count = 0, digest = 0, dcap = 0;
};

// matcher options (mode suffixes "W" = ugrep -w: option W, src/ugrep.cpp:8616-8618; "N" = ugrep -Y / -x: option N, :8612-8613)
static std::string g_matcher_opt;
// mode suffix "P": the same Matcher with its match predictor switched off.
// FIND normally jumps between candidate positions the Pattern's predictor
// (bitap/hash tables, lib/pattern.cpp:4342-4430, lib/matcher.cpp:797-950)
// accepts; with "P" every position is a candidate, which leaves the DFA's own
// semantics (lib/matcher.cpp:125-546).  The two differ where the predictor
// rejects a position at which the DFA matches through a meta edge (e.g.
// "a$|ab" before "\n" followed by more text, or "^\w+" without option N):
// tests/golden/make_anchor_golden.py records both.
static bool g_no_predict = false;

struct Unpredicted : public reflex::Matcher {
  Unpredicted(const reflex::Pattern& pat, const char *opt) : reflex::Matcher(pat, reflex::Input(), opt) { }
  bool advance_each(size_t loc)
  {
    if (loc >= end_)
    {
      set_current(end_);
      return false;
    }
    set_current(loc);
    return true;
  }
  void unpredict()
  {
    adv_ = static_cast<bool (reflex::Matcher::*)(size_t)>(&Unpredicted::advance_each);
  }
};

static Tally scan(const reflex::Pattern& pat, char *base, size_t n, size_t bias, std::vector<uint64_t> *list)
{
  Tally t;
  Unpredicted m(pat, g_matcher_opt.empty() ? NULL : g_matcher_opt.c_str());
  m.buffer(base, n + 1);
  if (g_no_predict)
  {
    if (pat.one_)
    {
      fprintf(stderr, "mode P: single-string pattern, nothing to switch off\n");
      exit(2);
    }
    m.unpredict();
  }
  while (size_t cap = m.find())
  {
    uint64_t st = m.first() + bias;
    uint64_t ln = m.size();
    ++t.count;
    t.digest += st * 31 + ln;
    t.dcap += (st + 1) * cap;
    if (list)
    {
      list->push_back(st);
      list->push_back(ln);
      list->push_back(cap);
    }
  }
  return t;
}

int main(int argc, char **argv)
{
  if (argc < 4 && !(argc == 2 && std::string(argv[1]) == "isutf8"))
  {
    fprintf(stderr, "usage: ref_harness dump|find|bench re|F PATTERN ... | isutf8 < specs\n");
    return 2;
  }
  if (std::string(argv[1]) == "isutf8")
  {
    // reflex::isutf8 (lib/simd.cpp:169) on each input spec read from stdin,
    // one per line; prints 1/0 per line (tests/golden/make_utf8_golden.py)
    char line[1 << 16];
    while (fgets(line, sizeof(line), stdin))
    {
      std::string spec(line);
      while (!spec.empty() && (spec.back() == '\n' || spec.back() == '\r'))
        spec.pop_back();
      std::vector<char> b = load_input(spec.c_str());
      size_t n = b.size() - 1;
      printf("%d\n", reflex::isutf8(b.data(), b.data() + n) ? 1 : 0);
    }
    return 0;
  }
  std::string cmd = argv[1], mode = argv[2], rx = argv[3];
  // mode suffixes: W = Matcher option W (ugrep -w), N = option N (ugrep -Y, and -x)
  // P = predictor off (see Unpredicted above)
  while (mode.size() > 1 && (mode[mode.size() - 1] == 'W' || mode[mode.size() - 1] == 'N' || mode[mode.size() - 1] == 'P'))
  {
    if (mode[mode.size() - 1] == 'P')
      g_no_predict = true;
    else
      g_matcher_opt.push_back(mode[mode.size() - 1]);
    mode.erase(mode.size() - 1);
  }
  std::string conv = build_regex(mode, rx);
  reflex::Pattern pat(conv, "r");
  if (cmd == "dump")
  {
    printf("{\"regex\": %zu, \"nop\": %u, \"len\": %u, \"min\": %u, \"one\": %d, \"lbk\": %u, \"pin\": %u, \"npy\": %u, \"opc\": [",
        conv.size(), (unsigned)pat.nop_, (unsigned)pat.len_, (unsigned)pat.min_, (int)pat.one_, (unsigned)pat.lbk_,
        (unsigned)pat.pin_, (unsigned)pat.npy_);
    for (size_t i = 0; i < pat.nop_; ++i)
      printf("%s%u", i ? ", " : "", (unsigned)pat.opc_[i]);
    // the regex the Pattern holds, through its public accessor (Pattern::operator[](0),
    // include/reflex/pattern.h:302): what the drop-in adapter compiles (UGPU_RX_REFLEX)
    const std::string whole = pat[0];
    printf("], \"conv_hex\": \"");
    for (size_t i = 0; i < whole.size(); ++i)
      printf("%02x", (unsigned)(unsigned char)whole[i]);
    printf("\"}\n");
    return 0;
  }
  if (argc < 5)
    return 2;
  std::vector<char> buf = load_input(argv[4]);
  size_t n = buf.size() - 1;
  if (cmd == "find")
  {
    bool want = argc > 5 && std::string(argv[5]) == "list";
    std::vector<uint64_t> list;
    Tally t = scan(pat, buf.data(), n, 0, want ? &list : NULL);
    printf("%llu %llu %llu\n", (unsigned long long)t.count, (unsigned long long)t.digest, (unsigned long long)t.dcap);
    for (size_t i = 0; i < list.size(); i += 3)
      printf("%llu %llu %llu\n", (unsigned long long)list[i], (unsigned long long)list[i + 1], (unsigned long long)list[i + 2]);
    return 0;
  }
  if (cmd == "bench")
  {
    int threads = argc > 5 ? atoi(argv[5]) : 1;
    int reps = argc > 6 ? atoi(argv[6]) : 3;
    // newline-split shards, one Matcher per thread sharing the Pattern (src/ugrep.cpp:4206)
    std::vector<size_t> cut(threads + 1, 0);
    cut[threads] = n;
    for (int i = 1; i < threads; ++i)
    {
      size_t c = std::max(cut[i - 1], n / threads * i);
      while (c < n && buf[c - 1] != '\n')
        ++c;
      cut[i] = c;
    }
    double best = 1e30;
    Tally tot;
    for (int r = 0; r < reps; ++r)
    {
      std::vector<Tally> part(threads);
      std::vector<std::vector<char> > copies(threads);
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int i = 0; i < threads; ++i)
        th.emplace_back([&, i]() {
          // each shard is scanned in place; the byte after the shard is
          // temporarily NUL-terminated in a private copy only at the cut
          size_t a = cut[i], b = cut[i + 1];
          part[i] = scan(pat, buf.data() + a, b - a, a, NULL);
        });
      for (auto& x : th)
        x.join();
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      best = std::min(best, s);
      tot = Tally();
      for (auto& p : part)
      {
        tot.count += p.count;
        tot.digest += p.digest;
        tot.dcap += p.dcap;
      }
    }
    printf("{\"bytes\": %zu, \"seconds\": %.6f, \"threads\": %d, \"count\": %llu, \"digest\": %llu, "
           "\"dcap\": %llu}\n",
        n, best, threads, (unsigned long long)tot.count, (unsigned long long)tot.digest,
        (unsigned long long)tot.dcap);
    return 0;
  }
  return 2;
}
