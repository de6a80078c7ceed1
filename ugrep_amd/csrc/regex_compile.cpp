// regex_compile.cpp -- host-side regex -> DFA -> opcode-word compiler.
//
// Replaces, for the FIND hot path, the reference's pattern pipeline
//   Matcher::convert(rx, notnewline|unicode)   (lib/convert.cpp, src/ugrep.cpp:8574-8578)
//   Pattern(conv, "r") -> parse/compile/encode_dfa  (lib/pattern.cpp:171-3063)
// with a from-scratch construction:
//   parse (ugrep's default ERE syntax, Unicode mode)  -> byte-level syntax tree
//   Unicode code point sets -> valid UTF-8 byte-range sequences (strict, like
//     lib/utf8.cpp utf8(a, b, .., strict=true) as called by convert.cpp:124-171)
//   Glushkov positions + subset construction -> DFA over bytes
//   Moore minimisation -> opcode words in the reference's format
//     (include/reflex/pattern.h:1155-1247; Appendix B of SURVEY.md in reverse),
// so ugpu_dfa_create() consumes the result exactly like a table dumped from a
// reference Pattern.  Parity is language equivalence with the reference's DFA
// per accept index (tests/test_compile.py), which implies identical FIND
// results on every input.
//
// Supported: literals (UTF-8), escapes \t\n\r\f\v\a\e \xHH \x{H..} \0ooo and
// escaped punctuation, '.', bracket expressions (ranges, negation, escapes,
// \w\d\s\h and \p{..} inside, POSIX [:name:]), \w \W \d \D \s \S \h \H,
// \p{NAME} \P{NAME} \pL (general categories and their long names, common
// scripts, POSIX-style names), groups ( ) (?: ), alternation,
// * + ? {n} {n,} {n,m}, -F literal mode, and -i (ASCII plus case_fold.inc pairs).
// Line anchors: a ^ that starts a top-level alternative and a $ that ends one
// (ugrep's -x wrapper ^(?:P)$, src/cnf.hpp:167-185, and ^P / P$ / ^a|b$),
// under (?m) (ugrep's pattern prefix, src/ugrep.cpp:8586) or in the ERE mode;
// they become per-context accepts encoded as META_BOL / META_EOL edges to
// accept-only states (include/reflex/pattern.h:942-943), the shape the
// reference's Pattern gives them (^ moved to the accept side).
// Word boundaries \b \B \< \> before the first atom of a top-level
// alternative (the begin-of-match forms META_WBB/NWB/BWB/EWB, which RE/flex
// also tests on the accept side, lib/pattern.cpp:2527-2538 k->anchor()) or
// after its last (META_WBE/NWE/BWE/EWE): per-context accepts over 64 contexts
// (ctx_bits.hpp), encoded as exhaustive meta-edge splits (encode()).
// Negative patterns (?^...) as whole top-level alternatives (ugrep -N,
// src/ugrep.cpp:6487): their accepts become REDO words.
// Lookahead X(?=Y) (round 6): HEAD/TAIL markers as the reference places them
// (Parser::lookahead_group), emitted as TAIL la / HEAD la words.
// Returns UGPU_UNSUPPORTED for what the GPU tables cannot express or this
// compiler does not cover (other anchors, word boundaries, lazy quantifiers,
// negative lookahead, nested or adjacent lookaheads, backreferences, other \p
// names, \p{Lu} under -i): the caller keeps
// the CPU matcher for those, as for any unsupported opcode table.
#include <stdint.h>
#include <stdlib.h>
#include <ctype.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <bitset>
#include <map>
#include <string>
#include <vector>

#include "ugpu.h"
#include "ctx_bits.hpp"

using ugpu::CTX_BOL;
using ugpu::CTX_BW;
using ugpu::CTX_EOL;
using ugpu::CTX_EW;
using ugpu::CTX_WB;
using ugpu::CTX_WE;

namespace {

#include "unicode_ranges.inc"
#include "case_fold.inc"

typedef std::vector<std::pair<uint32_t, uint32_t>> CpSet;  // sorted, disjoint, inclusive
typedef std::bitset<256> ByteSet;

const uint32_t kMaxCp = 0x10FFFF;
// the accept of a state that holds a negative pattern's end (encoded as a
// REDO word; the reference emits REDO for such a state whatever else it
// accepts, lib/pattern.cpp:2358-2363, :2945-2947)
const uint32_t kRedoAcc = 0xFFFFFFu;
const size_t kMaxPositions = 1u << 16;  // expansion guard ({n,m} of large subtrees)
const size_t kMaxStates = 1u << 16;

struct CompileError
{
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string &msg)
{
  throw CompileError{code, msg};
}

// ---------------------------------------------------------------- code point sets

CpSet normalize(CpSet s)
{
  std::sort(s.begin(), s.end());
  CpSet out;
  for (auto &r : s)
  {
    if (!out.empty() && r.first <= out.back().second + 1)
      out.back().second = std::max(out.back().second, r.second);
    else
      out.push_back(r);
  }
  return out;
}

// complement over [0, hi], surrogates included
CpSet complement_upto(const CpSet &s, uint32_t hi)
{
  CpSet out;
  uint32_t next = 0;
  for (auto &r : s)
  {
    if (r.first > hi)
      break;
    if (r.first > next)
      out.push_back({next, r.first - 1});
    next = r.second + 1;
  }
  if (next <= hi)
    out.push_back({next, hi});
  return out;
}

CpSet no_surrogates(const CpSet &s);

// complement over the Unicode scalar values (surrogates never match, as
// convert.cpp:124-162 skips D800-DFFF)
CpSet complement(const CpSet &s)
{
  return no_surrogates(complement_upto(s, kMaxCp));
}

CpSet minus(const CpSet &a, const CpSet &b)
{
  CpSet out;
  for (auto r : a)
  {
    uint32_t lo = r.first;
    for (auto &x : b)
    {
      if (x.second < lo || x.first > r.second)
        continue;
      if (x.first > lo)
        out.push_back({lo, x.first - 1});
      lo = x.second + 1;
      if (lo > r.second || x.second == kMaxCp)
        break;
    }
    if (lo <= r.second && lo != 0x110000)
      out.push_back({lo, r.second});
  }
  return out;
}

CpSet no_surrogates(const CpSet &s)
{
  return minus(s, CpSet{{0xD800, 0xDFFF}});
}

template <size_t N>
CpSet table_set(const uint32_t (&t)[N][2])
{
  CpSet s;
  for (size_t i = 0; i < N; ++i)
    s.push_back({t[i][0], t[i][1]});
  return s;
}

// \p{NAME} / [[:name:]] tables (unicode_ranges.inc registry); false if unknown
bool named_set(const std::string &name, CpSet &out, bool *pnl = NULL)
{
  for (const UClass &c : k_pclasses)
    if (name == c.name)
    {
      if (pnl)
        *pnl = c.pnl != 0;
      out.clear();
      for (unsigned i = 0; i < c.n; ++i)
        out.push_back({c.ranges[i][0], c.ranges[i][1]});
      return true;
    }
  return false;
}

CpSet word_set() { return table_set(k_word_ranges); }
CpSet digit_set() { return table_set(k_digit_ranges); }
CpSet space_set() { return table_set(k_space_ranges); }
CpSet hspace_set() { return CpSet{{'\t', '\t'}, {' ', ' '}}; }

// the other case of c >= 0x80 under (?i), or 0 (case_fold.inc)
uint32_t case_variant(uint32_t c)
{
  size_t lo = 0, hi = sizeof(k_case_sets) / sizeof(k_case_sets[0]);
  while (lo < hi)
  {
    size_t mid = (lo + hi) / 2;
    if (k_case_sets[mid][0] < c)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < sizeof(k_case_sets) / sizeof(k_case_sets[0]) && k_case_sets[lo][0] == c ? k_case_sets[lo][2] : 0;
}

// add the (?i) variants of every member >= 0x80 (rows of case_fold.inc)
void add_unicode_case(CpSet &s)
{
  CpSet extra;
  for (auto &row : k_case_sets)
  {
    uint32_t c = row[0];
    auto it = std::upper_bound(s.begin(), s.end(), std::make_pair(c, 0xFFFFFFFFu));
    if (it != s.begin() && (it - 1)->first <= c && c <= (it - 1)->second)
      extra.push_back({row[2], row[2]});
  }
  s.insert(s.end(), extra.begin(), extra.end());
  s = normalize(s);
}

void add_ascii_case(CpSet &s)
{
  CpSet extra;
  for (auto &r : s)
    for (uint32_t c = r.first; c <= r.second && c < 0x80; ++c)
    {
      if (c >= 'a' && c <= 'z')
        extra.push_back({c - 32, c - 32});
      else if (c >= 'A' && c <= 'Z')
        extra.push_back({c + 32, c + 32});
    }
  s.insert(s.end(), extra.begin(), extra.end());
  s = normalize(s);
}

// ---------------------------------------------------------------- syntax tree

enum Kind
{
  LEAF,  // one byte from `bytes`
  CAT,
  ALT,
  STAR,
  PLUS,
  OPT,
  EMPTY,
  LOOK  // X(?=Y): kids[0] = Y (Node::look, Node::look_alt)
};

struct Node
{
  Kind kind;
  ByteSet bytes;
  std::vector<int> kids;
  int look = -1;     // LOOK: the lookahead index (TAIL/HEAD la)
  int look_alt = 0;  // LOOK: its top-level alternative (accept index)
};

struct Tree
{
  std::vector<Node> nodes;
  size_t leaves = 0;

  int add(Kind k, std::vector<int> kids = {})
  {
    nodes.push_back(Node{k, ByteSet(), std::move(kids), -1, 0});
    return static_cast<int>(nodes.size() - 1);
  }
  int leaf(const ByteSet &b)
  {
    if (++leaves > kMaxPositions)
      fail(UGPU_UNSUPPORTED, "pattern expands to too many positions");
    int n = add(LEAF);
    nodes[n].bytes = b;
    return n;
  }
  int leaf_range(unsigned lo, unsigned hi)
  {
    ByteSet b;
    for (unsigned c = lo; c <= hi; ++c)
      b.set(c);
    return leaf(b);
  }
  int clone(int n)
  {
    Node copy = nodes[n];
    if (copy.kind == LEAF)
      return leaf(copy.bytes);
    std::vector<int> kids;
    for (int k : copy.kids)
      kids.push_back(clone(k));
    const int n2 = add(copy.kind, kids);
    nodes[n2].look = copy.look;  // (a repeated lookahead keeps its index, as the
    nodes[n2].look_alt = copy.look_alt;  // reference's iterated positions keep their location)
    return n2;
  }

  // UTF-8 byte-range sequences of [lo, hi] (same encoded length, split so that
  // each sequence is a product of byte ranges)
  void utf8_split(uint32_t lo, uint32_t hi, std::vector<std::vector<std::pair<uint8_t, uint8_t>>> &out)
  {
    static const uint32_t len_max[3] = {0x7F, 0x7FF, 0xFFFF};
    for (uint32_t m : len_max)
      if (lo <= m && hi > m)
      {
        utf8_split(lo, m, out);
        utf8_split(m + 1, hi, out);
        return;
      }
    if (hi <= 0x7F)
    {
      out.push_back({{static_cast<uint8_t>(lo), static_cast<uint8_t>(hi)}});
      return;
    }
    for (int i = 1; i < 4; ++i)
    {
      uint32_t m = (1u << (6 * i)) - 1;
      if ((lo & ~m) != (hi & ~m))
      {
        if ((lo & m) != 0)
        {
          utf8_split(lo, lo | m, out);
          utf8_split((lo | m) + 1, hi, out);
          return;
        }
        if ((hi & m) != m)
        {
          utf8_split(lo, (hi & ~m) - 1, out);
          utf8_split(hi & ~m, hi, out);
          return;
        }
      }
    }
    uint8_t a[4], b[4];
    int n = encode(lo, a);
    encode(hi, b);
    std::vector<std::pair<uint8_t, uint8_t>> seq;
    for (int i = 0; i < n; ++i)
      seq.push_back({a[i], b[i]});
    out.push_back(seq);
  }

  static int encode(uint32_t c, uint8_t *o)
  {
    if (c < 0x80)
    {
      o[0] = static_cast<uint8_t>(c);
      return 1;
    }
    if (c < 0x800)
    {
      o[0] = static_cast<uint8_t>(0xC0 | (c >> 6));
      o[1] = static_cast<uint8_t>(0x80 | (c & 0x3F));
      return 2;
    }
    if (c < 0x10000)
    {
      o[0] = static_cast<uint8_t>(0xE0 | (c >> 12));
      o[1] = static_cast<uint8_t>(0x80 | ((c >> 6) & 0x3F));
      o[2] = static_cast<uint8_t>(0x80 | (c & 0x3F));
      return 3;
    }
    o[0] = static_cast<uint8_t>(0xF0 | (c >> 18));
    o[1] = static_cast<uint8_t>(0x80 | ((c >> 12) & 0x3F));
    o[2] = static_cast<uint8_t>(0x80 | ((c >> 6) & 0x3F));
    o[3] = static_cast<uint8_t>(0x80 | (c & 0x3F));
    return 4;
  }

  // the byte ranges of s when its valid UTF-8 encodings are one product of
  // byte ranges (one code point length, no alternation), else empty
  std::vector<std::pair<uint8_t, uint8_t>> single_product(const CpSet &s0)
  {
    CpSet s = normalize(s0);
    std::vector<std::vector<std::pair<uint8_t, uint8_t>>> seqs;
    for (auto &r : s)
    {
      if (r.first < 0x80)
        return {};
      utf8_split(r.first, r.second, seqs);
      if (seqs.size() > 1)
        return {};
    }
    return seqs.size() == 1 ? seqs[0] : std::vector<std::pair<uint8_t, uint8_t>>();
  }

  // subtree matching exactly the valid UTF-8 encodings of the code points in s
  int cpset(const CpSet &s0)
  {
    CpSet s = normalize(s0);
    ByteSet ascii;
    std::vector<std::vector<std::pair<uint8_t, uint8_t>>> seqs;
    for (auto &r : s)
    {
      if (r.first < 0x80)
        for (uint32_t c = r.first; c <= std::min<uint32_t>(r.second, 0x7F); ++c)
          ascii.set(c);
      if (r.second >= 0x80)
        utf8_split(std::max<uint32_t>(r.first, 0x80), r.second, seqs);
    }
    std::vector<int> alts;
    if (ascii.any())
      alts.push_back(leaf(ascii));
    // share leading byte ranges: group sequences by their first range
    std::map<std::pair<uint8_t, uint8_t>, std::vector<std::vector<std::pair<uint8_t, uint8_t>>>> groups;
    for (auto &q : seqs)
      groups[q[0]].push_back(std::vector<std::pair<uint8_t, uint8_t>>(q.begin() + 1, q.end()));
    for (auto &g : groups)
      alts.push_back(add(CAT, {leaf_range(g.first.first, g.first.second), suffixes(g.second)}));
    if (alts.empty())
      fail(UGPU_INVAL, "empty character class");
    return alts.size() == 1 ? alts[0] : add(ALT, alts);
  }

  int suffixes(std::vector<std::vector<std::pair<uint8_t, uint8_t>>> &tails)
  {
    std::map<std::pair<uint8_t, uint8_t>, std::vector<std::vector<std::pair<uint8_t, uint8_t>>>> groups;
    for (auto &q : tails)
      groups[q[0]].push_back(std::vector<std::pair<uint8_t, uint8_t>>(q.begin() + 1, q.end()));
    std::vector<int> alts;
    for (auto &g : groups)
    {
      int head = leaf_range(g.first.first, g.first.second);
      if (g.second[0].empty())
        alts.push_back(head);
      else
        alts.push_back(add(CAT, {head, suffixes(g.second)}));
    }
    return alts.size() == 1 ? alts[0] : add(ALT, alts);
  }
};

// ---------------------------------------------------------------- parser

class Parser
{
 public:
  Parser(const std::string &rx, uint32_t flags, Tree &t)
      : s_(rx), flags_(flags), t_(t), ic_((flags & UGPU_RX_ICASE) != 0)
  {
  }

  // top-level alternatives (each gets its own accept index, as the reference's
  // Pattern numbers top-level choices: SURVEY Appendix D, foo|bar|baz -> TAKE 1/2/3)
  std::vector<int> parse_top()
  {
    std::vector<int> alts;
    if (flags_ & UGPU_RX_FIXED)
    {
      std::vector<int> seq;
      for (size_t i = 0; i < s_.size(); ++i)
        seq.push_back(literal_byte(static_cast<uint8_t>(s_[i])));
      alts.push_back(seq.empty() ? t_.add(EMPTY) : t_.add(CAT, seq));
      return alts;
    }
    if (!s_.empty() && s_[0] == '|')
      fail(UGPU_INVAL, "empty first alternative");  // the reference rejects "|a" (but not "a|")
    for (;;)
    {
      eol_ = false;
      begin_.clear();
      end_.clear();
      neg_node_ = -1;
      alt_index_ = static_cast<int>(alts.size()) + 1;
      const int a = parse_concat(true);
      alts.push_back(a);
      // a negative pattern (?^...) (ugrep -N, src/ugrep.cpp:6487): the whole
      // alternative, besides modifiers -- its accept is REDO.  The reference
      // negates the positions that follow a negated one too
      // (lib/pattern.cpp:2421-2432), so (?^...) inside a sequence negates its
      // tail: not modelled, refused.
      bool neg = false;
      if (neg_node_ >= 0)
      {
        bool whole = a == neg_node_;
        if (!whole && t_.nodes[a].kind == CAT)
        {
          int others = 0;
          for (int k : t_.nodes[a].kids)
            others += k != neg_node_ && t_.nodes[k].kind != EMPTY;
          whole = others == 0;
        }
        if (!whole)
          fail(UGPU_UNSUPPORTED, "(?^...) inside a sequence");
        neg = true;
      }
      negs.push_back(neg);
      // the alternative's meta edges in the order RE/flex chains them after
      // its last byte: the end assertions as written, then the begin ones
      // (^ \< ... moved to the accept side), e.g. ^\<ab\>$ -> EWE EOL BOL BWB
      std::vector<uint8_t> seq(end_);
      seq.insert(seq.end(), begin_.begin(), begin_.end());
      metaseqs.push_back(seq);
      if (p_ >= s_.size() || s_[p_] != '|')
        break;
      ++p_;
    }
    if (p_ != s_.size())
      fail(UGPU_INVAL, "unbalanced ')'");
    bool any_neg = false, any_meta = false;
    for (size_t k = 0; k < negs.size(); ++k)
    {
      any_neg = any_neg || negs[k];
      any_meta = any_meta || !metaseqs[k].empty();
    }
    if (any_neg && any_meta)
      fail(UGPU_UNSUPPORTED, "(?^...) with anchors or word boundaries");
    if (look_count_ && (any_neg || any_meta))
      fail(UGPU_UNSUPPORTED, "lookahead with anchors, word boundaries or (?^...)");
    return alts;
  }

  // lookaheads (?=...) in the pattern (indices 0 .. looks - 1)
  int looks() const { return look_count_; }

  // per top-level alternative: a negative pattern (?^...), whose accept is REDO
  std::vector<bool> negs;

  // per top-level alternative: the meta edges (META - META_MIN) its accept
  // passes through, in chain order
  std::vector<std::vector<uint8_t>> metaseqs;

 private:
  const std::string &s_;
  uint32_t flags_;
  Tree &t_;
  size_t p_ = 0;
  bool ic_;             // case-insensitive (flag, or RE/flex (?i) in REFLEX mode)
  bool dotall_ = false;  // REFLEX mode (?s): '.' matches '\n'
  bool multiline_ = false;  // REFLEX mode (?m): ^ and $ are line anchors
  bool eol_ = false;  // the top-level alternative being parsed ended with $
  int depth_ = 0;      // group nesting
  int neg_node_ = -1;  // the (?^...) group of the top-level alternative being parsed
  std::vector<uint8_t> begin_, end_;  // its begin / end assertions (META - META_MIN), as written
  int alt_index_ = 1;              // the top-level alternative being parsed (its accept index)
  // a \p{NAME} atom whose quantifier binds to its last byte-level atom only
  // (parse_atom sets them, parse_repeat consumes them; see there)
  bool p_quirk_ = false;
  std::vector<int> p_prefix_;
  int p_tail_ = -1;
  int look_count_ = 0;             // lookaheads so far
  bool in_look_ = false;           // parsing inside (?=...)
  size_t look_end_ = std::string::npos;  // the ')' of the last lookahead

  // "(?=" at p_ - 1 .. p_ + 1: X(?=Y) as the reference's Pattern compiles it
  // (lib/pattern.cpp:1331-1359): a HEAD marker in Y's first positions (the
  // states where Y starts record the position, HEAD la), a TAIL marker after
  // Y's last positions (the accepting states where Y completes move the match
  // end back to it, TAIL la, when their accept is this alternative's:
  // :2395-2419).  Indices count the lookaheads per top-level alternative in
  // order of their location, the alternatives in order (:2378-2393) -- the
  // running count here.  The reference merges nested and adjacent lookahead
  // ranges into one index (ORanges, include/reflex/ranges.h:664-671): refused.
  int lookahead_group()
  {
    const size_t open = p_ - 1;
    if (in_look_)
      fail(UGPU_UNSUPPORTED, "nested lookahead");
    if (look_end_ != std::string::npos && open == look_end_ + 1)
      fail(UGPU_UNSUPPORTED, "adjacent lookaheads");
    if (look_count_ >= 16)
      fail(UGPU_UNSUPPORTED, "more than 16 lookaheads");
    p_ += 2;
    if (p_ >= s_.size() || s_[p_] == ')')
      fail(UGPU_UNSUPPORTED, "empty lookahead");
    const bool ic = ic_, dot = dotall_;
    in_look_ = true;
    ++depth_;
    const int a = parse_alt();
    --depth_;
    in_look_ = false;
    ic_ = ic;
    dotall_ = dot;
    if (p_ >= s_.size() || s_[p_] != ')')
      fail(UGPU_INVAL, "missing ')'");
    look_end_ = p_++;
    const int n = t_.add(LOOK, {a});
    t_.nodes[n].look = look_count_++;
    t_.nodes[n].look_alt = alt_index_;
    return n;
  }

  // a word-boundary assertion at p_ (\b \B \< \>): its class mask (for the
  // begin of the match, bits 0-2; as the reference's META_WBB/NWB/BWB/EWB and
  // META_WBE/NWE/BWE/EWE hold: include/reflex/matcher.h:1281-1319), or 0
  int word_assertion(size_t q) const
  {
    if (q + 1 >= s_.size() || s_[q] != '\\')
      return 0;
    switch (s_[q + 1])
    {
      case 'b': return 1 | 2;  // \b: A or B
      case 'B': return 4;      // \B: N
      case '<': return 1;      // \< : begin of a word
      case '>': return 2;      // \> : end of a word
      default: return 0;
    }
  }

  bool icase() const { return ic_; }
  bool reflex() const { return (flags_ & UGPU_RX_REFLEX) != 0; }

  int literal_byte(uint8_t c)
  {
    ByteSet b;
    b.set(c);
    if (icase() && ((c | 0x20) >= 'a' && (c | 0x20) <= 'z'))
      b.set(c ^ 0x20);
    return t_.leaf(b);
  }

  // "(?^" at p_ - 1 .. p_ + 1: a negative pattern, at the top level only
  int negative_group()
  {
    if (depth_ != 0 || neg_node_ >= 0)
      fail(UGPU_UNSUPPORTED, "(?^...) inside a group");
    p_ += 2;
    ++depth_;
    const bool ic = ic_, dot = dotall_;
    const int a = parse_alt();
    ic_ = ic;
    dotall_ = dot;
    --depth_;
    if (p_ >= s_.size() || s_[p_] != ')')
      fail(UGPU_INVAL, "missing ')'");
    ++p_;
    neg_node_ = a;
    return a;
  }

  int parse_alt()
  {
    // an empty alternative inside a group is a regex_error in the reference
    // (only top-level alternatives may be empty)
    auto branch = [&]() {
      if (p_ >= s_.size() || s_[p_] == '|' || s_[p_] == ')')
        fail(UGPU_INVAL, "empty alternative in group");
      return parse_concat();
    };
    std::vector<int> alts{branch()};
    while (p_ < s_.size() && s_[p_] == '|')
    {
      ++p_;
      alts.push_back(branch());
    }
    return alts.size() == 1 ? alts[0] : t_.add(ALT, alts);
  }

  int parse_concat(bool top = false)
  {
    std::vector<int> seq;
    bool atoms = false;
    while (p_ < s_.size() && s_[p_] != '|' && s_[p_] != ')')
    {
      // line anchors of a top-level alternative: ^ before its first atom, $
      // as its last character (anything else stays UNSUPPORTED in parse_atom)
      if (top && (s_[p_] == '^' || s_[p_] == '$') && (multiline_ || !reflex()))
      {
        const bool first = s_[p_] == '^' && !atoms;
        const bool last = s_[p_] == '$' && (p_ + 1 == s_.size() || s_[p_ + 1] == '|');
        if (first || last)
        {
          if (p_ + 1 < s_.size() && strchr("*+?{", s_[p_ + 1]) != NULL)
            fail(UGPU_UNSUPPORTED, "repeated anchor");
          if (first)
            begin_.push_back(0x09);  // META_BOL
          else
          {
            end_.push_back(0x0a);  // META_EOL
            eol_ = true;
          }
          ++p_;
          continue;
        }
      }
      // word boundaries of a top-level alternative: before its first atom, or
      // followed only by other assertions and $ up to the alternative's end
      if (top && word_assertion(p_))
      {
        size_t q = p_;
        while (q < s_.size())
        {
          if (word_assertion(q))
            q += 2;
          else if (s_[q] == '$' && (multiline_ || !reflex()))
            ++q;
          else
            break;
        }
        const bool last = q == s_.size() || s_[q] == '|';
        if (!atoms || last)
        {
          if (p_ + 2 < s_.size() && strchr("*+?{", s_[p_ + 2]) != NULL)
            fail(UGPU_UNSUPPORTED, "repeated word boundary");
          const int m = word_assertion(p_);
          // an assertion with atoms after it tests the match begin
          // (META_WBB NWB BWB EWB), one with none the end (META_WBE NWE BWE
          // EWE; also an alternative of assertions only: "\\b" compiles to
          // META_WBE)
          const uint8_t code = last ? (m == 3 ? 0x02 : m == 4 ? 0x04 : m == 1 ? 0x07 : 0x08)
                                    : (m == 3 ? 0x01 : m == 4 ? 0x03 : m == 1 ? 0x05 : 0x06);
          (last ? end_ : begin_).push_back(code);
          p_ += 2;
          continue;
        }
        fail(UGPU_UNSUPPORTED, "word boundary between consumed characters");
      }
      // REFLEX mode: a (?imsx) modifier after atoms of its branch opens a group
      // that runs to the end of the enclosing group, later alternatives
      // included ("x(?i)ab|cd" is x(?i:ab|cd)); a leading one just sets the
      // flags for the rest of the enclosing group (measured on the reference's
      // tables: "(?i)foo|BAR" keeps two case-insensitive alternatives)
      if (reflex() && atoms && modifier_at(p_))
      {
        seq.push_back(parse_atom_reflex());  // sets the flags
        seq.push_back(p_ >= s_.size() || s_[p_] == ')' ? t_.add(EMPTY) : parse_alt());
        break;
      }
      if (eol_)
        fail(UGPU_UNSUPPORTED, "anchor");  // (unreachable: $ ends the alternative)
      atoms = atoms || !(reflex() && modifier_at(p_));
      seq.push_back(parse_repeat());
    }
    if (seq.empty())
      return t_.add(EMPTY);
    return seq.size() == 1 ? seq[0] : t_.add(CAT, seq);
  }

  bool parse_braces(int &lo, int &hi)
  {
    // {n}, {n,}, {n,m} at p_ (p_ on '{'); returns false when not a quantifier
    size_t q = p_ + 1;
    auto num = [&](int &v) {
      size_t st = q;
      v = 0;
      while (q < s_.size() && s_[q] >= '0' && s_[q] <= '9')
      {
        v = v * 10 + (s_[q++] - '0');
        if (v > 1000)
          fail(UGPU_UNSUPPORTED, "repeat count too large");
      }
      return q > st;
    };
    if (!num(lo))
      return false;
    hi = lo;
    if (q < s_.size() && s_[q] == ',')
    {
      ++q;
      if (!num(hi))
        hi = -1;
    }
    if (q >= s_.size() || s_[q] != '}')
      return false;
    if (hi >= 0 && hi < lo)
      fail(UGPU_INVAL, "bad repeat range");
    p_ = q + 1;
    return true;
  }

  int repeat(int a, int lo, int hi)
  {
    std::vector<int> seq;
    for (int i = 0; i < lo; ++i)
      seq.push_back(i == 0 ? a : t_.clone(a));
    if (hi < 0)
      seq.push_back(t_.add(STAR, {lo == 0 ? a : t_.clone(a)}));
    else
    {
      // X{lo,hi}: X^lo (X (X ...)?)? nested optionals
      int tail = -1;
      for (int i = hi - lo; i > 0; --i)
      {
        int x = (lo == 0 && i == 1) ? a : t_.clone(a);
        tail = t_.add(OPT, {tail < 0 ? x : t_.add(CAT, {x, tail})});
      }
      if (tail >= 0)
        seq.push_back(tail);
    }
    if (seq.empty())
      return t_.add(EMPTY);
    return seq.size() == 1 ? seq[0] : t_.add(CAT, seq);
  }

  int parse_repeat()
  {
    bool dot = p_ < s_.size() && s_[p_] == '.';
    // convert.cpp:2118-2160: a Unicode '.' becomes one UTF-8 character unless
    // it is followed by '*' or '+', where it stays the byte class [^\n]
    bool dot_byte = dot && p_ + 1 < s_.size() && (s_[p_ + 1] == '*' || s_[p_ + 1] == '+');
    p_quirk_ = false;
    int a = parse_atom(dot_byte);
    // Matcher::convert pastes a \p{NAME} class in as the text of its UTF-8
    // byte regex, grouped only when that has alternatives; a class whose
    // encoding is one sequence with leading single bytes (\p{Ogham} =
    // \xe1\x9a[\x80-\x9c], \p{Braille} = \xe2(?:[\xa0-\xa3][\x80-\xbf]), \p{Zl})
    // then takes a quantifier on its last atom only: \p{Ogham}+ is
    // \xe1\x9a[\x80-\x9c]+ (measured on the reference's converted regexes,
    // tests/test_pclass.py)
    const bool quirk = p_quirk_;
    std::vector<int> prefix = p_prefix_;
    int q = quirk ? p_tail_ : a;
    bool quantified = false;
    while (p_ < s_.size())
    {
      char c = s_[p_];
      int lo, hi;
      if (c == '*')
      {
        ++p_;
        q = t_.add(STAR, {q});
      }
      else if (c == '+')
      {
        ++p_;
        q = t_.add(PLUS, {q});
      }
      else if (c == '?')
      {
        ++p_;
        q = t_.add(OPT, {q});
      }
      else if (c == '{')
      {
        if (!parse_braces(lo, hi))
          fail(UGPU_INVAL, "bad repeat");
        q = repeat(q, lo, hi);
      }
      else
        break;
      quantified = true;
      if (p_ < s_.size() && s_[p_] == '?')
        fail(UGPU_UNSUPPORTED, "lazy quantifier");
      if (p_ < s_.size() && s_[p_] == '+' )
        fail(UGPU_UNSUPPORTED, "possessive quantifier");
    }
    p_quirk_ = false;
    if (!quirk || !quantified)
      return quirk ? a : q;
    prefix.push_back(q);
    return t_.add(CAT, prefix);
  }

  uint32_t utf8_char()
  {
    // decode one (valid) UTF-8 character of the pattern at p_
    uint8_t c = static_cast<uint8_t>(s_[p_++]);
    if (c < 0x80)
      return c;
    int n = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : c >= 0xC0 ? 1 : -1;
    if (n < 0)
      fail(UGPU_UNSUPPORTED, "invalid UTF-8 in pattern");
    uint32_t v = c & (0x3F >> n);
    for (int i = 0; i < n; ++i)
    {
      if (p_ >= s_.size() || (static_cast<uint8_t>(s_[p_]) & 0xC0) != 0x80)
        fail(UGPU_UNSUPPORTED, "invalid UTF-8 in pattern");
      v = (v << 6) | (static_cast<uint8_t>(s_[p_++]) & 0x3F);
    }
    return v;
  }

  int hexval(char c)
  {
    if (c >= '0' && c <= '9')
      return c - '0';
    if (c >= 'a' && c <= 'f')
      return c - 'a' + 10;
    if (c >= 'A' && c <= 'F')
      return c - 'A' + 10;
    return -1;
  }

  // escape at p_ (just past '\'): returns true and a class set in `set`, or a
  // single code point in `cp`
  bool parse_escape(CpSet &set, uint32_t &cp, bool in_bracket)
  {
    if (p_ >= s_.size())
      fail(UGPU_INVAL, "trailing backslash");
    char c = s_[p_++];
    switch (c)
    {
      case 'w': set = word_set(); return true;
      case 'd': set = digit_set(); return true;
      case 's': set = space_set(); return true;
      case 'h': set = hspace_set(); return true;
      // negated classes, as the reference's DFAs have them (probed per code
      // point, tests/test_compile.py): outside brackets \W \D \H complement
      // over all scalar values (also '\n') and \S excludes '\n'; inside a
      // bracket \W and \D complement only up to the table's last code point,
      // while \S and \H keep the surrogate encodings
      case 'W':
        set = in_bracket ? no_surrogates(complement_upto(word_set(), word_set().back().second))
                         : complement(word_set());
        return true;
      case 'D':
        set = in_bracket ? no_surrogates(complement_upto(digit_set(), digit_set().back().second))
                         : complement(digit_set());
        return true;
      case 'S':
        set = minus(in_bracket ? complement_upto(space_set(), kMaxCp) : complement(space_set()),
                    CpSet{{'\n', '\n'}});
        return true;
      case 'H':
        set = in_bracket ? complement_upto(hspace_set(), kMaxCp) : complement(hspace_set());
        return true;
      case 'p':
      case 'P':
      {
        // \p{NAME}, \pL (lib/unicode.cpp, lib/language_scripts.cpp); \P
        // complements like \W: over all scalar values outside brackets, up to
        // the table's last code point inside
        std::string name;
        if (p_ < s_.size() && s_[p_] == '{')
        {
          size_t q = s_.find('}', p_);
          if (q == std::string::npos)
            fail(UGPU_INVAL, "missing '}'");
          name = s_.substr(p_ + 1, q - p_ - 1);
          p_ = q + 1;
        }
        else if (p_ < s_.size())
          name = std::string(1, s_[p_++]);
        CpSet t;
        bool pnl = true;
        if (!named_set(name, t, &pnl))
          fail(UGPU_UNSUPPORTED, "class \\p{" + name + "}");
        if (icase() && (name == "Lu" || name == "Ll" || name == "Lt" || name == "Upper" || name == "Lower" ||
                        name == "Uppercase_Letter" || name == "Lowercase_Letter" || name == "Titlecase_Letter"))
          fail(UGPU_UNSUPPORTED, "case class under -i");  // the reference widens these differently
        if (c == 'p')
          set = t;
        else
        {
          set = complement(t);  // '\n' stays out when the class itself holds it (pnl)
          if (!pnl)
            set = minus(set, CpSet{{'\n', '\n'}});
        }
        return true;
      }
      case 't': cp = '\t'; return false;
      case 'n': cp = '\n'; return false;
      case 'r': cp = '\r'; return false;
      case 'f': cp = '\f'; return false;
      case 'v': cp = '\v'; return false;
      case 'a': cp = '\a'; return false;
      case 'e': cp = 0x1B; return false;
      case 'x':
      {
        uint32_t v = 0;
        if (p_ < s_.size() && s_[p_] == '{')
        {
          size_t q = p_ + 1;
          int digits = 0;
          while (q < s_.size() && hexval(s_[q]) >= 0)
          {
            v = v * 16 + hexval(s_[q++]);
            if (++digits > 6)
              fail(UGPU_INVAL, "bad \\x{}");
          }
          if (q >= s_.size() || s_[q] != '}' || digits == 0 || v > kMaxCp)
            fail(UGPU_INVAL, "bad \\x{}");
          p_ = q + 1;
        }
        else
        {
          int digits = 0;
          while (digits < 2 && p_ < s_.size() && hexval(s_[p_]) >= 0)
          {
            v = v * 16 + hexval(s_[p_++]);
            ++digits;
          }
          if (digits == 0)
            fail(UGPU_INVAL, "bad \\x");
        }
        cp = v;
        return false;
      }
      case '0':
      {
        uint32_t v = 0;
        for (int i = 0; i < 3 && p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '7'; ++i)
          v = v * 8 + (s_[p_++] - '0');
        cp = v;
        return false;
      }
      default:
        break;
    }
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '1' && c <= '9'))
      fail(UGPU_UNSUPPORTED, std::string("escape \\") + c + (in_bracket ? " in bracket" : ""));
    --p_;
    cp = utf8_char();
    return false;
  }

  CpSet parse_bracket()
  {
    // p_ just past '['
    bool neg = false;
    if (p_ < s_.size() && s_[p_] == '^')
    {
      neg = true;
      ++p_;
    }
    CpSet set;
    bool first = true;
    for (;;)
    {
      if (p_ >= s_.size())
        fail(UGPU_INVAL, "unterminated bracket");
      char c = s_[p_];
      if (c == ']' && !first)
      {
        ++p_;
        break;
      }
      first = false;
      if (c == '[' && p_ + 1 < s_.size() && s_[p_ + 1] == ':')
      {
        // [:name:] (lib/posix.cpp names, the Unicode tables in Unicode mode)
        size_t q = s_.find(":]", p_ + 2);
        std::string name = q == std::string::npos ? "" : s_.substr(p_ + 2, q - p_ - 2);
        if (name.empty() || name[0] == '^')
          fail(UGPU_UNSUPPORTED, "POSIX bracket class");
        std::string cap = name;
        cap[0] = static_cast<char>(toupper(static_cast<unsigned char>(cap[0])));
        if (name == "xdigit")
          cap = "XDigit";
        else if (name == "ascii")
          cap = "ASCII";
        CpSet t;
        if (!named_set(cap, t))
          fail(UGPU_UNSUPPORTED, "POSIX bracket class [:" + name + ":]");
        set.insert(set.end(), t.begin(), t.end());
        p_ = q + 2;
        first = false;
        continue;
      }
      if (c == '[' && p_ + 1 < s_.size() && (s_[p_ + 1] == '.' || s_[p_ + 1] == '='))
        fail(UGPU_UNSUPPORTED, "POSIX collating element");
      uint32_t lo;
      CpSet cls;
      if (c == '\\')
      {
        ++p_;
        if (parse_escape(cls, lo, true))
        {
          set.insert(set.end(), cls.begin(), cls.end());
          continue;
        }
      }
      else
        lo = utf8_char();
      uint32_t hi = lo;
      if (p_ + 1 < s_.size() && s_[p_] == '-' && s_[p_ + 1] != ']')
      {
        ++p_;
        if (s_[p_] == '\\')
        {
          ++p_;
          if (parse_escape(cls, hi, true))
            fail(UGPU_INVAL, "class in range");
        }
        else
          hi = utf8_char();
        if (hi < lo)
          fail(UGPU_INVAL, "bad range");
      }
      set.push_back({lo, hi});
    }
    set = normalize(set);
    if (icase())
    {
      add_ascii_case(set);
      add_unicode_case(set);
    }
    if (neg)
      set = minus(complement(set), CpSet{{'\n', '\n'}});  // notnewline
    return set;
  }

  // ---- REFLEX mode: the RE/flex regex a Pattern holds (Pattern::operator[](0),
  // include/reflex/pattern.h:302), i.e. Matcher::convert's output
  // (lib/convert.cpp): bytes, not code points -- Unicode classes, '.' and -i
  // over non-ASCII letters are already expanded into byte sequences; inline
  // modifiers (?i) (?s) (?m) and (?i:...) scopes; \Q...\E quoting.

  // one byte escape at p_ (just past '\')
  uint8_t reflex_escape_byte()
  {
    if (p_ >= s_.size())
      fail(UGPU_INVAL, "trailing backslash");
    const char c = s_[p_++];
    switch (c)
    {
      case 't': return '\t';
      case 'n': return '\n';
      case 'r': return '\r';
      case 'f': return '\f';
      case 'v': return '\v';
      case 'a': return '\a';
      case 'e': return 0x1B;
      case '0':
      {
        uint32_t v = 0;
        for (int i = 0; i < 3 && p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '7'; ++i)
          v = v * 8 + (s_[p_++] - '0');
        if (v > 0xFF)
          fail(UGPU_UNSUPPORTED, "octal escape above 0xFF in byte mode");
        return static_cast<uint8_t>(v);
      }
      case 'x':
      {
        uint32_t v = 0;
        int digits = 0;
        const bool brace = p_ < s_.size() && s_[p_] == '{';
        if (brace)
          ++p_;
        while ((brace || digits < 2) && p_ < s_.size() && hexval(s_[p_]) >= 0)
        {
          v = v * 16 + hexval(s_[p_++]);
          if (++digits > 6)
            fail(UGPU_INVAL, "bad \\x");
        }
        if (brace)
        {
          if (p_ >= s_.size() || s_[p_] != '}')
            fail(UGPU_INVAL, "bad \\x{}");
          ++p_;
        }
        if (digits == 0)
          fail(UGPU_INVAL, "bad \\x");
        if (v > 0xFF)
          fail(UGPU_UNSUPPORTED, "\\x above 0xFF in byte mode");
        return static_cast<uint8_t>(v);
      }
      default:
        break;
    }
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '1' && c <= '9'))
      fail(UGPU_UNSUPPORTED, std::string("escape \\") + c + " in byte mode");
    return static_cast<uint8_t>(c);
  }

  // class escapes the Pattern itself resolves in a byte-mode regex (ugrep -U
  // leaves them to it: Matcher::convert without the unicode flag):
  // \s \S \h \H \d \D \l \L \u \U \w \W are the POSIX classes Space, Blank,
  // Digit, Lower, Upper, Word and their 256-byte complements (lib/pattern.cpp
  // :1660-1676 with its posix table :2714-2735; the complements include '\n')
  bool pattern_class_escape(char c, ByteSet &b)
  {
    const char *lower = "shdluw";
    const char *k = strchr(lower, c | 0x20);
    if (k == NULL || c == '\0')
      return false;
    if ((c | 0x20) == 'u' && p_ < s_.size() && s_[p_] == '{')
      return false;  // \u{...}: a code point
    if (icase() && ((c | 0x20) == 'l' || (c | 0x20) == 'u'))
      fail(UGPU_UNSUPPORTED, std::string("escape \\") + c + " under (?i)");
    ByteSet x;
    switch (c | 0x20)
    {
      case 's':
        for (unsigned v = '\t'; v <= '\r'; ++v)
          x.set(v);
        x.set(' ');
        break;
      case 'h':
        x.set('\t');
        x.set(' ');
        break;
      case 'd':
        for (unsigned v = '0'; v <= '9'; ++v)
          x.set(v);
        break;
      case 'l':
        for (unsigned v = 'a'; v <= 'z'; ++v)
          x.set(v);
        break;
      case 'u':
        for (unsigned v = 'A'; v <= 'Z'; ++v)
          x.set(v);
        break;
      case 'w':
        for (unsigned v = 0; v < 256; ++v)
          if ((v >= '0' && v <= '9') || (v >= 'A' && v <= 'Z') || (v >= 'a' && v <= 'z') || v == '_')
            x.set(v);
        break;
    }
    if (c >= 'A' && c <= 'Z')
      x.flip();
    b |= x;
    return true;
  }

  // "(?imsx-imsx)" starts at q
  bool modifier_at(size_t q) const
  {
    if (q + 1 >= s_.size() || s_[q] != '(' || s_[q + 1] != '?')
      return false;
    q += 2;
    while (q < s_.size() && strchr("imsx-", s_[q]) != NULL)
      ++q;
    return q < s_.size() && s_[q] == ')';
  }

  void fold_ascii(ByteSet &b)
  {
    for (unsigned x = 'a'; x <= 'z'; ++x)
      if (b.test(x) || b.test(x ^ 0x20))
      {
        b.set(x);
        b.set(x ^ 0x20);
      }
  }

  ByteSet parse_byte_bracket()
  {
    // p_ just past '['
    bool neg = false;
    if (p_ < s_.size() && s_[p_] == '^')
    {
      neg = true;
      ++p_;
    }
    ByteSet b;
    bool first = true;
    for (;;)
    {
      if (p_ >= s_.size())
        fail(UGPU_INVAL, "unterminated bracket");
      const char c = s_[p_];
      if (c == ']' && !first)
      {
        ++p_;
        break;
      }
      first = false;
      if (c == '[' && p_ + 1 < s_.size() && (s_[p_ + 1] == ':' || s_[p_ + 1] == '.' || s_[p_ + 1] == '='))
        fail(UGPU_UNSUPPORTED, "POSIX bracket in byte mode");
      uint8_t lo, hi;
      ++p_;
      if (c == '\\' && p_ < s_.size())
      {
        const char e = s_[p_++];
        if (pattern_class_escape(e, b))
          continue;
        --p_;
      }
      lo = c == '\\' ? reflex_escape_byte() : static_cast<uint8_t>(c);
      hi = lo;
      if (p_ + 1 < s_.size() && s_[p_] == '-' && s_[p_ + 1] != ']')
      {
        ++p_;
        const char d = s_[p_++];
        hi = d == '\\' ? reflex_escape_byte() : static_cast<uint8_t>(d);
        if (hi < lo)
          fail(UGPU_INVAL, "bad range");
      }
      for (unsigned x = lo; x <= hi; ++x)
        b.set(x);
    }
    if (icase())
      fold_ascii(b);
    if (neg)
      b.flip();
    return b;
  }

  int parse_atom_reflex()
  {
    const char c = s_[p_];
    switch (c)
    {
      case '(':
      {
        ++p_;
        const bool ic = ic_, dot = dotall_;
        if (p_ + 1 < s_.size() && s_[p_] == '?' && s_[p_ + 1] == '^')
          return negative_group();
        if (p_ + 1 < s_.size() && s_[p_] == '?' && s_[p_ + 1] == '=')
          return lookahead_group();
        if (p_ < s_.size() && s_[p_] == '?')
        {
          // (?imsx-imsx) modifies the rest of the enclosing group,
          // (?imsx-imsx:...) just the group; anything else ((?=, (?^ ...) is not a DFA
          size_t q = p_ + 1;
          bool on = true, i = ic_, d = dotall_, m = multiline_;
          while (q < s_.size() && strchr("imsx-", s_[q]) != NULL)
          {
            switch (s_[q])
            {
              case '-': on = false; break;
              case 'i': i = on; break;
              case 's': d = on; break;
              case 'x': if (on) fail(UGPU_UNSUPPORTED, "free-space mode"); break;
              case 'm': m = on; break;
              default: break;
            }
            ++q;
          }
          if (q < s_.size() && s_[q] == ')')
          {
            p_ = q + 1;
            ic_ = i;
            dotall_ = d;
            multiline_ = m;
            return t_.add(EMPTY);
          }
          if (q >= s_.size() || s_[q] != ':')
            fail(UGPU_UNSUPPORTED, "(? group");
          p_ = q + 1;
          ic_ = i;
          dotall_ = d;
        }
        ++depth_;
        int a = parse_alt();
        --depth_;
        if (p_ >= s_.size() || s_[p_] != ')')
          fail(UGPU_INVAL, "missing ')'");
        ++p_;
        ic_ = ic;
        dotall_ = dot;
        return a;
      }
      case '[':
        ++p_;
        return t_.leaf(parse_byte_bracket());
      case '.':
      {
        ++p_;
        ByteSet b;
        b.set();
        if (!dotall_)
          b.reset('\n');
        return t_.leaf(b);
      }
      case '^':
      case '$':
        fail(UGPU_UNSUPPORTED, "anchor");
      case '*':
      case '+':
      case '?':
      case '{':
        fail(UGPU_INVAL, "nothing to repeat");
      case '\\':
      {
        ++p_;
        if (p_ < s_.size() && s_[p_] == 'Q')
        {
          // \Q...\E: literal bytes
          ++p_;
          size_t q = s_.find("\\E", p_);
          const size_t e = q == std::string::npos ? s_.size() : q;
          std::vector<int> seq;
          for (; p_ < e; ++p_)
            seq.push_back(literal_byte(static_cast<uint8_t>(s_[p_])));
          p_ = q == std::string::npos ? s_.size() : q + 2;
          if (seq.empty())
            return t_.add(EMPTY);
          return seq.size() == 1 ? seq[0] : t_.add(CAT, seq);
        }
        if (p_ < s_.size())
        {
          ByteSet cls;
          const char e = s_[p_++];
          if (pattern_class_escape(e, cls))
            return t_.leaf(cls);
          --p_;
        }
        if (p_ < s_.size() && strchr("bBAzZ<>`'GkKEXRNuUcCldDwWsShHpPiIjJ", s_[p_]) != NULL)
          fail(UGPU_UNSUPPORTED, std::string("escape \\") + s_[p_] + " in byte mode");
        return literal_byte(reflex_escape_byte());
      }
      default:
        ++p_;
        return literal_byte(static_cast<uint8_t>(c));
    }
  }

  int parse_atom(bool dot_byte)
  {
    if (reflex())
      return parse_atom_reflex();
    char c = s_[p_];
    switch (c)
    {
      case '(':
      {
        ++p_;
        if (p_ + 1 < s_.size() && s_[p_] == '?' && s_[p_ + 1] == '^')
          return negative_group();
        if (p_ + 1 < s_.size() && s_[p_] == '?' && s_[p_ + 1] == '=')
          return lookahead_group();
        if (p_ < s_.size() && s_[p_] == '?')
        {
          if (p_ + 1 < s_.size() && s_[p_ + 1] == ':')
            p_ += 2;
          else
            fail(UGPU_UNSUPPORTED, "(? group");
        }
        ++depth_;
        int a = parse_alt();
        --depth_;
        if (p_ >= s_.size() || s_[p_] != ')')
          fail(UGPU_INVAL, "missing ')'");
        ++p_;
        return a;
      }
      case '[':
        ++p_;
        return t_.cpset(parse_bracket());
      case '.':
        ++p_;
        if (dot_byte)
        {
          ByteSet b;
          b.set();
          b.reset('\n');
          return t_.leaf(b);
        }
        else
        {
          // [^\n\x80-\xbf][\x80-\xbf]*  (convert.cpp:2118-2150)
          ByteSet lead, cont;
          for (unsigned x = 0; x < 256; ++x)
            (x >= 0x80 && x <= 0xBF ? cont : lead).set(x);
          lead.reset('\n');
          int l = t_.leaf(lead);
          return t_.add(CAT, {l, t_.add(STAR, {t_.leaf(cont)})});
        }
      case '^':
      case '$':
        fail(UGPU_UNSUPPORTED, "anchor");
      case '*':
      case '+':
      case '?':
      case '{':
        fail(UGPU_INVAL, "nothing to repeat");
      case '\\':
      {
        ++p_;
        if (p_ < s_.size() && strchr("bBAzZ<>`'GkKQEXRNuUcCl", s_[p_]) != NULL)
          fail(UGPU_UNSUPPORTED, std::string("escape \\") + s_[p_]);
        CpSet set;
        uint32_t cp;
        const bool pclass = p_ < s_.size() && s_[p_] == 'p';
        if (parse_escape(set, cp, false))
        {
          if (icase())
          {
            add_ascii_case(set);
            add_unicode_case(set);
          }
          const std::vector<std::pair<uint8_t, uint8_t>> seq = pclass ? t_.single_product(set) : decltype(seq)();
          if (seq.size() >= 2 && seq[0].first == seq[0].second)
          {
            // (parse_repeat: a quantifier takes the last atom of convert's text)
            size_t j = 0;
            while (j < seq.size() && seq[j].first == seq[j].second)
              ++j;
            if (j == seq.size())
              --j;  // (one code point: the last byte is the last atom)
            p_prefix_.clear();
            for (size_t k = 0; k < j; ++k)
              p_prefix_.push_back(t_.leaf_range(seq[k].first, seq[k].second));
            std::vector<int> rest;
            for (size_t k = j; k < seq.size(); ++k)
              rest.push_back(t_.leaf_range(seq[k].first, seq[k].second));
            p_tail_ = rest.size() == 1 ? rest[0] : t_.add(CAT, rest);
            p_quirk_ = true;
            std::vector<int> all(p_prefix_);
            all.push_back(p_tail_);
            return t_.add(CAT, all);
          }
          return t_.cpset(set);
        }
        return code_point(cp, true);
      }
      default:
        return code_point(utf8_char());
    }
  }

  // escaped: from \x{..}/\0ooo, which (?i) leaves unfolded (measured on the
  // reference's tables: (?i)\x{e9} matches only U+00E9, (?i)é also U+00C9)
  int code_point(uint32_t cp, bool escaped = false)
  {
    if (cp < 0x80)
      return literal_byte(static_cast<uint8_t>(cp));
    CpSet s{{cp, cp}};
    uint32_t v = icase() && !escaped ? case_variant(cp) : 0;
    if (v)
      s.push_back({v, v});
    return t_.cpset(s);
  }
};

// ---------------------------------------------------------------- Glushkov + subsets

struct Glushkov
{
  const Tree &t;
  std::vector<int> pos_of;               // node -> position (leaves)
  std::vector<ByteSet> bytes;            // position -> bytes
  std::vector<std::vector<int>> follow;  // position -> follow positions
  std::vector<int> accept;               // position -> accept index (end markers), 0 otherwise
  std::vector<std::vector<uint8_t>> metas;  // end marker -> its alternative's meta edges (Parser::metaseqs)
  std::vector<bool> neg;                    // end marker of a negative pattern (Parser::negs): REDO
  // lookahead markers (no bytes, never followed): HEAD la (the reference's
  // "(" position) and TAIL la (its ticked ")" position, valid in states that
  // accept alternative look_alt), -1 = none
  std::vector<int> look_head, look_tail, look_alt;

  struct Info
  {
    bool nullable;
    std::vector<int> first, last;
  };

  explicit Glushkov(const Tree &tree) : t(tree), pos_of(tree.nodes.size(), -1) {}

  static void merge(std::vector<int> &a, const std::vector<int> &b)
  {
    std::vector<int> out;
    std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(out));
    a.swap(out);
  }

  void link(const std::vector<int> &from, const std::vector<int> &to)
  {
    for (int p : from)
      merge(follow[p], to);
  }

  int new_pos(const ByteSet &b, int acc)
  {
    bytes.push_back(b);
    follow.emplace_back();
    accept.push_back(acc);
    metas.emplace_back();
    neg.push_back(false);
    look_head.push_back(-1);
    look_tail.push_back(-1);
    look_alt.push_back(0);
    return static_cast<int>(bytes.size() - 1);
  }

  Info walk(int n)
  {
    const Node &nd = t.nodes[n];
    Info r;
    switch (nd.kind)
    {
      case LEAF:
      {
        int p = new_pos(nd.bytes, 0);
        return Info{false, {p}, {p}};
      }
      case EMPTY:
        return Info{true, {}, {}};
      case CAT:
      {
        r = walk(nd.kids[0]);
        for (size_t i = 1; i < nd.kids.size(); ++i)
        {
          Info b = walk(nd.kids[i]);
          link(r.last, b.first);
          if (r.nullable)
            merge(r.first, b.first);
          if (b.nullable)
            merge(b.last, r.last);
          r.last.swap(b.last);
          r.nullable = r.nullable && b.nullable;
        }
        return r;
      }
      case ALT:
      {
        r.nullable = false;
        for (int k : nd.kids)
        {
          Info b = walk(k);
          r.nullable = r.nullable || b.nullable;
          merge(r.first, b.first);
          merge(r.last, b.last);
        }
        return r;
      }
      case LOOK:
      {
        // lib/pattern.cpp:1346-1358: first(Y) + HEAD, last(Y) -> TAIL, last
        // = last(Y) + TAIL; a nullable Y also starts with TAIL and ends with HEAD
        Info y = walk(nd.kids[0]);
        const int h = new_pos(ByteSet(), 0);
        look_head[h] = nd.look;
        const int tl = new_pos(ByteSet(), 0);
        look_tail[tl] = nd.look;
        look_alt[tl] = nd.look_alt;
        link(y.last, std::vector<int>{tl});
        r.nullable = y.nullable;
        r.first = y.first;
        merge(r.first, std::vector<int>{h});
        r.last = y.last;
        merge(r.last, std::vector<int>{tl});
        if (y.nullable)
        {
          merge(r.first, std::vector<int>{tl});
          merge(r.last, std::vector<int>{h});
        }
        return r;
      }
      case STAR:
      case PLUS:
      case OPT:
      {
        r = walk(nd.kids[0]);
        if (nd.kind != OPT)
          link(r.last, r.first);
        if (nd.kind != PLUS)
          r.nullable = true;
        return r;
      }
    }
    return r;
  }
};

// accept index per line context (bit 0: the walk began at a line begin, bit 1:
// a line end follows), the lowest satisfied top-level alternative, 0 = none
typedef std::array<uint32_t, 4> Ctx4;
// per context: 4 line contexts as Ctx4, or (word boundaries) 64 contexts in
// the tables' layout (ctx_bits.hpp)
typedef std::vector<uint32_t> CtxN;

// the word-boundary classes of a 64-context index: of the match begin (A:
// at_bw && at_wb, B: neither, N: one) and of the position (A: at_we && at_ew)
inline int bcls_of(uint32_t ctx)
{
  const bool bw = ctx & CTX_BW, wb = ctx & CTX_WB;
  return bw && wb ? 0 : (!bw && !wb) ? 1 : 2;
}
inline int ecls_of(uint32_t ctx)
{
  const bool we = ctx & CTX_WE, ew = ctx & CTX_EW;
  return we && ew ? 0 : (!we && !ew) ? 1 : 2;
}
// a context of classes (bc, ec) and line bits
inline uint32_t ctx_of(int bc, int ec, bool bol, bool eol)
{
  uint32_t c = bc == 0 ? (CTX_BW | CTX_WB) : bc == 1 ? 0u : CTX_BW;
  c |= ec == 0 ? (CTX_WE | CTX_EW) : ec == 1 ? 0u : CTX_WE;
  return c | (bol ? CTX_BOL : 0u) | (eol ? CTX_EOL : 0u);
}

// Whether meta edge `m` (META - META_MIN) holds in context ctx: 4 line
// contexts (bit 0 bol, bit 1 eol) or 64 (ctx_bits.hpp)
inline bool meta_holds_ctx(uint8_t m, uint32_t ctx, bool word)
{
  if (!word)
    return m == 0x09 ? (ctx & 1) != 0 : m == 0x0a ? (ctx & 2) != 0 : false;
  const bool eol = ctx & CTX_EOL, ew = ctx & CTX_EW, we = ctx & CTX_WE, bol = ctx & CTX_BOL, wb = ctx & CTX_WB,
             bw = ctx & CTX_BW;
  switch (m)
  {
    case 0x01: return bw == wb;
    case 0x02: return we == ew;
    case 0x03: return bw != wb;
    case 0x04: return we != ew;
    case 0x05: return bw && wb;
    case 0x06: return !bw && !wb;
    case 0x07: return !we && !ew;
    case 0x08: return we && ew;
    case 0x09: return bol;
    default: return eol;
  }
}

// The accept of a DFA state whose ends are `acc` (accept index, meta edges),
// as RE/flex builds and the interpreter evaluates it (lib/matcher.cpp:193-450):
// the state's TAKE is its lowest index without meta edges; its meta edges,
// one per distinct next meta, are tried in descending META code (the order
// encode_dfa emits them, lib/pattern.cpp:2945-2990), the first that holds is
// followed to the alternatives that wait for it, whose finished ones give the
// TAKE there (lowest index), and so on (at most 5 jumps).  So the accept is not
// the lowest satisfied index: in ^ab|ab$ with both anchors holding, EOL is
// tried first and gives 2.
uint32_t meta_accept(const std::vector<std::pair<uint32_t, const std::vector<uint8_t> *>> &acc, uint32_t ctx,
                     bool word)
{
  uint32_t cap = 0;
  std::vector<std::pair<uint32_t, size_t>> cur;  // (index into acc, next meta)
  for (size_t i = 0; i < acc.size(); ++i)
  {
    if (acc[i].second->empty())
      cap = cap == 0 || acc[i].first < cap ? acc[i].first : cap;
    else
      cur.emplace_back(static_cast<uint32_t>(i), 0);
  }
  for (int jumps = 0; jumps < 5 && !cur.empty(); ++jumps)
  {
    int best = -1;
    for (auto &c : cur)
    {
      const uint8_t m = (*acc[c.first].second)[c.second];
      if (m > best && meta_holds_ctx(m, ctx, word))
        best = m;
    }
    if (best < 0)
      break;
    std::vector<std::pair<uint32_t, size_t>> nxt;
    uint32_t done = 0;
    for (auto &c : cur)
    {
      const std::vector<uint8_t> &ms = *acc[c.first].second;
      if (ms[c.second] != best)
        continue;
      if (c.second + 1 == ms.size())
        done = done == 0 || acc[c.first].first < done ? acc[c.first].first : done;
      else
        nxt.emplace_back(c.first, c.second + 1);
    }
    if (done)
      cap = done;
    cur.swap(nxt);
  }
  return cap;
}

struct Dfa
{
  std::vector<std::vector<uint32_t>> next;  // state -> 256 targets (0 = dead state)
  std::vector<uint32_t> acc;                // accept index without context (cx[s][0]), 0 = none
  std::vector<CtxN> cx;                     // accept index per context
  uint32_t nctx = 4;                        // 4 (line anchors) or 64 (word boundaries)
  bool anchored = false;                    // some accept depends on the context
  // lookahead per state: bits 0-15 TAIL la, bits 16-31 HEAD la (empty: none)
  std::vector<uint32_t> look;
};

inline uint32_t look_of(const Dfa &d, size_t s) { return d.look.empty() ? 0u : d.look[s]; }

Dfa subsets(Glushkov &g, const std::vector<int> &start)
{
  Dfa d;
  std::map<std::vector<int>, uint32_t> id;
  std::vector<std::vector<int>> sets;
  auto intern = [&](const std::vector<int> &s) -> uint32_t {
    auto it = id.find(s);
    if (it != id.end())
      return it->second;
    if (sets.size() >= kMaxStates)
      fail(UGPU_UNSUPPORTED, "DFA too large");
    uint32_t k = static_cast<uint32_t>(sets.size());
    id.emplace(s, k);
    sets.push_back(s);
    return k;
  };
  intern({});  // state 0: dead
  intern(start);
  // byte classes over all positions, to do one union per class
  std::vector<int> cls(256, 0);
  {
    std::map<std::vector<bool>, int> sig;
    for (int b = 0; b < 256; ++b)
    {
      std::vector<bool> v(g.bytes.size());
      for (size_t p = 0; p < g.bytes.size(); ++p)
        v[p] = g.bytes[p].test(b);
      auto it = sig.emplace(v, static_cast<int>(sig.size())).first;
      cls[b] = it->second;
    }
  }
  int ncls = *std::max_element(cls.begin(), cls.end()) + 1;
  std::vector<int> rep(ncls, -1);
  for (int b = 0; b < 256; ++b)
    if (rep[cls[b]] < 0)
      rep[cls[b]] = b;
  for (const auto &ms : g.metas)
    for (uint8_t m : ms)
      if (m <= 0x08)
        d.nctx = 64;
  for (size_t k = 0; k < sets.size(); ++k)
  {
    std::vector<int> cur = sets[k];  // copy: sets grows
    CtxN cx(d.nctx, 0);
    std::vector<std::pair<uint32_t, const std::vector<uint8_t> *>> acc;  // (accept index, meta edges) of the state's ends
    bool redo = false;
    for (int p : cur)
      if (g.accept[p])
      {
        acc.emplace_back(static_cast<uint32_t>(g.accept[p]), &g.metas[p]);
        redo = redo || g.neg[p];
      }
    if (!acc.empty())
      for (uint32_t ctx = 0; ctx < d.nctx; ++ctx)
        cx[ctx] = redo ? kRedoAcc : meta_accept(acc, ctx, d.nctx == 64);
    d.acc.push_back(cx[0]);
    {
      // the state's lookahead block (lib/pattern.cpp:2374-2419): HEAD la for
      // every "(" marker; TAIL la for a ")" marker of the alternative the state
      // accepts (its lowest accept index)
      uint32_t acc0 = 0, lk = 0;
      for (int p : cur)
        if (g.accept[p] && (acc0 == 0 || static_cast<uint32_t>(g.accept[p]) < acc0))
          acc0 = static_cast<uint32_t>(g.accept[p]);
      for (int p : cur)
      {
        if (g.look_head[p] >= 0)
          lk |= 1u << (16 + g.look_head[p]);
        if (g.look_tail[p] >= 0 && acc0 != 0 && static_cast<uint32_t>(g.look_alt[p]) == acc0)
          lk |= 1u << g.look_tail[p];
      }
      d.look.push_back(lk);
    }
    for (uint32_t ctx = 1; ctx < d.nctx; ++ctx)
      d.anchored = d.anchored || cx[ctx] != cx[0];
    d.cx.push_back(cx);
    std::vector<uint32_t> row(256, 0);
    std::vector<uint32_t> by_cls(ncls, 0);
    for (int c = 0; c < ncls; ++c)
    {
      std::vector<int> nx;
      for (int p : cur)
        if (!g.accept[p] && g.bytes[p].test(rep[c]))
          Glushkov::merge(nx, g.follow[p]);
      by_cls[c] = nx.empty() ? 0 : intern(nx);
    }
    for (int b = 0; b < 256; ++b)
      row[b] = by_cls[cls[b]];
    d.next.push_back(row);
  }
  return d;
}

// Moore minimisation; states that cannot reach an accept collapse into the
// dead state 0.  Returns the minimal DFA with the start state at index 1.
Dfa minimize(const Dfa &d, uint32_t start)
{
  size_t n = d.acc.size();
  std::vector<uint32_t> part(n);
  // lookahead blocks count only in states that can still reach an accept (a
  // HEAD in a state that never accepts changes no match: such states stay dead)
  std::vector<uint32_t> lk(n, 0);
  if (!d.look.empty())
  {
    std::vector<bool> live(n, false);
    for (size_t s = 0; s < n; ++s)
      for (uint32_t v : d.cx[s])
        live[s] = live[s] || v != 0;
    for (bool grew = true; grew;)
    {
      grew = false;
      for (size_t s = 0; s < n; ++s)
        if (!live[s])
          for (int b = 0; b < 256 && !live[s]; ++b)
            if (live[d.next[s][b]])
              live[s] = grew = true;
    }
    for (size_t s = 0; s < n; ++s)
      lk[s] = live[s] ? d.look[s] : 0;
  }
  {
    std::map<std::pair<CtxN, uint32_t>, uint32_t> m;
    for (size_t s = 0; s < n; ++s)
      part[s] = m.emplace(std::make_pair(d.cx[s], lk[s]), static_cast<uint32_t>(m.size())).first->second;
  }
  size_t nparts = 0;
  for (;;)
  {
    std::map<std::vector<uint32_t>, uint32_t> m;
    std::vector<uint32_t> np(n);
    for (size_t s = 0; s < n; ++s)
    {
      std::vector<uint32_t> sig;
      sig.reserve(257);
      sig.push_back(part[s]);
      for (int b = 0; b < 256; ++b)
        sig.push_back(part[d.next[s][b]]);
      np[s] = m.emplace(sig, static_cast<uint32_t>(m.size())).first->second;
    }
    part.swap(np);
    if (m.size() == nparts)
      break;
    nparts = m.size();
  }
  // renumber by BFS from the start; the dead state's block becomes 0
  uint32_t dead = part[0];
  std::vector<int64_t> newid(nparts, -1);
  std::vector<uint32_t> rep(nparts);
  for (size_t s = n; s-- > 0;)
    rep[part[s]] = static_cast<uint32_t>(s);
  Dfa out;
  out.anchored = d.anchored;
  out.nctx = d.nctx;
  newid[dead] = 0;
  out.acc.push_back(0);
  out.cx.push_back(CtxN(d.nctx, 0));
  out.next.push_back(std::vector<uint32_t>(256, 0));
  if (!d.look.empty())
    out.look.push_back(0);
  std::vector<uint32_t> order{part[start]};
  if (part[start] != dead)
    newid[part[start]] = 1;
  for (size_t i = 0; i < order.size(); ++i)
  {
    uint32_t blk = order[i];
    if (blk == dead)
      continue;
    uint32_t s = rep[blk];
    std::vector<uint32_t> row(256);
    for (int b = 0; b < 256; ++b)
    {
      uint32_t tb = part[d.next[s][b]];
      if (newid[tb] < 0)
      {
        newid[tb] = static_cast<int64_t>(order.size()) + 1;
        order.push_back(tb);
      }
      row[b] = static_cast<uint32_t>(newid[tb]);
    }
    out.acc.push_back(d.acc[s]);
    out.cx.push_back(d.cx[s]);
    out.next.push_back(row);
    if (!d.look.empty())
      out.look.push_back(lk[s]);
  }
  return out;
}

// Split states by their walk gap (bytes since the walk's last accept, 0 on
// accepting states and at the start) so that every state has one gap, the
// property xg_kernel's tables need (tables.cpp, "gap transducer").  Minimising
// can merge states the reference's construction keeps apart (e.g. UTF-8
// continuation states reached from the start and after an accept); unfolding
// restores a layout the gap kernel takes.  Gives up (returns d) when a gap
// exceeds the kernel's bound or the table would grow past 4x.
Dfa unfold_gaps(const Dfa &d)
{
  const int kMaxGap = 6;
  size_t n = d.acc.size();
  if (n < 2 || d.anchored)
    return d;  // (no gap transducer for context-dependent accepts: tables.cpp)
  for (size_t s = 0; s < n; ++s)
    if (look_of(d, s))
      return d;  // (nor for lookahead tables)
  std::map<std::pair<uint32_t, int>, uint32_t> id;
  std::vector<std::pair<uint32_t, int>> order{{0, -1}, {1, 0}};
  id[order[0]] = 0;
  id[order[1]] = 1;
  Dfa out;
  for (size_t i = 0; i < order.size(); ++i)
  {
    uint32_t s = order[i].first;
    int g = order[i].second;
    std::vector<uint32_t> row(256, 0);
    if (s != 0)
      for (int b = 0; b < 256; ++b)
      {
        uint32_t t = d.next[s][b];
        if (t == 0)
          continue;
        int ng = d.acc[t] ? 0 : g + 1;
        if (ng > kMaxGap)
          return d;
        auto key = std::make_pair(t, ng);
        auto it = id.find(key);
        if (it == id.end())
        {
          if (order.size() >= 4 * n)
            return d;
          it = id.emplace(key, static_cast<uint32_t>(order.size())).first;
          order.push_back(key);
        }
        row[b] = it->second;
      }
    out.next.push_back(row);
    out.acc.push_back(d.acc[s]);
    out.cx.push_back(d.cx[s]);
  }
  return out;
}

// ---------------------------------------------------------------- opcode encoding

std::vector<uint32_t> encode(const Dfa &d)
{
  // states 1..n-1 are emitted in order as blocks 0..n-2 (state 1, the start,
  // at word 0), then the accept-only blocks that context-dependent accepts
  // point at through META_BOL / META_EOL words
  size_t n = d.acc.size();
  if (n < 2)
  {
    // no live start: a start state that halts on every byte
    return std::vector<uint32_t>{0x00FFFFFFu};
  }
  struct Run
  {
    unsigned lo, hi;
    uint32_t target;  // block index + 1, 0 = HALT
  };
  struct Block
  {
    uint32_t take = 0;
    uint32_t look = 0;  // TAIL la (bits 0-15), HEAD la (bits 16-31)
    std::vector<std::pair<uint32_t, uint32_t>> metas;  // (META - META_MIN, block index + 1)
    std::vector<Run> runs;
  };
  const uint32_t kBol = 0x09, kEol = 0x0a;  // META_BOL, META_EOL - META_MIN (pattern.h:942-943)
  std::vector<Block> blocks(n - 1);
  for (size_t s = 1; s < n; ++s)
  {
    int b = 255;
    while (b >= 0)
    {
      uint32_t t = d.next[s][b];
      int e = b;
      while (e > 0 && d.next[s][e - 1] == t)
        --e;
      // dead runs become HALT words: every byte of a state block is covered
      // and its last word has lo == 0, as encode_dfa emits them
      blocks[s - 1].runs.push_back(Run{static_cast<unsigned>(e), static_cast<unsigned>(b), t});
      b = e - 1;
    }
    blocks[s - 1].look = look_of(d, s);
  }
  // accept-only blocks: P(v) = TAKE v; Q(a, b) = TAKE a, then META_EOL -> P(b)
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> extra;
  auto accept_only = [&](uint32_t a, uint32_t b) -> uint32_t {
    auto key = std::make_pair(a, b);
    auto it = extra.find(key);
    if (it != extra.end())
      return it->second;
    Block k;
    k.take = a;
    if (b != a)
    {
      uint32_t pb = 0;
      {
        auto key2 = std::make_pair(b, b);
        auto it2 = extra.find(key2);
        if (it2 == extra.end())
        {
          Block pk;
          pk.take = b;
          pk.runs.push_back(Run{0, 255, 0});
          blocks.push_back(pk);
          it2 = extra.emplace(key2, static_cast<uint32_t>(blocks.size())).first;
        }
        pb = it2->second;
      }
      k.metas.push_back(std::make_pair(kEol, pb));
    }
    k.runs.push_back(Run{0, 255, 0});
    blocks.push_back(k);
    return extra.emplace(key, static_cast<uint32_t>(blocks.size())).first->second;
  };
  // a state's accept per line context f = cx[s] (bit 0 bol, bit 1 eol) as the
  // reference evaluates it (lib/matcher.cpp:193-450): its TAKE f[0], then the
  // first meta edge that holds -- BOL to Q(f[1], f[3]) (whose EOL edge gives
  // f[3]), else EOL to P(f[2])
  // the line encoding of f (bit 0 bol, bit 1 eol) into block k
  auto line_encode = [&](size_t bi, const Ctx4 &f) {
    blocks[bi].take = f[0];
    const bool by_bol = f[1] != f[0] || f[3] != f[2];
    const bool by_eol = f[2] != f[0] || f[3] != f[1];
    if (by_bol && by_eol)
    {
      const uint32_t q = accept_only(f[1], f[3]);
      blocks[bi].metas.push_back(std::make_pair(kBol, q));
      if (f[2] != f[0])
      {
        const uint32_t pe = accept_only(f[2], f[2]);
        blocks[bi].metas.push_back(std::make_pair(kEol, pe));
      }
    }
    else if (by_bol)
    {
      const uint32_t pb = accept_only(f[1], f[1]);  // (before indexing: blocks may grow)
      blocks[bi].metas.push_back(std::make_pair(kBol, pb));
    }
    else if (by_eol)
    {
      const uint32_t pe = accept_only(f[2], f[2]);
      blocks[bi].metas.push_back(std::make_pair(kEol, pe));
    }
  };
  if (d.nctx == 64)
  {
    // word boundaries: per state, an exhaustive split over the match begin's
    // class (META_BWB A, META_EWB B, META_NWB N: exactly one holds), each
    // target an exhaustive split over the position's class (META_EWE A,
    // META_BWE B, META_NWE N), each of those the line encoding -- at most 4
    // meta jumps (the interpreter follows 5, lib/matcher.cpp:194-195).  A
    // block with splits carries no TAKE (a later TAKE cannot cancel one).
    const uint32_t kBWB = 0x05, kEWB = 0x06, kNWB = 0x03, kEWE = 0x08, kBWE = 0x07, kNWE = 0x04;
    std::map<Ctx4, uint32_t> line_blocks;
    auto line_block = [&](const Ctx4 &f) -> uint32_t {
      auto it = line_blocks.find(f);
      if (it != line_blocks.end())
        return it->second;
      Block k;
      k.runs.push_back(Run{0, 255, 0});
      blocks.push_back(k);
      const uint32_t id = static_cast<uint32_t>(blocks.size());
      line_encode(id - 1, f);
      return line_blocks.emplace(f, id).first->second;
    };
    auto line_of = [](const CtxN &f, int bc, int ec) {
      Ctx4 r;
      for (int i = 0; i < 4; ++i)
        r[i] = f[ctx_of(bc, ec, i & 1, (i >> 1) & 1)];
      return r;
    };
    // the position-class level for begin class bc into block bi
    auto e_encode = [&](size_t bi, const CtxN &f, int bc) {
      const Ctx4 a = line_of(f, bc, 0), b = line_of(f, bc, 1), c = line_of(f, bc, 2);
      if (a == b && b == c)
      {
        line_encode(bi, a);
        return;
      }
      const uint32_t ta = line_block(a), tb = line_block(b), tc = line_block(c);
      blocks[bi].metas.push_back(std::make_pair(kEWE, ta));
      blocks[bi].metas.push_back(std::make_pair(kBWE, tb));
      blocks[bi].metas.push_back(std::make_pair(kNWE, tc));
    };
    std::map<std::array<Ctx4, 3>, uint32_t> e_blocks;
    auto e_block = [&](const CtxN &f, int bc) -> uint32_t {
      const std::array<Ctx4, 3> key{line_of(f, bc, 0), line_of(f, bc, 1), line_of(f, bc, 2)};
      auto it = e_blocks.find(key);
      if (it != e_blocks.end())
        return it->second;
      Block k;
      k.runs.push_back(Run{0, 255, 0});
      blocks.push_back(k);
      const uint32_t id = static_cast<uint32_t>(blocks.size());
      e_encode(id - 1, f, bc);
      return e_blocks.emplace(key, id).first->second;
    };
    for (size_t s = 1; s < n; ++s)
    {
      const CtxN f = d.cx[s];  // (copy: blocks grows)
      bool by_b = false;
      for (uint32_t ctx = 0; ctx < 64 && !by_b; ++ctx)
        by_b = f[ctx] != f[ctx_of(0, ecls_of(ctx), ctx & CTX_BOL, ctx & CTX_EOL)];
      if (by_b)
      {
        const uint32_t xa = e_block(f, 0), xb = e_block(f, 1), xn = e_block(f, 2);
        blocks[s - 1].metas.push_back(std::make_pair(kBWB, xa));
        blocks[s - 1].metas.push_back(std::make_pair(kEWB, xb));
        blocks[s - 1].metas.push_back(std::make_pair(kNWB, xn));
      }
      else
        e_encode(s - 1, f, 0);
    }
  }
  for (size_t s = 1; s < n && d.nctx == 4; ++s)
  {
    Ctx4 f;
    std::copy(d.cx[s].begin(), d.cx[s].end(), f.begin());
    Block &k = blocks[s - 1];
    k.take = f[0];
    const bool by_bol = f[1] != f[0] || f[3] != f[2];
    const bool by_eol = f[2] != f[0] || f[3] != f[1];
    if (by_bol && by_eol)
    {
      const uint32_t q = accept_only(f[1], f[3]);
      blocks[s - 1].metas.push_back(std::make_pair(kBol, q));
      if (f[2] != f[0])
      {
        const uint32_t pe = accept_only(f[2], f[2]);
        blocks[s - 1].metas.push_back(std::make_pair(kEol, pe));
      }
    }
    else if (by_bol)
    {
      const uint32_t pb = accept_only(f[1], f[1]);
      blocks[s - 1].metas.push_back(std::make_pair(kBol, pb));
    }
    else if (by_eol)
    {
      const uint32_t pe = accept_only(f[2], f[2]);
      blocks[s - 1].metas.push_back(std::make_pair(kEol, pe));
    }
  }
  const size_t nb = blocks.size();
  for (int pass = 0; pass < 2; ++pass)
  {
    bool lng = pass == 1;
    std::vector<uint32_t> at(nb + 1, 0);
    uint32_t w = 0;
    for (size_t i = 0; i < nb; ++i)
    {
      at[i + 1] = w;
      w += blocks[i].take ? 1 : 0;
      w += static_cast<uint32_t>(__builtin_popcount(blocks[i].look));
      w += static_cast<uint32_t>(blocks[i].metas.size()) * (lng ? 2 : 1);
      for (auto &r : blocks[i].runs)
        w += (lng && r.target != 0) ? 2 : 1;
    }
    if (!lng && w >= 0xFFFE)
      continue;
    if (w > 0xFFFFFF)
      fail(UGPU_UNSUPPORTED, "opcode table too large");
    std::vector<uint32_t> out;
    out.reserve(w);
    for (size_t i = 0; i < nb; ++i)
    {
      const Block &k = blocks[i];
      if (k.take == kRedoAcc)
        out.push_back(0xFD000000u);  // REDO (lib/pattern.cpp:2945-2947)
      else if (k.take)
        out.push_back(0xFE000000u | k.take);
      // TAIL la then HEAD la, each ascending (lib/pattern.cpp:2953-2964)
      for (uint32_t i = 0; i < 16; ++i)
        if (k.look >> i & 1u)
          out.push_back(0xFC000000u | i);
      for (uint32_t i = 0; i < 16; ++i)
        if (k.look >> (16 + i) & 1u)
          out.push_back(0xFB000000u | i);
      for (auto &m : k.metas)
      {
        if (lng)
        {
          out.push_back(m.first << 24 | 0xFFFEu);
          out.push_back(0xFF000000u | at[m.second]);
        }
        else
          out.push_back(m.first << 24 | at[m.second]);
      }
      for (auto &r : k.runs)
      {
        if (r.target == 0)
          out.push_back(r.lo << 24 | r.hi << 16 | 0xFFFFu);
        else if (lng)
        {
          out.push_back(r.lo << 24 | r.hi << 16 | 0xFFFEu);
          out.push_back(0xFF000000u | at[r.target]);
        }
        else
          out.push_back(r.lo << 24 | r.hi << 16 | at[r.target]);
      }
    }
    return out;
  }
  fail(UGPU_UNSUPPORTED, "opcode table too large");
}

thread_local std::string g_compile_error;

}  // namespace

// Word ranges for option W (engine.hip: at_wb/at_we's iswword table,
// include/reflex/matcher.h:457-1192, the same Unicode 15.1 ranges as \w)
void ugpu_word_ranges(std::vector<uint32_t> &out)
{
  out.clear();
  for (auto &r : k_word_ranges)
  {
    out.push_back(r[0]);
    out.push_back(r[1]);
  }
}

// ---------------------------------------------------------------- assertion groups
//
// An alternative that begins with a group holding line anchors or word
// boundaries at the start of its own alternatives -- (^|,)foo, (\<|_)id --
// or ends with one holding them at their ends -- foo($|,) -- has those
// assertions at the ends of the match only, but inside a group, which the
// parser keeps for the per-context accepts of top-level alternatives.  Such a
// group is distributed over its alternative: (^|,)foo -> ^foo|,foo, every
// copy with the original alternative's accept index.  The reference's
// matches for both forms are the same (checked with its matcher on
// tests/golden/asgroup_cases.json, make_asgroup_golden.py).  Only plain
// groups "(" and "(?:" without a quantifier are distributed, at most 64
// alternatives; patterns with other "(?" constructs than a leading modifier
// or with \Q are left to the parser (its error stands).
namespace {

// the end of the token at i: an escape pair, a bracket expression, or a byte
size_t rx_token_end(const std::string &r, size_t i)
{
  if (r[i] == '\\')
    return i + 2 <= r.size() ? i + 2 : r.size();
  if (r[i] != '[')
    return i + 1;
  size_t j = i + 1;
  if (j < r.size() && r[j] == '^')
    ++j;
  if (j < r.size() && r[j] == ']')
    ++j;
  while (j < r.size() && r[j] != ']')
  {
    if (r[j] == '\\')
      j += 2;
    else if (r[j] == '[' && j + 1 < r.size() && (r[j + 1] == ':' || r[j + 1] == '.' || r[j + 1] == '='))
    {
      const size_t e = r.find(std::string(1, r[j + 1]) + "]", j + 2);
      j = e == std::string::npos ? r.size() : e + 2;
    }
    else
      ++j;
  }
  return j < r.size() ? j + 1 : r.size();
}

// the top-level alternatives of r (split at '|' outside groups and brackets);
// false when the parentheses do not balance
bool rx_split(const std::string &r, std::vector<std::string> &out)
{
  out.clear();
  int depth = 0;
  size_t from = 0;
  for (size_t i = 0; i < r.size(); i = rx_token_end(r, i))
  {
    if (r[i] == '(')
      ++depth;
    else if (r[i] == ')' && --depth < 0)
      return false;
    else if (r[i] == '|' && depth == 0)
    {
      out.push_back(r.substr(from, i - from));
      from = i + 1;
    }
  }
  out.push_back(r.substr(from));
  return depth == 0;
}

// the index of the ')' closing the '(' at i (npos: none)
size_t rx_close(const std::string &r, size_t i)
{
  int depth = 0;
  for (size_t j = i; j < r.size(); j = rx_token_end(r, j))
  {
    if (r[j] == '(')
      ++depth;
    else if (r[j] == ')' && --depth == 0)
      return j;
  }
  return std::string::npos;
}

bool rx_word_assertion_at(const std::string &r, size_t i)
{
  return i + 1 < r.size() && r[i] == '\\' && strchr("bB<>", r[i + 1]) != NULL;
}

bool rx_plain_group(const std::string &r, size_t i, size_t j, std::string &inner);
bool rx_split(const std::string &r, std::vector<std::string> &out);
size_t rx_close(const std::string &r, size_t i);

// a group's alternative begins with an assertion and has something after it,
// or with a plain group one of whose alternatives does
bool rx_lead_assert(const std::string &a)
{
  if (!a.empty() && a[0] == '^')
    return true;
  if (rx_word_assertion_at(a, 0))
    return a.size() > 2;
  if (a.empty() || a[0] != '(')
    return false;
  const size_t j = rx_close(a, 0);
  std::string inner;
  std::vector<std::string> parts;
  if (j == std::string::npos || !rx_plain_group(a, 0, j, inner) || !rx_split(inner, parts) ||
      (j + 1 < a.size() && strchr("*+?{", a[j + 1]) != NULL))
    return false;
  for (const std::string &x : parts)
    if (rx_lead_assert(x))
      return true;
  return false;
}

// a group's alternative ends with an assertion ($, or a word boundary after
// something), or with a plain group one of whose alternatives does
bool rx_tail_assert(const std::string &a)
{
  if (a.empty())
    return false;
  // (the last token: scan from the start, escapes decide; a group is one token)
  size_t last = std::string::npos;
  for (size_t i = 0; i < a.size();)
  {
    last = i;
    if (a[i] == '(')
    {
      const size_t j = rx_close(a, i);
      if (j == std::string::npos)
        return false;
      i = j + 1;
    }
    else
      i = rx_token_end(a, i);
  }
  if (a[last] == '$')
    return true;
  if (rx_word_assertion_at(a, last))
    return last > 0;
  if (a[last] != '(' || a.back() != ')')
    return false;
  std::string inner;
  std::vector<std::string> parts;
  if (!rx_plain_group(a, last, a.size() - 1, inner) || !rx_split(inner, parts))
    return false;
  for (const std::string &x : parts)
    if (rx_tail_assert(x))
      return true;
  return false;
}

// the contents of the plain group spanning [i, j] ("(" or "(?:"), or false
bool rx_plain_group(const std::string &r, size_t i, size_t j, std::string &inner)
{
  size_t b = i + 1;
  if (b < r.size() && r[b] == '?')
  {
    if (b + 1 < r.size() && r[b + 1] == ':')
      b += 2;
    else
      return false;
  }
  inner = r.substr(b, j - b);
  return true;
}

void rx_distribute(const std::string &a, std::vector<std::string> &out, size_t cap, bool &refuse)
{
  if (out.size() > cap || refuse)
    return;
  std::vector<std::string> parts;
  std::string inner;
  // a leading group with assertions at its alternatives' starts
  if (!a.empty() && a[0] == '(')
  {
    const size_t j = rx_close(a, 0);
    if (j != std::string::npos && rx_plain_group(a, 0, j, inner) &&
        (j + 1 >= a.size() || strchr("*+?{", a[j + 1]) == NULL) && rx_split(inner, parts))
    {
      bool any = false;
      for (const std::string &x : parts)
        any = any || rx_lead_assert(x);
      if (any)
      {
        for (const std::string &x : parts)
          rx_distribute(x + a.substr(j + 1), out, cap, refuse);
        return;
      }
    }
  }
  // a trailing group with assertions at its alternatives' ends
  if (!a.empty() && a.back() == ')')
  {
    // (the '(' whose group closes at the end)
    for (size_t i = 0; i < a.size(); i = rx_token_end(a, i))
    {
      if (a[i] != '(')
        continue;
      const size_t j = rx_close(a, i);
      if (j == a.size() - 1)
      {
        if (rx_plain_group(a, i, j, inner) && rx_split(inner, parts))
        {
          bool any = false;
          for (const std::string &x : parts)
            any = any || rx_tail_assert(x);
          if (any)
          {
            // ^...($|\s): the reference moves the begin anchor to the accept
            // side, where its EOL edge (which holds before "\r\n") ends the
            // match before a sibling that could consume the '\r' -- the
            // distributed form would take the longer match (measured on
            // (^|\s)foo(\s|$)); refused when a sibling is not a plain byte
            bool eol = false, other = false;
            for (const std::string &x : parts)
            {
              eol = eol || x == "$";
              other = other || (x != "$" && !x.empty() && strchr("\\[.(", x[0]) != NULL);
            }
            if (a[0] == '^' && eol && other)
            {
              refuse = true;
              return;
            }
            for (const std::string &x : parts)
              rx_distribute(a.substr(0, i) + x, out, cap, refuse);
            return;
          }
        }
        break;
      }
      if (j == std::string::npos)
        break;
      i = j;  // (skip the group: rx_token_end moves past its ')')
    }
  }
  out.push_back(a);
}

// r's top-level alternatives with their assertion groups distributed, and
// each one's accept index; false when nothing was distributed
bool rx_assertion_groups(const std::string &r, std::string &rewritten, std::vector<int> &accept)
{
  if (r.find("\\Q") != std::string::npos)
    return false;
  // a leading modifier (?imsx) applies to every alternative: kept in front
  size_t body = 0;
  if (r.size() > 2 && r[0] == '(' && r[1] == '?')
  {
    size_t k = 2;
    while (k < r.size() && isalpha(static_cast<unsigned char>(r[k])))
      ++k;
    if (k < r.size() && r[k] == ')' && k > 2)
      body = k + 1;
  }
  for (size_t q = r.find("(?", body); q != std::string::npos; q = r.find("(?", q + 1))
    if (r.compare(q, 3, "(?:") != 0)
      return false;
  std::vector<std::string> alts;
  if (!rx_split(r.substr(body), alts))
    return false;
  rewritten = r.substr(0, body);
  accept.clear();
  bool changed = false;
  for (size_t k = 0; k < alts.size(); ++k)
  {
    std::vector<std::string> out;
    bool refuse = false;
    rx_distribute(alts[k], out, 64, refuse);
    if (refuse || out.size() > 64 || accept.size() + out.size() > 64)
      return false;
    changed = changed || out.size() != 1 || out[0] != alts[k];
    for (const std::string &x : out)
    {
      rewritten += (accept.empty() ? "" : "|") + x;
      accept.push_back(static_cast<int>(k + 1));
    }
  }
  return changed;
}

// opcode words of rx; accept: the accept index of each top-level alternative
// (empty: 1, 2, ...)
std::vector<uint32_t> compile_words(const std::string &rx, uint32_t flags, const std::vector<int> &accept)
{
  Tree tree;
  Parser parser(rx, flags, tree);
  std::vector<int> alts = parser.parse_top();
  Glushkov g(tree);
  std::vector<int> start;
  for (size_t k = 0; k < alts.size(); ++k)
  {
    Glushkov::Info info = g.walk(alts[k]);
    int end = g.new_pos(ByteSet(), k < accept.size() ? accept[k] : static_cast<int>(k + 1));
    if (k < parser.metaseqs.size())
      g.metas[end] = parser.metaseqs[k];
    g.neg[end] = k < parser.negs.size() && parser.negs[k];
    g.link(info.last, std::vector<int>{end});
    Glushkov::merge(start, info.first);
    if (info.nullable)
      Glushkov::merge(start, std::vector<int>{end});
  }
  Dfa d = subsets(g, start);
  Dfa m = unfold_gaps(minimize(d, 1));
  return encode(m);
}

}  // namespace

extern "C" {

int ugpu_compile(const char *regex, size_t len, uint32_t flags, uint32_t **opc, uint32_t *nop)
{
  if (!opc || !nop || (!regex && len))
    return UGPU_INVAL;
  *opc = NULL;
  *nop = 0;
  try
  {
    std::string rx(regex ? regex : "", len);
    std::vector<uint32_t> words;
    try
    {
      words = compile_words(rx, flags, std::vector<int>());
    }
    catch (const CompileError &e)
    {
      // assertions inside a leading or trailing group: distributed over the
      // alternative (rx_assertion_groups), else the parser's error stands
      std::string r2;
      std::vector<int> accept;
      if (e.code != UGPU_UNSUPPORTED || (flags & UGPU_RX_FIXED) || !rx_assertion_groups(rx, r2, accept))
        throw;
      words = compile_words(r2, flags, accept);
    }
    uint32_t *buf = static_cast<uint32_t *>(malloc(words.size() * sizeof(uint32_t)));
    if (!buf)
      return UGPU_NOMEM;
    memcpy(buf, words.data(), words.size() * sizeof(uint32_t));
    *opc = buf;
    *nop = static_cast<uint32_t>(words.size());
    g_compile_error.clear();
    return UGPU_OK;
  }
  catch (const CompileError &e)
  {
    g_compile_error = e.msg;
    return e.code;
  }
  catch (const std::bad_alloc &)
  {
    g_compile_error = "out of memory";
    return UGPU_NOMEM;
  }
}

void ugpu_opc_free(uint32_t *opc)
{
  free(opc);
}

const char *ugpu_compile_error(void)
{
  return g_compile_error.c_str();
}

}  // extern "C"
