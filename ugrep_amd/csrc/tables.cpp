// tables.cpp -- RE/flex opcode words -> dense DFA tables (see tables.hpp).
//
// Opcode word format: include/reflex/pattern.h:1155-1247
//   goto  lo<<24 | hi<<16 | index16        (HALT index 0xFFFF, LONG index 0xFFFE
//                                            + next word 0xFF000000|index24)
//   halt  0x00FFFFFF
//   take  0xFE000000 | accept                (head of an accepting state block)
//   redo  0xFD000000, tail 0xFC.., head 0xFB.., meta gotos (hi byte 0)
// State block layout (lib/pattern.cpp:2943-3063): [REDO|TAKE]? TAIL* HEAD*
// then gotos in descending lo order; the interpreter takes the first goto whose
// [lo,hi] holds the byte (lib/matcher.cpp:467-502).
#include "tables.hpp"

#include <algorithm>
#include <cctype>
#include <map>
#include <set>
#include <unordered_map>

namespace ugpu {

namespace {

inline bool word_is_goto(uint32_t w) { return (uint32_t)(w << 8) >= (w & 0xff000000u); }
inline bool word_is_meta(uint32_t w) { return (w & 0x00ff0000u) == 0 && (w >> 24) > 0; }

constexpr uint32_t kHalt = 0xffff;
constexpr uint32_t kMaxLook = 4;  // lookahead indices the engine keeps per walk (tables.hpp look)
constexpr uint32_t kLong = 0xfffe;
constexpr int64_t kDead = -1;

struct RawState {
  uint32_t pc;
  uint32_t cap;
  int64_t target_pc[256];
  std::vector<std::pair<uint32_t, uint32_t> > metas;  // (META code - 0x100, target pc) in block order
  uint32_t look = 0;  // lookahead: TAIL la -> bit la, HEAD la -> bit 8 + la (tables.hpp look)
};

constexpr uint32_t kMetaBol = 0x09, kMetaEol = 0x0a;  // META_BOL / META_EOL - META_MIN (pattern.h:942-943)
// word boundaries (pattern.h:933-940): WBB WBE NWB NWE BWB EWB BWE EWE
constexpr uint32_t kMetaWordMin = 0x01, kMetaWordMax = 0x08;

// Whether meta edge `op` holds in context ctx (tables.hpp CTX_*), as the
// interpreter tests it after fetching the byte at the current position
// (lib/matcher.cpp:294-404; include/reflex/matcher.h:1281-1319 at_ewe ..
// at_wbb over at_wb/at_bw of the match begin and at_ew/at_we of the position).
bool meta_holds(uint32_t op, uint32_t ctx, bool word)
{
  if (!word) return op == kMetaBol ? (ctx & 2) != 0 : (ctx & 1) != 0;  // (line contexts: bit 1 bol, bit 0 eol)
  const bool eol = ctx & CTX_EOL, ew = ctx & CTX_EW, we = ctx & CTX_WE, bol = ctx & CTX_BOL, wb = ctx & CTX_WB,
             bw = ctx & CTX_BW;
  switch (op) {
    case 0x01: return bw == wb;    // META_WBB \b at begin: at_bw() == at_wb()
    case 0x02: return we == ew;    // META_WBE \b at end:   at_we() == at_ew()
    case 0x03: return bw != wb;    // META_NWB \B at begin
    case 0x04: return we != ew;    // META_NWE \B at end
    case 0x05: return bw && wb;    // META_BWB \< at begin
    case 0x06: return !bw && !wb;  // META_EWB \> at begin
    case 0x07: return !we && !ew;  // META_BWE \< at end
    case 0x08: return we && ew;    // META_EWE \> at end
    case kMetaBol: return bol;
    default: return eol;           // kMetaEol
  }
}

// Bucket approximation used by the GPU prefilter: the bytes whose 3-bit
// fields (lo3, mid3, hi2) each occur among the members' fields.
struct Bucket {
  uint8_t lo = 0, mid = 0, hi = 0;  // bitsets of field values
  void add(int b)
  {
    lo |= (uint8_t)(1u << (b & 7));
    mid |= (uint8_t)(1u << ((b >> 3) & 7));
    hi |= (uint8_t)(1u << (b >> 6));
  }
  bool has(int b) const { return (lo >> (b & 7) & 1) && (mid >> ((b >> 3) & 7) & 1) && (hi >> (b >> 6) & 1); }
  static Bucket all()
  {
    Bucket x;
    x.lo = x.mid = 0xff;
    x.hi = 0x0f;
    return x;
  }
  Bucket& operator|=(const Bucket& o)
  {
    lo |= o.lo;
    mid |= o.mid;
    hi |= o.hi;
    return *this;
  }
  // fraction of text bytes (printable ASCII and '\n') in the approximation
  double text_frac() const
  {
    int n = has('\n') ? 1 : 0;
    for (int b = 0x20; b < 0x7f; ++b) n += has(b) ? 1 : 0;
    return n / 96.0;
  }
};

// First bytes of a term group with the bytes that may follow them.
struct Lead {
  Bucket b, c, d;
  Lead& operator|=(const Lead& o)
  {
    b |= o.b;
    c |= o.c;
    d |= o.d;
    return *this;
  }
  double density() const { return b.text_frac() * c.text_frac() * d.text_frac(); }
};

// Partition the leads (one per first byte) into the two prefilter groups,
// minimising the summed candidate density of the group approximations:
// exhaustive up to 14 leads, greedy beyond.  Returns that density (<= 1).
double group_leads(const std::vector<Lead>& leads, Lead (&g)[2])
{
  g[0] = Lead();
  g[1] = Lead();
  const size_t n = leads.size();
  double best = 2.0;
  if (n <= 14) {
    const uint32_t lim = n ? 1u << (n - 1) : 1u;
    for (uint32_t m = 0; m < lim; ++m) {  // lead 0 always in group 0
      Lead x, y;
      for (size_t i = 0; i < n; ++i) ((i > 0 && (m >> (i - 1) & 1)) ? y : x) |= leads[i];
      const double c = x.density() + y.density();
      if (c < best) {
        best = c;
        g[0] = x;
        g[1] = y;
      }
    }
  } else {
    for (const Lead& l : leads) {
      Lead x = g[0], y = g[1];
      x |= l;
      y |= l;
      if (x.density() + g[1].density() <= g[0].density() + y.density())
        g[0] = x;
      else
        g[1] = y;
    }
    best = g[0].density() + g[1].density();
  }
  return n ? (best < 1.0 ? best : 1.0) : 0.0;
}

// The prefilter's byte tables (tables.hpp ft) from the two group leads: bit
// 2 s + k of T0[b & 7], T1[(b >> 3) & 7], T2[b >> 6] for group k's set s
void fill_ft(const Lead (&g)[2], uint8_t (&ft)[20])
{
  for (int k = 0; k < 2; ++k) {
    const Bucket* bk[3] = {&g[k].b, &g[k].c, &g[k].d};
    for (int s = 0; s < 3; ++s) {
      const uint8_t bit = (uint8_t)(1u << (2 * s + k));
      for (int v = 0; v < 8; ++v) {
        if (bk[s]->lo >> v & 1) ft[v] |= bit;
        if (bk[s]->mid >> v & 1) ft[8 + v] |= bit;
      }
      for (int v = 0; v < 4; ++v)
        if (bk[s]->hi >> v & 1) ft[16 + v] |= bit;
    }
  }
}

// Restart-locality (tables.hpp): breadth-first over the configurations a FIND
// walk can be in -- main walk state m, the live "shadow" walks the chain would
// start at every position after the current anchor (p+1, or the end of the
// last accept), and whether the next byte is the walk's first -- over one
// representative byte per column class.  The table is restart-local iff no
// shadow ever accepts while the main walk is alive and not accepting, and
// every shadow dies on the byte that kills the main walk.
bool restart_local(const std::vector<uint32_t>& nxt, uint32_t start, uint32_t first_acc,
                   const std::vector<int>& reps)
{
  typedef std::pair<std::pair<uint32_t, bool>, std::vector<uint32_t> > Cfg;
  std::set<Cfg> seen;
  std::vector<Cfg> work;
  work.push_back(Cfg(std::make_pair(start, true), std::vector<uint32_t>()));
  seen.insert(work.back());
  while (!work.empty()) {
    const Cfg cfg = work.back();
    work.pop_back();
    const uint32_t m = cfg.first.first;
    const bool first = cfg.first.second;
    for (int c : reps) {
      const uint32_t m2 = nxt[(size_t)m * 256 + c];
      std::vector<uint32_t> r2;
      for (uint32_t r : cfg.second) {
        const uint32_t t = nxt[(size_t)r * 256 + c];
        if (t) r2.push_back(t);
      }
      Cfg next;
      if (m2 == 0) {
        if (!r2.empty()) return false;  // a shadow walk outlives the main walk
        continue;
      } else if (m2 >= first_acc) {
        next = Cfg(std::make_pair(m2, false), std::vector<uint32_t>());  // shadows lie inside the match
      } else {
        for (uint32_t t : r2)
          if (t >= first_acc) return false;  // a match would start inside the walk
        if (!first) {
          const uint32_t t = nxt[(size_t)start * 256 + c];
          if (t >= first_acc) return false;
          if (t) r2.push_back(t);
        }
        std::sort(r2.begin(), r2.end());
        r2.erase(std::unique(r2.begin(), r2.end()), r2.end());
        next = Cfg(std::make_pair(m2, false), r2);
      }
      if (seen.insert(next).second) {
        if (seen.size() > 200000) return false;  // too many configurations: treat as not local
        work.push_back(next);
      }
    }
  }
  return true;
}

// Code-point run tables (tables.hpp xu_*).  Tokens are the strings that take
// the start state to its first accepting state; they must be single code
// points (ASCII x, or x >= 0xC0 followed by continuation bytes), which also
// makes the set prefix-free and the tokens non-overlapping.  The language is
// then S+ exactly when every state a a token ends in accepts, after one byte
// or more, the same strings as the start state (then a word of the language
// splits greedily into tokens, and the longest match at p is the longest run
// of consecutive tokens from p).
// DfaTables::dom.  For each state s, a lock-step walk of the pairs (a, b)
// reachable from (start, s) over one byte per column class: L(start) is not a
// subset of L(s) iff some reachable pair has a accepting and b not (the dead
// state 0 is the non-accepting sink; a pair with a dead is fine).  A search
// that finds no bad pair proves every pair it visited (the inclusion is
// closed under the successor relation), and those pairs are not searched
// again.  Bounded work: past the budget the remaining states stay unset (no
// skip, which is always safe).
void build_dom(const std::vector<uint32_t>& nxt, uint32_t S, uint32_t first_acc, uint32_t start_sid,
               const std::vector<int>& reps, std::vector<uint32_t>& dom)
{
  dom.assign((S + 31) / 32, 0u);
  if (S > 1024) {
    dom.clear();
    return;
  }
  std::vector<uint8_t> good((size_t)S * S, 0);
  std::vector<uint32_t> stamp((size_t)S * S, 0);
  std::vector<uint32_t> todo;
  uint64_t budget = 1ull << 25;  // pair x class steps over all states
  for (uint32_t s = 1; s < S && budget; ++s) {
    const uint32_t tag = s;
    bool bad = false;
    todo.clear();
    auto visit = [&](uint32_t a, uint32_t b) {
      if (a == 0) return;  // nothing accepted from the dead state
      const size_t k = (size_t)a * S + b;
      if (good[k] || stamp[k] == tag) return;
      if (b == 0 || (a >= first_acc && b < first_acc)) {
        bad = true;
        return;
      }
      stamp[k] = tag;
      todo.push_back((uint32_t)k);
    };
    visit(start_sid, s);
    for (size_t i = 0; i < todo.size() && !bad; ++i) {
      const uint32_t a = todo[i] / S, b = todo[i] % S;
      for (int c : reps) visit(nxt[(size_t)a * 256 + c], nxt[(size_t)b * 256 + c]);
      budget = budget > reps.size() ? budget - reps.size() : 0;
      if (!budget) bad = true;
    }
    if (bad) continue;
    for (uint32_t k : todo) good[k] = 1;
    dom[s >> 5] |= 1u << (s & 31);
  }
}

void build_xu(const std::vector<uint32_t>& nxt, uint32_t S, uint32_t first_acc, uint32_t start_sid, DfaTables& t)
{
  auto acc = [&](uint32_t s) { return s >= first_acc; };
  auto go = [&](uint32_t s, int c) { return nxt[(size_t)s * 256 + c]; };
  auto cont = [](int c) { return (c & 0xc0) == 0x80; };
  std::vector<uint8_t> tab(kXuTab, 0);
  std::vector<uint32_t> bm3(kXuBm3, 0);
  std::set<uint32_t> ends;  // states a token ends in
  std::map<uint32_t, int> s3_ok;  // states after 3 bytes of a 4-byte token: 1 = every continuation ends a token
  std::vector<std::pair<uint32_t, uint64_t> > l3;  // 3-byte leads (x << 8 | y) and their third-byte sets
  for (int x = 0; x < 256; ++x) {
    const uint32_t s1 = go(start_sid, x);
    if (!s1) continue;
    if (cont(x)) return;  // a token may not start with a continuation byte
    if (acc(s1)) {
      ends.insert(s1);
      if (x < 0x80)
        tab[x] = 0x01;
      else
        for (int y = 0; y < 256; ++y) tab[256 + (x & 63) * 256 + y] = 0x01;
      continue;
    }
    if (x < 0xc0) return;  // ASCII bytes are whole code points
    for (int y = 0; y < 256; ++y) {
      const uint32_t s2 = go(s1, y);
      if (!s2) continue;
      if (!cont(y)) return;
      uint8_t& e = tab[256 + (x & 63) * 256 + y];
      if (acc(s2)) {
        ends.insert(s2);
        e = 0x03;
        continue;
      }
      int nacc = 0, nlive = 0;
      uint64_t zset = 0;  // continuation bytes z completing a 3-byte token
      for (int z = 0; z < 256; ++z) {
        const uint32_t s3 = go(s2, z);
        if (!s3) continue;
        if (!cont(z)) return;
        if (acc(s3)) {
          ends.insert(s3);
          ++nacc;
          zset |= 1ull << (z & 63);
          continue;
        }
        ++nlive;
        auto it = s3_ok.find(s3);
        if (it == s3_ok.end()) {
          int ok = 1;
          for (int w = 0; w < 256 && ok; ++w) {
            const uint32_t s4 = go(s3, w);
            if (!s4) continue;
            if (!cont(w) || !acc(s4)) ok = 0;
            else ends.insert(s4);
          }
          it = s3_ok.emplace(s3, ok).first;
        }
        if (!it->second) return;
      }
      if (nacc && nlive) return;  // 3- and 4-byte tokens sharing two bytes: not UTF-8
      if (nlive) {
        e = XU_SLOW;
      } else if (nacc) {
        if (x < 0xe0 || x > 0xef) return;  // (the bitmap index assumes a 3-byte lead)
        e = XU_L3;
        l3.emplace_back((uint32_t)x << 8 | (uint32_t)y, zset);
      }
    }
  }
  // classes of continuation bytes: refine {all 64} by the third-byte sets of
  // the 3-byte leads while at most 3 classes result -- the blocks most frequent
  // in text first: General Punctuation (E2 80: quotes, dashes), then E2 82
  // (the euro sign's block), E2 81, then by code point; the leads whose set is
  // a union of classes get the class bits, the rest (XU_MIX) go to xu_bm3 and
  // make the fast U kernel hand the range to the exact one
  auto rank = [](uint32_t xy) { return xy == 0xe280 ? 0 : xy == 0xe282 ? 1 : xy == 0xe281 ? 2 : 3; };
  std::vector<std::pair<uint32_t, uint64_t> > order = l3;
  std::stable_sort(order.begin(), order.end(), [&](const std::pair<uint32_t, uint64_t>& a,
                                                   const std::pair<uint32_t, uint64_t>& b) {
    const int ra = rank(a.first), rb = rank(b.first);
    return ra != rb ? ra < rb : a.first < b.first;
  });
  std::vector<uint64_t> parts(1, ~0ull);
  for (const auto& l : order) {
    std::vector<uint64_t> np;
    for (uint64_t q : parts) {
      if (q & l.second) np.push_back(q & l.second);
      if (q & ~l.second) np.push_back(q & ~l.second);
    }
    if (np.size() <= 3) parts = np;
  }
  for (int z = 0x80; z < 0xc0; ++z)
    for (size_t k = 0; k < parts.size(); ++k)
      if (parts[k] >> (z & 63) & 1) tab[kXuCls + z] = (uint8_t)(0x10u << k);
  for (const auto& l : l3) {
    const int x = (int)(l.first >> 8), y = (int)(l.first & 0xff);
    uint8_t m = 0;
    uint64_t cover = 0;
    for (size_t k = 0; k < parts.size(); ++k)
      if ((parts[k] & l.second) == parts[k]) {
        m |= (uint8_t)(0x10u << k);
        cover |= parts[k];
      }
    if (cover == l.second) {
      tab[256 + (x & 63) * 256 + y] = (uint8_t)(XU_L3 | m);
    } else {
      tab[256 + (x & 63) * 256 + y] = XU_MIX;
      for (int z = 0x80; z < 0xc0; ++z)
        if (l.second >> (z & 63) & 1) {
          const uint32_t i = (uint32_t)(x & 15) << 12 | (uint32_t)(y & 63) << 6 | (uint32_t)(z & 63);
          bm3[i >> 5] |= 1u << (i & 31);
        }
    }
  }
  if (ends.empty()) return;
  // the fill byte for positions outside [lo, readable end): starts no token
  // and continues none
  int null = -1;
  for (int b = 255; b >= 0 && null < 0; --b)
    if (!cont(b) && !go(start_sid, b)) null = b;
  if (null < 0) return;
  // every token end behaves like the start state on non-empty strings
  for (uint32_t a : ends) {
    std::set<std::pair<uint32_t, uint32_t> > seen;
    std::vector<std::pair<uint32_t, uint32_t> > work;
    work.emplace_back(a, start_sid);
    while (!work.empty()) {
      const auto pq = work.back();
      work.pop_back();
      for (int c = 0; c < 256; ++c) {
        const uint32_t p = go(pq.first, c), q = go(pq.second, c);
        if (acc(p) != acc(q)) return;
        if ((p == 0) != (q == 0)) return;  // (minimised tables: a live state can accept)
        if (p && seen.insert(std::make_pair(p, q)).second) {
          if (seen.size() > 100000) return;
          work.emplace_back(p, q);
        }
      }
    }
  }
  (void)S;
  t.xu = true;
  t.xu_null = (uint8_t)null;
  tab[129] = (uint8_t)null;  // (an unused slot: exported with the table)
  t.xu_tab = std::move(tab);
  t.xu_bm3 = std::move(bm3);
}

}  // namespace

// Language equivalence with accept indices (tables.hpp): breadth-first over
// state pairs from the two start states; states that cannot reach an
// accepting state count as dead.
bool tables_equivalent(const DfaTables& a, const DfaTables& b)
{
  auto step = [](const DfaTables& t, uint32_t s, int c) {
    const size_t i = (size_t)s * t.row + (t.format == FMT_BYTE ? (uint32_t)c : t.cls[c]);
    return t.format == FMT_WIDE ? t.trans32[i] / t.row : (uint32_t)t.trans[i] / t.row;  // (wide: u32 entries)
  };
  auto live = [&](const DfaTables& t) {  // co-reachable states
    std::vector<std::vector<uint32_t> > rev(t.states);
    for (uint32_t s = 1; s < t.states; ++s)
      for (int c = 0; c < 256; ++c) {
        const uint32_t n = step(t, s, c);
        if (n) rev[n].push_back(s);
      }
    std::vector<bool> ok(t.states, false);
    std::vector<uint32_t> work;
    for (uint32_t s = 1; s < t.states; ++s)
      if (t.caps[s]) {
        ok[s] = true;
        work.push_back(s);
      }
    while (!work.empty()) {
      const uint32_t s = work.back();
      work.pop_back();
      for (uint32_t r : rev[s])
        if (!ok[r]) {
          ok[r] = true;
          work.push_back(r);
        }
    }
    return ok;
  };
  // the accept of state s in a 64-context (ctx_bits.hpp) of either layout
  auto acc = [](const DfaTables& t, uint32_t s, uint32_t ctx) -> uint32_t {
    if (t.ctx_word) return t.acap[(size_t)s * 64 + ctx];
    if (t.anchored) return t.acap[(size_t)s * 4 + ((ctx & CTX_BOL) ? 2 : 0) + ((ctx & CTX_EOL) ? 1 : 0)];
    return t.caps[s];
  };
  const std::vector<bool> la = live(a), lb = live(b);
  const uint32_t sa = a.start / a.row, sb = b.start / b.row;
  std::set<std::pair<uint32_t, uint32_t> > seen;
  std::vector<std::pair<uint32_t, uint32_t> > work;
  auto norm = [](const std::vector<bool>& l, uint32_t s) { return s && l[s] ? s : 0u; };
  const std::pair<uint32_t, uint32_t> p0(norm(la, sa), norm(lb, sb));
  work.push_back(p0);
  seen.insert(p0);
  while (!work.empty()) {
    const std::pair<uint32_t, uint32_t> p = work.back();
    work.pop_back();
    if ((p.first == 0) != (p.second == 0)) return false;
    if (p.first == 0) continue;
    if (a.anchored || b.anchored) {
      // (conditional accepts: caps is only a prefilter superset there)
      for (uint32_t ctx = 0; ctx < 64; ++ctx)
        if (acc(a, p.first, ctx) != acc(b, p.second, ctx)) return false;
    } else if (a.caps[p.first] != b.caps[p.second]) {
      return false;
    }
    // (lookahead: the same TAIL/HEAD words in both states)
    if ((a.lookahead ? a.look[p.first] : 0u) != (b.lookahead ? b.look[p.second] : 0u)) return false;
    for (int c = 0; c < 256; ++c) {
      const std::pair<uint32_t, uint32_t> q(norm(la, step(a, p.first, c)), norm(lb, step(b, p.second, c)));
      if (seen.insert(q).second) work.push_back(q);
    }
  }
  return true;
}

int build_tables(const uint32_t* opc, uint32_t nop, DfaTables& out, std::string& err)
{
  if (opc == nullptr || nop == 0) {
    err = "empty opcode table";
    return 2;
  }
  std::vector<RawState> raw;
  std::unordered_map<uint32_t, uint32_t> index_of_pc;  // pc -> raw index
  raw.reserve(64);
  raw.push_back(RawState{0, 0, {}, {}});
  index_of_pc[0] = 0;
  for (size_t qi = 0; qi < raw.size(); ++qi) {
    uint32_t pc = raw[qi].pc;
    uint32_t k = pc;
    uint32_t cap = 0;
    // block header: TAKE, then meta edges (no goto words: the interpreter
    // tests them in block order before the byte edges, lib/matcher.cpp:193-450)
    while (k < nop && !word_is_goto(opc[k])) {
      const uint32_t w = opc[k], op = w >> 24;
      if (op == 0xfe) {
        cap = w & 0xffffff;
      } else if (w == 0xFD000000u) {
        cap = kCapRedo;  // REDO (lib/pattern.cpp:2945-2947): a negative pattern's accept
      } else if ((op == 0xfc || op == 0xfb) && (w & 0xffffff) < kMaxLook) {
        // TAIL / HEAD la (lib/pattern.cpp:2953-2964; lookahead_of = the low 16 bits)
        raw[qi].look |= (op == 0xfc ? 1u : 0x100u) << (w & 0xffff);
      } else if (op == 0xfc || op == 0xfb) {
        err = "more lookaheads than the engine keeps";
        return 1;
      } else if (word_is_meta(w)) {
        const uint32_t idx = w & 0xffff;
        if (op != kMetaBol && op != kMetaEol && !(op >= kMetaWordMin && op <= kMetaWordMax)) {
          err = "opcode table uses meta edges other than ^, $ and word boundaries (\\A, \\Z, indent)";
          return 1;
        }
        uint64_t t = idx;
        if (idx == kLong) {
          if (k + 1 >= nop) {
            err = "LONG meta goto without index word";
            return 2;
          }
          t = opc[k + 1] & 0xffffff;
          ++k;
        }
        if (idx == kHalt || t >= nop) {
          err = "meta goto target out of range";
          return 2;
        }
        raw[qi].metas.emplace_back(op, (uint32_t)t);
        if (index_of_pc.find((uint32_t)t) == index_of_pc.end()) {
          index_of_pc[(uint32_t)t] = (uint32_t)raw.size();
          raw.push_back(RawState{(uint32_t)t, 0, {}, {}});
        }
      } else {
        err = "opcode table uses indent words";
        return 1;
      }
      ++k;
    }
    int64_t tgt[256];
    bool have[256];
    std::fill(have, have + 256, false);
    int remaining = 256;
    while (remaining > 0) {
      if (k >= nop) {
        err = "state block runs past the end of the opcode table";
        return 2;
      }
      uint32_t w = opc[k];
      if (!word_is_goto(w)) {
        err = "state block does not cover every byte";
        return 2;
      }
      if (word_is_meta(w)) {
        err = "meta edge after a byte edge";
        return 1;
      }
      uint32_t lo = w >> 24, hi = (w >> 16) & 0xff, idx = w & 0xffff;
      int64_t t;
      if (idx == kHalt) {
        t = kDead;
      } else if (idx == kLong) {
        if (k + 1 >= nop) {
          err = "LONG goto without index word";
          return 2;
        }
        t = opc[k + 1] & 0xffffff;
      } else {
        t = idx;
      }
      if (t != kDead && (uint64_t)t >= nop) {
        err = "goto target out of range";
        return 2;
      }
      for (uint32_t c = lo; c <= hi; ++c)
        if (!have[c]) {
          have[c] = true;
          tgt[c] = t;
          --remaining;
        }
      k += (idx == kLong) ? 2 : 1;
    }
    for (int c = 0; c < 256; ++c) {
      int64_t t = tgt[c];
      if (t != kDead && index_of_pc.find((uint32_t)t) == index_of_pc.end()) {
        index_of_pc[(uint32_t)t] = (uint32_t)raw.size();
        raw.push_back(RawState{(uint32_t)t, 0, {}, {}});
      }
    }
    raw[qi].cap = cap;
    std::copy(tgt, tgt + 256, raw[qi].target_pc);
  }

  // acceptance per (bol, eol) context: the reference's meta evaluation at a
  // state (lib/matcher.cpp:193-450): its own TAKE, then the first meta edge
  // that holds, that target's TAKE, its first meta edge that holds, ... (at
  // most 5 meta jumps); a meta target that goes on with byte edges is not
  // supported (the reference would continue that walk from the same byte)
  // (word boundaries: 64 contexts, tables.hpp CTX_*; line anchors only: 4)
  const uint32_t n = (uint32_t)raw.size();
  bool anchored = false, word = false, redo = false;
  for (uint32_t i = 0; i < n; ++i) {
    anchored = anchored || !raw[i].metas.empty();
    redo = redo || raw[i].cap == kCapRedo;
    for (const auto& m : raw[i].metas) word = word || (m.first >= kMetaWordMin && m.first <= kMetaWordMax);
  }
  if (redo && anchored) {
    err = "REDO (a negative pattern) in a table with anchors or word boundaries";
    return 1;
  }
  bool look = false;
  for (uint32_t i = 0; i < n; ++i) look = look || raw[i].look != 0;
  if (look && (anchored || redo)) {
    err = "lookahead in a table with anchors, word boundaries or REDO";
    return 1;
  }
  if (look) {
    // a HEAD la in the start state with a TAIL la anywhere: the TAIL can move
    // the match end back to the walk's start, an empty match, and the
    // reference then asks its advance function for the next candidate and
    // ends the FIND when it has none (lib/matcher.cpp:682-707) -- behaviour
    // of the Pattern's prediction, not of the table (a*(?=b), (?=x))
    uint32_t tails = 0;
    for (uint32_t i = 0; i < n; ++i) tails |= raw[i].look & 0xffu;
    if ((raw[0].look >> 8) & tails) {
      err = "lookahead after a prefix that can be empty (empty matches)";
      return 1;
    }
  }
  const uint32_t nctx = word ? 64u : 4u;
  std::vector<uint32_t> acc4((size_t)n * nctx, 0);
  for (uint32_t i = 0; i < n; ++i) {
    for (uint32_t ctx = 0; ctx < nctx; ++ctx) {
      uint32_t cap = raw[i].cap, cur = i;
      for (int jumps = 0; jumps < 5; ++jumps) {
        uint32_t to = ~0u;
        for (const auto& m : raw[cur].metas)
          if (meta_holds(m.first, ctx, word)) {
            to = index_of_pc[m.second];
            break;
          }
        if (to == ~0u) break;
        for (int c = 0; c < 256; ++c)
          if (raw[to].target_pc[c] != kDead) {
            err = "a meta edge's target state goes on with byte edges";
            return 1;
          }
        if (raw[to].cap) cap = raw[to].cap;
        cur = to;
      }
      acc4[(size_t)i * nctx + ctx] = cap;
    }
  }
  auto accepts = [&](uint32_t i) {
    uint32_t a = 0;
    for (uint32_t ctx = 0; ctx < nctx; ++ctx) a |= acc4[(size_t)i * nctx + ctx];
    return a;
  };
  // renumber: dead = 0, non-accepting states, then accepting states (for an
  // anchored table: accepting in some context)
  std::vector<uint32_t> sid(n);
  uint32_t next_id = 1;
  for (uint32_t i = 0; i < n; ++i)
    if (!accepts(i)) sid[i] = next_id++;
  const uint32_t first_acc = next_id;
  for (uint32_t i = 0; i < n; ++i)
    if (accepts(i)) sid[i] = next_id++;
  const uint32_t S = next_id;

  // dense next[sid][byte] in new ids
  std::vector<uint32_t> nxt((size_t)S * 256, 0);
  std::vector<uint32_t> caps(S, 0), acap((size_t)S * nctx, 0), lookv(look ? S : 0, 0);
  for (uint32_t i = 0; i < n; ++i) {
    caps[sid[i]] = raw[i].cap;
    if (look) lookv[sid[i]] = raw[i].look;
    for (uint32_t ctx = 0; ctx < nctx; ++ctx) acap[(size_t)sid[i] * nctx + ctx] = acc4[(size_t)i * nctx + ctx];
    if (anchored && !raw[i].cap) {  // (caps: the state's accept in some context, for the prefilter's superset)
      for (uint32_t ctx = 0; ctx < nctx && !caps[sid[i]]; ++ctx) caps[sid[i]] = acc4[(size_t)i * nctx + ctx];
    }
    for (int c = 0; c < 256; ++c) {
      int64_t t = raw[i].target_pc[c];
      nxt[(size_t)sid[i] * 256 + c] = (t == kDead) ? 0 : sid[index_of_pc[(uint32_t)t]];
    }
  }

  // byte equivalence classes (identical columns over all states)
  std::map<std::vector<uint32_t>, uint32_t> colmap;
  std::vector<uint8_t> cls(256);
  for (int c = 0; c < 256; ++c) {
    std::vector<uint32_t> col(S);
    for (uint32_t s = 0; s < S; ++s) col[s] = nxt[(size_t)s * 256 + c];
    auto it = colmap.find(col);
    if (it == colmap.end()) it = colmap.emplace(col, (uint32_t)colmap.size()).first;
    cls[c] = (uint8_t)it->second;
  }
  const uint32_t C = (uint32_t)colmap.size();

  DfaTables t;
  t.states = S;
  t.classes = C;
  if ((uint64_t)S * 256 <= 65536) {
    t.format = FMT_BYTE;
    t.row = 256;
    t.log_row = 8;
  } else {
    uint32_t r = 1, lr = 0;
    while (r < C) {
      r <<= 1;
      ++lr;
    }
    if ((uint64_t)S * r > (1ull << 26)) {
      err = "DFA too large (more than 2^26 table entries)";
      return 1;
    }
    t.format = (uint64_t)S * r > 65536 ? FMT_WIDE : FMT_CLASS;
    t.row = r;
    t.log_row = lr;
  }
  const uint32_t R = t.row;
  if (t.format == FMT_WIDE) {
    t.cls = cls;
    t.trans32.assign((size_t)S * R, 0);
    for (uint32_t s = 0; s < S; ++s)
      for (int c = 0; c < 256; ++c) t.trans32[(size_t)s * R + cls[c]] = nxt[(size_t)s * 256 + c] * R;
  } else {
  t.trans.assign((size_t)S * R, 0);
  if (t.format == FMT_BYTE) {
    for (uint32_t s = 0; s < S; ++s)
      for (int c = 0; c < 256; ++c) t.trans[(size_t)s * R + c] = (uint16_t)(nxt[(size_t)s * 256 + c] * R);
    for (int c = 0; c < 256; ++c) t.cls.push_back((uint8_t)c);
  } else {
    t.cls = cls;
    for (uint32_t s = 0; s < S; ++s)
      for (int c = 0; c < 256; ++c) t.trans[(size_t)s * R + cls[c]] = (uint16_t)(nxt[(size_t)s * 256 + c] * R);
  }
  }
  t.caps = caps;
  t.look = lookv;
  t.lookahead = look;
  t.acap = acap;
  t.anchored = anchored;
  t.ctx_word = word;
  if (word) {
    std::map<std::vector<uint32_t>, uint32_t> rows;
    rows.emplace(std::vector<uint32_t>(64, 0), 0u);
    t.acap_rows.assign(64, 0);
    t.acap_map.assign(S, 0);
    for (uint32_t s = 0; s < S; ++s) {
      std::vector<uint32_t> r(acap.begin() + (size_t)s * 64, acap.begin() + (size_t)(s + 1) * 64);
      auto it = rows.find(r);
      if (it == rows.end()) {
        it = rows.emplace(r, (uint32_t)rows.size()).first;
        t.acap_rows.insert(t.acap_rows.end(), r.begin(), r.end());
      }
      t.acap_map[s] = it->second;
    }
  }
  // shape (ugpu_dfa_info.shape): a finite language (no cycle reachable from
  // the start), and word-context accepts in states that also go on with bytes
  {
    std::vector<uint8_t> color(S, 0);  // 0 new, 1 on the path, 2 done
    std::vector<std::pair<uint32_t, int>> stack;
    bool cycle = false;
    stack.emplace_back(sid[0], 0);
    color[sid[0]] = 1;
    while (!stack.empty() && !cycle) {
      auto& top = stack.back();
      if (top.second == 256) {
        color[top.first] = 2;
        stack.pop_back();
        continue;
      }
      const uint32_t v = nxt[(size_t)top.first * 256 + top.second++];
      if (v == 0) continue;
      if (color[v] == 1) cycle = true;
      else if (color[v] == 0) {
        color[v] = 1;
        stack.emplace_back(v, 0);
      }
    }
    t.finite = !cycle;
    t.word_cond_edges = false;
    if (word)
      for (uint32_t s = 1; s < S && !t.word_cond_edges; ++s) {
        bool uniform = true, edges = false;
        for (uint32_t ctx = 1; ctx < nctx; ++ctx) uniform = uniform && acap[(size_t)s * nctx + ctx] == acap[(size_t)s * nctx];
        for (int c = 0; c < 256 && !edges; ++c) edges = nxt[(size_t)s * 256 + c] != 0;
        t.word_cond_edges = !uniform && edges;
      }
  }
  const uint32_t start_sid = sid[0];
  t.start_acc = start_sid >= first_acc;
  // FIND transducer for restart-local tables (tables.hpp); none of the
  // transducer forms below holds for conditional acceptance (anchored tables)
  const bool wide = t.format == FMT_WIDE;
  if (R >= 4 && !anchored && !wide) {
    std::vector<int> reps;  // one byte per column class
    {
      std::vector<bool> seen_cls(256, false);
      for (int c = 0; c < 256; ++c)
        if (!seen_cls[cls[c]]) {
          seen_cls[cls[c]] = true;
          reps.push_back(c);
        }
    }
    if (restart_local(nxt, start_sid, first_acc, reps)) {
      t.restart_local = true;
      t.xtrans.assign((size_t)S * R, 0);
      for (uint32_t s = 0; s < S; ++s)
        for (int c : reps) {
          const uint32_t col = t.format == FMT_BYTE ? (uint32_t)c : cls[c];
          const uint32_t nx = nxt[(size_t)s * 256 + c], r = nxt[(size_t)start_sid * 256 + c];
          uint32_t x;
          if (nx)
            x = nx * R;
          else
            x = (r ? r : start_sid) * R | XT_DEAD | (r ? XT_LIVE : 0);
          if (t.format == FMT_BYTE) {
            for (int b = 0; b < 256; ++b)  // every byte of the class
              if (cls[b] == cls[c]) t.xtrans[(size_t)s * R + b] = (uint16_t)x;
          } else {
            t.xtrans[(size_t)s * R + col] = (uint16_t)x;
          }
        }
    }
  }
  // dominated restarts (tables.hpp dom) for the plain walks
  if (!anchored && !word && !look) {
    std::vector<int> reps;
    std::vector<bool> seen_cls(256, false);
    for (int c = 0; c < 256; ++c)
      if (!seen_cls[cls[c]]) {
        seen_cls[cls[c]] = true;
        reps.push_back(c);
      }
    build_dom(nxt, S, first_acc, start_sid, reps, t.dom);
    if (!t.dom.empty()) {
      std::vector<bool> seen(S, false);
      std::vector<uint32_t> order{start_sid};
      seen[start_sid] = true;
      t.dom_all = true;
      for (size_t i = 0; i < order.size() && t.dom_all; ++i) {
        const uint32_t a = order[i];
        if (a != start_sid && a < first_acc && !((t.dom[a >> 5] >> (a & 31)) & 1u)) t.dom_all = false;
        for (int c : reps) {
          const uint32_t n = nxt[(size_t)a * 256 + c];
          if (n && !seen[n]) {
            seen[n] = true;
            order.push_back(n);
          }
        }
      }
    }
  }
  // immediate transducer (tables.hpp, xi_kernel.hip)
  if (t.restart_local && start_sid < first_acc) {
    std::vector<int> sig(S, -1);  // walk states reachable from start -> sigma
    std::vector<uint32_t> order;
    sig[start_sid] = 0;
    order.push_back(start_sid);
    bool ok = true;
    for (size_t i = 0; i < order.size() && ok; ++i)
      for (int c = 0; c < 256 && ok; ++c) {
        const uint32_t n = nxt[(size_t)order[i] * 256 + c];
        if (n == 0) continue;
        if (n == start_sid || n < first_acc) ok = false;  // re-enters start, or a walk state that does not accept
        if (ok && sig[n] < 0) {
          sig[n] = (int)order.size();
          order.push_back(n);
        }
      }
    std::vector<bool> sync(256, false);
    int first_sync = -1;
    for (int c = 0; ok && c < 256; ++c) {
      bool y = nxt[(size_t)start_sid * 256 + c] == 0;
      for (size_t i = 1; i < order.size() && y; ++i) y = nxt[(size_t)order[i] * 256 + c] == 0;
      sync[c] = y;
      if (y && first_sync < 0) first_sync = c;
    }
    // sync bytes must be common in text (a space or a newline among them):
    // with only rare ones (\D: digits) lane tails serialise over long runs,
    // and dense_kernel's speculative walk is the better choice
    if (ok && order.size() <= 32 && first_sync >= 0 && (sync[' '] || sync['\n'])) {
      t.immediate = true;
      t.sync_byte = (uint8_t)first_sync;
      t.xid_rows = (uint32_t)order.size() * 8;
      t.xid.assign((size_t)t.xid_rows * 256, 0);
      for (uint32_t id = 0; id < t.xid_rows; ++id) {
        const uint32_t sg = id >> 3, s = order[sg];
        for (int c = 0; c < 256; ++c) {
          const uint32_t nx = nxt[(size_t)s * 256 + c];
          uint32_t to = 0, st = 0;
          if (nx) {
            to = (uint32_t)sig[nx];
            st = sg == 0 ? 1u : 0u;  // leaving start begins a match
          } else {
            const uint32_t r = nxt[(size_t)start_sid * 256 + c];  // the walk dies (or none runs): restart here
            if (r) {
              to = (uint32_t)sig[r];
              st = 1;
            }
          }
          t.xid[(size_t)id * 256 + c] =
              (uint8_t)(to << 3 | (sync[c] ? XI_Y : 0u) | (to ? XI_IN : 0u) | (st ? XI_ST : 0u));
        }
      }
    }
  }
  // gap transducer (tables.hpp, xg_kernel.hip)
  if (t.restart_local && R >= 64 && start_sid < first_acc) {
    std::vector<int> gap(S, -1);
    std::vector<std::pair<uint32_t, int> > work;  // (state, gap) pairs, BFS over walks from start
    std::set<std::pair<uint32_t, int> > seen;
    work.push_back(std::make_pair(start_sid, 0));
    seen.insert(work.back());
    bool ok = true;
    while (!work.empty() && ok) {
      const std::pair<uint32_t, int> cur = work.back();
      work.pop_back();
      if (gap[cur.first] >= 0 && gap[cur.first] != cur.second) ok = false;
      gap[cur.first] = cur.second;
      for (int c = 0; c < 256 && ok; ++c) {
        const uint32_t n = nxt[(size_t)cur.first * 256 + c];
        if (n == 0) continue;
        const std::pair<uint32_t, int> nx(n, n >= first_acc ? 0 : cur.second + 1);
        if (nx.second > 6) ok = false;
        if (seen.insert(nx).second) work.push_back(nx);
      }
    }
    std::vector<uint8_t> sync(256, 0);
    bool any_sync = false;
    for (int c = 0; ok && c < 256; ++c) {
      bool y = nxt[(size_t)start_sid * 256 + c] == 0;
      for (uint32_t s2 = 1; s2 < S && y; ++s2)
        if (gap[s2] >= 0 && s2 != start_sid) y = nxt[(size_t)s2 * 256 + c] == 0;
      sync[c] = y ? 1 : 0;
      any_sync |= y;
    }
    if (ok && any_sync && (sync[' '] || sync['\n'])) {  // common sync bytes (see above)
      t.gap = true;
      t.xg_sync = sync;
      t.xg.assign((size_t)S * R, 0);
      for (uint32_t s2 = 0; s2 < S; ++s2)
        for (int c = 0; c < 256; ++c) {
          const uint32_t col = t.format == FMT_BYTE ? (uint32_t)c : cls[c];
          const uint32_t nx = nxt[(size_t)s2 * 256 + c], r = nxt[(size_t)start_sid * 256 + c];
          uint32_t x;
          if (nx) {
            x = nx * R;
            if (nx >= first_acc) x |= XG_A | (uint32_t)((gap[s2] < 0 ? 0 : gap[s2]) + 1) << XG_LSHIFT;
          } else {
            x = (r ? r : start_sid) * R | XT_DEAD | (r ? XT_LIVE : 0);
            if (r && r >= first_acc) x |= XG_A | 1u << XG_LSHIFT;
          }
          t.xg[(size_t)s2 * R + col] = (uint16_t)x;
        }
      // device form: product states (s, accepted) by BFS from (start, 0)
      std::map<std::pair<uint32_t, int>, uint32_t> pid;
      std::vector<std::pair<uint32_t, int> > pst;
      auto prod = [&](uint32_t s2, int a) {
        auto it = pid.find(std::make_pair(s2, a));
        if (it != pid.end()) return it->second;
        const uint32_t id = (uint32_t)pst.size();
        pid.emplace(std::make_pair(s2, a), id);
        pst.push_back(std::make_pair(s2, a));
        return id;
      };
      std::vector<int> rep(C, -1);
      for (int c = 0; c < 256; ++c)
        if (rep[cls[c]] < 0) rep[cls[c]] = c;
      prod(start_sid, 0);
      std::vector<std::vector<uint16_t> > rows;  // per product state: entry per column
      for (size_t i = 0; i < pst.size() && pst.size() <= kXg2MaxStates; ++i) {
        const uint32_t s2 = pst[i].first;
        const int a = pst[i].second;
        std::vector<uint16_t> row(C, 0);
        for (uint32_t col = 0; col < C; ++col) {
          const int c = rep[col];
          const uint32_t nx = nxt[(size_t)s2 * 256 + c], r = nxt[(size_t)start_sid * 256 + c];
          uint32_t to, L = 0, F = 0, D = 0;
          if (nx) {
            int a2 = a;
            if (nx >= first_acc) {
              L = (uint32_t)(gap[s2] < 0 ? 0 : gap[s2]) + 1;
              F = a ? 0u : 1u;
              a2 = 1;
            }
            to = prod(nx, a2);
          } else {
            D = 1;
            if (r && r >= first_acc) {
              L = 1;
              F = 1;
              to = prod(r, 1);
            } else {
              to = prod(r ? r : start_sid, 0);
            }
          }
          row[col] = (uint16_t)((2 * to) << XG2_ROWSHIFT | D * XG2_D | F * XG2_F | L);
        }
        rows.push_back(row);
      }
      uint32_t pad = (uint32_t)pst.size();
      while (pad % 4 != 2) ++pad;
      // (the kernel stages the table plus 512 B of byte tables in 160 KB of LDS)
      if (pst.size() <= kXg2MaxStates && ((uint64_t)C * pad + 7) / 8 * 16 <= 160u * 1024 - 1536) {
        t.xg2_states = (uint32_t)pst.size();
        t.xg2_cols = C;
        t.xg2_pad = pad;
        t.xg2.assign((size_t)C * pad, 0);
        for (uint32_t p2 = 0; p2 < t.xg2_states; ++p2)
          for (uint32_t col = 0; col < C; ++col) t.xg2[(size_t)col * pad + p2] = rows[p2][col];
        t.xg2_cls = cls;
      } else {
        t.gap = false;  // (product table too large: dense_kernel serves it)
      }
    }
  }
  // two-state tables (tables.hpp XcProg, xc_kernel.hip): start --G--> A,
  // A --X--> A, G a subset of X, both sets inside ASCII
  if (start_sid < first_acc && !anchored && !wide) {
    uint32_t A = 0;
    bool ok = true;
    for (int c = 0; c < 256 && ok; ++c) {
      const uint32_t nx = nxt[(size_t)start_sid * 256 + c];
      if (nx && A == 0) A = nx;
      if (nx && nx != A) ok = false;
    }
    ok = ok && A >= first_acc;
    bool G[256], X[256];
    for (int c = 0; c < 256 && ok; ++c) {
      const uint32_t nx = nxt[(size_t)A * 256 + c];
      if (nx && nx != A) ok = false;
      G[c] = nxt[(size_t)start_sid * 256 + c] == A;
      X[c] = nx == A;
      if (G[c] && !X[c]) ok = false;
    }
    if (ok) {
      t.xc = true;
      t.xc_tab.assign(256, 0);
      for (int c = 0; c < 256; ++c) t.xc_tab[c] = (uint8_t)((G[c] ? 0x80 : 0) | (X[c] ? 0x40 : 0));
      bool wordset = true;  // X = the ASCII word bytes [0-9A-Za-z_] (option W on xc_kernel)
      bool wordsub = true;  // X inside them ([A-Za-z]+, [0-9]+, [a-z_]+ ...)
      auto aword = [](int c) { return c < 0x80 && (std::isalnum(c) || c == '_'); };
      for (int c = 0; c < 256; ++c) {
        wordset = wordset && X[c] == aword(c);
        wordsub = wordsub && (!X[c] || aword(c));
      }
      t.xc_w = wordset;
      t.xc_wsub = wordsub && !wordset;
      if (t.xc_wsub)  // (bit 5: an ASCII word byte, for option W's subset mode)
        for (int c = 0; c < 256; ++c)
          if (aword(c)) t.xc_tab[c] |= 0x20;
    }
  }
  t.start = start_sid * R;
  t.accepting = S - first_acc;
  t.accb = (t.accepting > 0) ? first_acc * R : (wide ? 0xFFFFFFFFu : 0x10000u);
  for (uint32_t s = first_acc; s < S; ++s) {
    if (s == first_acc)
      t.cap1 = caps[s];
    else if (caps[s] != t.cap1)
      t.cap1 = 0;
  }
  if (anchored) t.cap1 = 0;  // (conditional accepts: the accept index comes from acap)
  // (REDO: the matches that end in it are not reported, which the one-index
  // kernels -- transducers, carry chains, code-point runs -- do not model)
  t.redo = redo;
  if (redo) t.cap1 = 0;
  if (!t.xc && !wide && t.cap1 != 0 && start_sid < first_acc) build_xu(nxt, S, first_acc, start_sid, t);
  // prefilter (see tables.hpp): per first byte c, the bytes that can follow
  // it (second) and follow those (third); "all" once a prefix accepts
  std::vector<Lead> leads;
  for (int c = 0; c < 256; ++c) {
    const uint32_t s1 = nxt[(size_t)start_sid * 256 + c];
    if (s1 == 0) continue;
    Lead l;
    l.b.add(c);
    if (s1 >= first_acc) {  // 1-byte match: no follow-up test
      l.c = Bucket::all();
      l.d = Bucket::all();
      leads.push_back(l);
      continue;
    }
    bool short2 = false;
    for (int d = 0; d < 256; ++d) {
      const uint32_t s2 = nxt[(size_t)s1 * 256 + d];
      if (s2 == 0) continue;
      l.c.add(d);
      if (s2 >= first_acc) short2 = true;
      for (int e = 0; e < 256; ++e)
        if (nxt[(size_t)s2 * 256 + e] != 0) l.d.add(e);
    }
    if (short2) l.d = Bucket::all();  // a match may end after 2 bytes
    leads.push_back(l);
  }
  t.first_bytes = (uint32_t)leads.size();
  Lead g[2];
  t.fdensity = group_leads(leads, g);
  fill_ft(g, t.ft);
  // the sparse kernel pays off when few positions survive the prefilter
  // (a start state that accepts: empty matches anywhere, no candidate filter)
  t.filter = t.format == FMT_BYTE && !leads.empty() && t.fdensity <= 0.15 && start_sid < first_acc;
  if (look) {
    // lookahead tables: a match end can move back to a HEAD position, which
    // none of the transducer forms or the candidate walks model; they take the
    // lookahead walk (device_common.hpp kWalkLook) on wfind_kernel
    t.filter = false;
    t.restart_local = false;
    t.xtrans.clear();
    t.immediate = false;
    t.xid.clear();
    t.gap = false;
    t.xc = false;
    t.xu = false;
  }
  out = std::move(t);
  return 0;
}

// Loop-needle tables (host_api.cpp loop_needle): the prefilter looks for the
// strings of N -- one lead per string (its first three bytes, any byte past
// its end), grouped as the first-byte leads are.  Returns the estimated
// candidate density.
double needle_filter(const std::vector<std::string>& needles, uint8_t (&ft)[20])
{
  std::vector<Lead> leads;
  for (const std::string& n : needles) {
    Lead l;
    Bucket* bk[3] = {&l.b, &l.c, &l.d};
    for (size_t s = 0; s < 3; ++s)
      if (s < n.size())
        bk[s]->add((unsigned char)n[s]);
      else
        *bk[s] = Bucket::all();
    leads.push_back(l);
  }
  Lead g[2];
  const double d = group_leads(leads, g);
  for (int i = 0; i < 20; ++i) ft[i] = 0;
  fill_ft(g, ft);
  return d;
}

}  // namespace ugpu
