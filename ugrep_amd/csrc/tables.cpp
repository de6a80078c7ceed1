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
#include <map>
#include <unordered_map>

namespace ugpu {

namespace {

inline bool word_is_goto(uint32_t w) { return (uint32_t)(w << 8) >= (w & 0xff000000u); }
inline bool word_is_meta(uint32_t w) { return (w & 0x00ff0000u) == 0 && (w >> 24) > 0; }

constexpr uint32_t kHalt = 0xffff;
constexpr uint32_t kLong = 0xfffe;
constexpr int64_t kDead = -1;

struct RawState {
  uint32_t pc;
  uint32_t cap;
  int64_t target_pc[256];
};

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
};

// Split a byte set over two buckets minimising the union of their
// approximations (exhaustive for small sets, greedy otherwise).
void split_set(const bool in[256], Bucket& b1, Bucket& b2)
{
  std::vector<int> mem;
  for (int b = 0; b < 256; ++b)
    if (in[b]) mem.push_back(b);
  b1 = Bucket();
  b2 = Bucket();
  if (mem.empty()) return;
  auto cost = [](const Bucket& x, const Bucket& y) {
    int n = 0;
    for (int b = 0; b < 256; ++b) n += (x.has(b) || y.has(b)) ? 1 : 0;
    return n;
  };
  if (mem.size() <= 12) {
    int best = 1 << 30;
    const uint32_t lim = 1u << (mem.size() - 1);
    for (uint32_t m = 0; m < lim; ++m) {  // member 0 always in bucket 1
      Bucket x, y;
      for (size_t i = 0; i < mem.size(); ++i) ((i > 0 && (m >> (i - 1) & 1)) ? y : x).add(mem[i]);
      const int c = cost(x, y);
      if (c < best) {
        best = c;
        b1 = x;
        b2 = y;
      }
    }
    return;
  }
  for (int b : mem) {
    Bucket x = b1, y = b2;
    x.add(b);
    y.add(b);
    if (cost(x, b2) <= cost(b1, y))
      b1 = x;
    else
      b2 = y;
  }
}

}  // namespace

int build_tables(const uint32_t* opc, uint32_t nop, DfaTables& out, std::string& err)
{
  if (opc == nullptr || nop == 0) {
    err = "empty opcode table";
    return 2;
  }
  std::vector<RawState> raw;
  std::unordered_map<uint32_t, uint32_t> index_of_pc;  // pc -> raw index
  raw.reserve(64);
  raw.push_back(RawState{0, 0, {}});
  index_of_pc[0] = 0;
  for (size_t qi = 0; qi < raw.size(); ++qi) {
    uint32_t pc = raw[qi].pc;
    uint32_t k = pc;
    uint32_t cap = 0;
    // block header
    while (k < nop && !word_is_goto(opc[k])) {
      uint32_t op = opc[k] >> 24;
      if (op == 0xfe) {
        cap = opc[k] & 0xffffff;
      } else {
        err = "opcode table uses REDO/TAIL/HEAD/indent words";
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
        err = "opcode table uses meta edges (anchors / word boundaries)";
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
        raw.push_back(RawState{(uint32_t)t, 0, {}});
      }
    }
    raw[qi].cap = cap;
    std::copy(tgt, tgt + 256, raw[qi].target_pc);
  }

  // renumber: dead = 0, non-accepting states, then accepting states
  const uint32_t n = (uint32_t)raw.size();
  std::vector<uint32_t> sid(n);
  uint32_t next_id = 1;
  for (uint32_t i = 0; i < n; ++i)
    if (raw[i].cap == 0) sid[i] = next_id++;
  const uint32_t first_acc = next_id;
  for (uint32_t i = 0; i < n; ++i)
    if (raw[i].cap != 0) sid[i] = next_id++;
  const uint32_t S = next_id;

  // dense next[sid][byte] in new ids
  std::vector<uint32_t> nxt((size_t)S * 256, 0);
  std::vector<uint32_t> caps(S, 0);
  for (uint32_t i = 0; i < n; ++i) {
    caps[sid[i]] = raw[i].cap;
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
    if ((uint64_t)S * r > 65536) {
      err = "DFA too large for 16-bit device tables";
      return 1;
    }
    t.format = FMT_CLASS;
    t.row = r;
    t.log_row = lr;
  }
  const uint32_t R = t.row;
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
  t.caps = caps;
  const uint32_t start_sid = sid[0];
  t.start = start_sid * R;
  t.accepting = S - first_acc;
  t.accb = (t.accepting > 0) ? first_acc * R : 0x10000u;
  // prefilter sets (see tables.hpp): A = first bytes that complete a match,
  // B = other first bytes, C = bytes that can follow a byte of B, D = bytes
  // that can follow such a pair; short2 = some 2-byte prefix already accepts
  bool setA[256] = {}, setB[256] = {}, setC[256] = {}, setD[256] = {};
  bool short2 = false;
  uint32_t nf = 0;
  for (int c = 0; c < 256; ++c) {
    const uint32_t s1 = nxt[(size_t)start_sid * 256 + c];
    if (s1 == 0) continue;
    ++nf;
    if (s1 >= first_acc) {
      setA[c] = true;
      continue;
    }
    setB[c] = true;
    for (int d = 0; d < 256; ++d) {
      const uint32_t s2 = nxt[(size_t)s1 * 256 + d];
      if (s2 == 0) continue;
      setC[d] = true;
      if (s2 >= first_acc) short2 = true;
      for (int e = 0; e < 256; ++e)
        if (nxt[(size_t)s2 * 256 + e] != 0) setD[e] = true;
    }
  }
  t.first_bytes = nf;
  Bucket a1, a2, b1, b2, c1, c2, d1, d2;
  split_set(setA, a1, a2);
  a1 = Bucket();  // A uses one bucket (bit 0): merge both halves
  for (int c = 0; c < 256; ++c)
    if (setA[c]) a1.add(c);
  split_set(setB, b1, b2);
  split_set(setC, c1, c2);
  if (short2) {  // a match may end after 2 bytes: no third-byte test
    for (int c = 0; c < 256; ++c) setD[c] = true;
  }
  split_set(setD, d1, d2);
  const Bucket* bk[7] = {&a1, &b1, &b2, &c1, &c2, &d1, &d2};
  for (int bit = 0; bit < 7; ++bit) {
    for (int v = 0; v < 8; ++v) {
      if (bk[bit]->lo >> v & 1) t.ft[v] |= (uint8_t)(1u << bit);
      if (bk[bit]->mid >> v & 1) t.ft[8 + v] |= (uint8_t)(1u << bit);
    }
    for (int v = 0; v < 4; ++v)
      if (bk[bit]->hi >> v & 1) t.ft[16 + v] |= (uint8_t)(1u << bit);
  }
  // candidate density on printable ASCII + newline, assuming independent bytes
  auto frac = [](const Bucket& x, const Bucket& y) {
    int n = 0;
    for (int b = 0x20; b < 0x7f; ++b) n += (x.has(b) || y.has(b)) ? 1 : 0;
    return n / 95.0;
  };
  const double pa = frac(a1, a1), pb = frac(b1, b2), pc = frac(c1, c2), pd = frac(d1, d2);
  t.fdensity = pa + (1.0 - pa) * pb * pc * pd;
  // the sparse kernel pays off when few positions survive the prefilter
  t.filter = t.format == FMT_BYTE && nf > 0 && t.fdensity <= 0.15;
  out = std::move(t);
  return 0;
}

}  // namespace ugpu
