// device_common.hpp -- device building blocks shared by the scan kernels:
// flattened DFA table lookup, the exact FIND walk, match emitters, and the
// chain step/merge used to stitch speculative pieces.
#pragma once
#include <type_traits>

#include "ctx_bits.hpp"
#include "scan_kernels.hpp"

namespace ugpu {

// ---------------------------------------------------------------- tables
// FMT 0: next[state][byte] (u16 row offsets); 1: cls[byte] + next[state][class]
// (u16); 2 (wide tables, states x row > 64 Ki): as 1 with u32 row offsets,
// read from global memory (the exact-walk kernels only: wfind, fix, forest)
template <int FMT>
struct Tab {
  using E = typename std::conditional<FMT == 2, uint32_t, uint16_t>::type;
  const E* trans;
  const uint8_t* cls;
  uint32_t start, accb;
  __device__ __forceinline__ uint32_t step(uint32_t s, uint32_t b) const
  {
    if constexpr (FMT == 0)
      return trans[s | b];
    else
      return trans[s + cls[b]];
  }
};

// the table of a scan in global memory
template <int FMT>
__device__ __forceinline__ Tab<FMT> tab_global(const ScanParams& P)
{
  if constexpr (FMT == 2)
    return Tab<2>{P.trans32, P.cls, P.start, P.accb};
  else
    return Tab<FMT>{P.trans, P.cls, P.start, P.accb};
}

// bytes [base, lend) are staged in LDS; anything else is read from global
struct Win {
  const uint8_t* lds;
  uint64_t base, lend;
  const uint8_t* g;
  uint64_t rend;
  uint32_t eof;
  // option W only (walk<FMT, 1>): Word ranges and the buffer's first byte
  const uint32_t* wtab = nullptr;
  uint32_t nwtab = 0;
  uint64_t bob = 0;
  // line anchors / option N only (walk<FMT, 2>): per-context accept indices
  // (tables.hpp acap), the row shift of the table's entries, whether position
  // bob starts a line, option N
  const uint32_t* acap = nullptr;
  uint32_t log_row = 0;
  uint32_t bol0 = 1;
  uint32_t nul = 0;
  uint32_t cword = 0;  // word-boundary meta edges: 64 contexts (ctx_bits.hpp), Word ranges in wtab
  const uint32_t* amap = nullptr;  // cword: each state's row of acap (tables.hpp acap_map)
  // loop-needle tables (ScanParams::lb_cls): the 256-bit set C of C+ N
  const uint32_t* lb = nullptr;
  // option W: per-state accept indices (ScanParams::caps; kCapRedo: REDO)
  const uint32_t* caps = nullptr;
  // dominated restarts (ScanParams::dom): bit = state id
  const uint32_t* dom = nullptr;
  // lookahead (ScanParams::look, walk mode kWalkLook): per state TAIL / HEAD masks
  const uint32_t* look = nullptr;
  // an LDS copy of bytes [wa, wa + wn) that the W / context walks read instead
  // of global memory (sparse_kernel's per-lane candidate window; wn = 0: none)
  const uint8_t* wl = nullptr;
  uint64_t wa = 0;
  uint32_t wn = 0;
};

// the byte at k (< rend) for the W and context walks: from the LDS window when
// it holds k, else from global memory
__device__ __forceinline__ uint32_t wbyte(const struct Win& w, uint64_t k)
{
  const uint64_t o = k - w.wa;  // (below the window: wraps to a large value)
  return o < w.wn ? (uint32_t)w.wl[o] : (uint32_t)w.g[k];
}

// Walk modes (template argument W of walk / chain_step / merge)
constexpr int kWalkPlain = 0, kWalkWord = 1, kWalkCtx = 2, kWalkLook = 3;

// The window of a scan: bytes from global memory, W / anchor context from P.
__device__ __forceinline__ Win win_of(const ScanParams& P)
{
  Win w;
  w.lds = nullptr;
  w.base = 0;
  w.lend = 0;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  w.wtab = P.wtab;
  w.nwtab = P.nwtab;
  w.bob = P.bob;
  w.acap = P.acap;
  w.log_row = P.log_row;
  w.bol0 = P.bol0;
  w.nul = P.nul;
  w.cword = P.ctx_word;
  w.amap = P.amap;
  w.lb = P.lb_cls;
  w.caps = P.caps;
  w.dom = P.dom;
  w.look = P.look;
  return w;
}

// ---------------------------------------------------------------- option W
// Matcher option W (ugrep -w): a walk starts only where at_wb() holds and a
// TAKE counts only where at_we() holds (lib/matcher.cpp:107, :142, :208;
// include/reflex/matcher.h:1194-1237, WITH_SPAN forms).  Bytes are read from
// global memory; at and past the readable end they read as 0 (the reference
// buffer's NUL terminator).  iswword = binary search over the Unicode 15.1
// Word ranges (matcher.h:457-1192).
__device__ __forceinline__ uint32_t wrd(const Win& w, uint64_t k) { return k < w.rend ? wbyte(w, k) : 0u; }

__device__ __forceinline__ bool wisword(const Win& w, uint32_t c)
{
  int lo = 0, hi = (int)w.nwtab - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (c < w.wtab[2 * mid])
      hi = mid - 1;
    else if (c > w.wtab[2 * mid + 1])
      lo = mid + 1;
    else
      return true;
  }
  return false;
}

// reflex::utf8(const char*) (include/reflex/utf8.h:138-215, restricted form)
__device__ __forceinline__ uint32_t wutf8(const Win& w, uint64_t k)
{
  const uint32_t c = wrd(w, k);
  if (c < 0x80) return c;
  uint32_t c1 = wrd(w, k + 1);
  if (c < 0xC0 || (c == 0xC0 && c1 != 0x80) || c == 0xC1 || (c1 & 0xC0) != 0x80) return 0xFFFD;
  c1 &= 0x3F;
  if (c < 0xE0) return ((c & 0x1F) << 6) | c1;
  uint32_t c2 = wrd(w, k + 2);
  if ((c == 0xE0 && c1 < 0x20) || (c2 & 0xC0) != 0x80) return 0xFFFD;
  c2 &= 0x3F;
  if (c < 0xF0) return ((c & 0x0F) << 12) | (c1 << 6) | c2;
  const uint32_t c3 = wrd(w, k + 3);
  if ((c == 0xF0 && c1 < 0x10) || (c == 0xF4 && c1 >= 0x10) || c >= 0xF5 || (c3 & 0xC0) != 0x80) return 0xFFFD;
  return ((c & 0x07) << 18) | (c1 << 12) | (c2 << 6) | (c3 & 0x3F);
}

__device__ __forceinline__ bool walnum(uint32_t c) { return (c - '0' < 10u) || ((c | 0x20u) - 'a' < 26u); }

// at_wb() for a walk starting at p
__device__ __forceinline__ bool at_wb(const Win& w, uint64_t p)
{
  if (p <= w.bob) return true;  // BOB
  const uint32_t c = wbyte(w, p - 1);
  if (c == '\n') return true;
  if (c == '_') return false;
  if ((c & 0xC0) == 0x80) {
    uint64_t k = p - 1;
    if (k > w.bob && (wbyte(w, --k) & 0xC0) == 0x80)
      if (k > w.bob && (wbyte(w, --k) & 0xC0) == 0x80)
        if (k > w.bob) --k;
    return !wisword(w, wutf8(w, k));
  }
  return !walnum(c);
}

// at_we() for a match ending at q (q at the end of the stream: EOF)
__device__ __forceinline__ bool at_we(const Win& w, uint64_t q, uint32_t& ovf)
{
  if (q >= w.rend) {
    if (!w.eof) ovf = 1;
    return true;
  }
  const uint32_t c = wbyte(w, q);
  if (c == '_') return false;
  if ((c & 0xC0) == 0xC0) {
    // the code point after the match decides; when its bytes run past a readable
    // end that is not EOF, so does the next chunk (a stream feed, a shard halo)
    const uint64_t need = c >= 0xF0 ? 4u : c >= 0xE0 ? 3u : 2u;
    if (q + need > w.rend && !w.eof) ovf = 1;
    return !wisword(w, wutf8(w, q));
  }
  return !walnum(c);
}

// ---------------------------------------------------------------- anchors
// Line anchors (META_BOL `^`, META_EOL `$`) and option N.  The reference fixes
// `bol` at the walk start (lib/matcher.cpp:93: at_bol(), the byte before is
// '\n' or the position is the buffer begin) and tests `$` on the byte after
// the current position (:294-316: '\n', EOF, or '\r' before '\n'); the
// accept at a state is tables.hpp acap[sid * 4 + bol * 2 + eol].
// eol at q (q at the end of the stream: EOF; at a readable end that is not
// EOF the answer depends on bytes not read yet: ovf)
__device__ __forceinline__ uint32_t at_eol(const Win& w, uint64_t q, uint32_t& ovf)
{
  if (q >= w.rend) {
    if (!w.eof) ovf = 1;
    return 1u;
  }
  const uint32_t c = wbyte(w, q);
  if (c == '\n') return 1u;
  if (c != '\r') return 0u;
  if (q + 1 >= w.rend) {
    if (!w.eof) ovf = 1;
    return 0u;
  }
  return wbyte(w, q + 1) == '\n' ? 1u : 0u;
}

// Word-boundary meta edges (META_WBB .. META_EWE, include/reflex/pattern.h:
// 933-940), tested by the interpreter after it fetched the byte at the
// current position q (lib/matcher.cpp:317-404) through
// include/reflex/matcher.h:1194-1319: at_wb / at_bw of the match begin p
// (txt_, len_ = 0 during FIND; fixed for the walk like bol) and at_ew / at_we
// of q.
// at_bw(): a word character at the match begin p (matcher.h:1239-1254)
__device__ __forceinline__ bool at_bw(const Win& w, uint64_t p, uint32_t& ovf)
{
  if (p >= w.rend && !w.eof) ovf = 1;
  const uint32_t c = wrd(w, p);
  if (c == '_') return true;
  if ((c & 0xC0) == 0xC0) {
    const uint64_t need = c >= 0xF0 ? 4u : c >= 0xE0 ? 3u : 2u;
    if (p + need > w.rend && !w.eof) ovf = 1;
    return wisword(w, wutf8(w, p));
  }
  return walnum(c);
}

// at_ew(): a word character before q (matcher.h:1256-1279; before the buffer
// begin: got_ = BOB, no word)
__device__ __forceinline__ bool at_ew(const Win& w, uint64_t q)
{
  if (q <= w.bob) return false;
  const uint32_t c = wbyte(w, q - 1);
  if (c == '\n') return false;
  if (c == '_') return true;
  if ((c & 0xC0) == 0x80 && q - w.bob >= 2) {
    // back over at most two more continuation bytes to the lead byte
    uint64_t k = q - 2;
    if ((wbyte(w, k) & 0xC0) == 0x80)
      if (k > w.bob && (wbyte(w, --k) & 0xC0) == 0x80)
        if (k > w.bob) --k;
    return wisword(w, wutf8(w, k));
  }
  return walnum(c);
}

// at_we() as the meta edges call it: at_we(c, pos_) with pos_ one past the
// byte c at q (matcher.h:1281-1313), so a lead byte's code point is decoded
// from the byte after it (a continuation byte in valid UTF-8: no word
// character, the boundary holds); at EOF true
__device__ __forceinline__ bool at_we_meta(const Win& w, uint64_t q, uint32_t& ovf)
{
  if (q >= w.rend) {
    if (!w.eof) ovf = 1;
    return true;
  }
  const uint32_t c = wbyte(w, q);
  if (c == '_') return false;
  if ((c & 0xC0) == 0xC0) {
    if (q + 5 > w.rend && !w.eof) ovf = 1;
    return !wisword(w, wutf8(w, q + 1));
  }
  return !walnum(c);
}

// at_wb() as the meta edges call it during a walk from p whose last accept
// ended at cur (p before any): got_ is the byte before p, but a continuation
// byte there is decoded back from cur_ - 1 (matcher.h:1202-1210), and TAKE
// moves cur_ (lib/matcher.cpp:207-217).  Only reached for p > bob.
__device__ __forceinline__ bool at_wb_cur(const Win& w, uint64_t cur)
{
  uint64_t k = cur - 1;
  if (k > w.bob && (wbyte(w, --k) & 0xC0) == 0x80)
    if (k > w.bob && (wbyte(w, --k) & 0xC0) == 0x80)
      if (k > w.bob) --k;
  return !wisword(w, wutf8(w, k));
}

// the walk bits of a walk starting at p (shifted into the acap index):
// line contexts bol << 1; word contexts CTX_BOL | CTX_WB | CTX_BW
__device__ __forceinline__ uint32_t ctx_walk_bits(const Win& w, uint64_t p, uint32_t& ovf)
{
  const uint32_t bol = p <= w.bob ? w.bol0 : (wbyte(w, p - 1) == '\n' ? 1u : 0u);
  if (!w.cword) return bol << 1;
  return (bol ? CTX_BOL : 0u) | (at_wb(w, p) ? CTX_WB : 0u) | (at_bw(w, p, ovf) ? CTX_BW : 0u);
}

// accept at q in the state of entry e: the acap index (0 = none; the dead
// state's indices never accept).  wb: ctx_walk_bits of the walk.
__device__ __forceinline__ uint32_t ctx_accept(const Win& w, uint32_t e, uint32_t wb, uint64_t q, uint32_t& ovf)
{
  if (w.cword) {
    const uint32_t b = (w.amap[e >> w.log_row] << 6) | wb;
    const uint32_t k = b | at_eol(w, q, ovf) | (at_ew(w, q) ? CTX_EW : 0u) | (at_we_meta(w, q, ovf) ? CTX_WE : 0u);
    return w.acap[k] ? k : 0u;
  }
  const uint32_t b = ((e >> w.log_row) << 2) | wb;
  const uint32_t a0 = w.acap[b], a1 = w.acap[b + 1];
  if (a0 == a1) return a0 ? b : 0u;
  const uint32_t k = b + at_eol(w, q, ovf);
  return w.acap[k] ? k : 0u;
}

// Longest match starting at p (0 = none).  `le` = entry of the last accepting
// state (its row identifies the accept index).  Mirrors the reference walk:
// TAKE on entering an accepting state (lib/matcher.cpp:207-217), stop on HALT
// (:528-541) or EOF (:460-465).  Mode kWalkCtx: `le` = the acap index of the
// last accept (also for an empty match at p: then le != 0 and 0 is returned).
template <int FMT, int W = kWalkPlain>
__device__ __forceinline__ uint64_t walk(const Tab<FMT>& T, const Win& w, uint64_t p, uint32_t& le, uint32_t& ovf)
{
  uint32_t s = T.start;
  uint64_t q = p, last = p;
  le = 0;
  if constexpr (W == kWalkCtx) {
    uint32_t bol = ctx_walk_bits(w, p, ovf);
    // (a continuation byte before p: at_wb follows the last accept, at_wb_cur)
    const bool wbc = w.cword && p > w.bob && (wbyte(w, p - 1) & 0xC0) == 0x80;
    // (a start state below accb accepts in no context: no lookups)
    le = s >= T.accb ? ctx_accept(w, s, bol, q, ovf) : 0u;
    while (q < w.rend) {
      const uint32_t e = T.step(s, wbyte(w, q));
      if (e == 0) return last - p;
      s = e;
      ++q;
      if (e >= T.accb) {
        if (wbc && last != p) bol = (bol & ~CTX_WB) | (at_wb_cur(w, last) ? CTX_WB : 0u);
        const uint32_t a = ctx_accept(w, e, bol, q, ovf);
        if (a) {
          last = q;
          le = a;
        }
      }
    }
    if (!w.eof) ovf = 1;
    return last - p;
  }
  if constexpr (W == kWalkWord) {
    if (!at_wb(w, p)) return 0;
    while (q < w.rend) {
      const uint32_t e = T.step(s, wbyte(w, q));
      if (e == 0) return last - p;
      s = e;
      ++q;
      // (a REDO accept, ugrep -N, does not test at_we: lib/matcher.cpp:151-156,
      // :218-225; the emitters step over a match whose last accept is REDO)
      if (e >= T.accb && ((w.caps && w.caps[e >> w.log_row] == kCapRedo) || at_we(w, q, ovf))) {
        last = q;
        le = e;
      }
    }
    if (!w.eof) ovf = 1;
    return last - p;
  }
  if constexpr (W == kWalkLook) {
    // lookahead (tables.hpp look): each state's block on entry, as the
    // reference runs it (lib/matcher.cpp:139-175): TAKE (the match would end
    // here), TAIL la (it ends where HEAD la was recorded in this walk, if it
    // was), HEAD la (record here); records cleared per walk (:104)
    uint32_t lap[4] = {~0u, ~0u, ~0u, ~0u};  // (offsets from p; ~0: not recorded)
    // option W (lookahead tables have no word contexts, so a Word table means
    // W): the walk starts where at_wb holds, a TAKE counts where at_we holds,
    // TAIL / HEAD as without W (lib/matcher.cpp:107, :142, :157-175, :208)
    const bool wm = w.nwtab != 0;
    if (wm && !at_wb(w, p)) return 0;
    auto enter = [&](uint32_t e, uint64_t at) __attribute__((always_inline)) {
      if (e >= T.accb && (!wm || at_we(w, at, ovf))) {
        last = at;
        le = e;
      }
      const uint32_t lk = w.look[e >> w.log_row];
      if (lk) {
#pragma unroll
        for (int la = 0; la < 4; ++la)
          if (((lk >> la) & 1u) && lap[la] != ~0u) last = p + lap[la];
#pragma unroll
        for (int la = 0; la < 4; ++la)
          if ((lk >> (8 + la)) & 1u) lap[la] = (uint32_t)(at - p);
      }
    };
    enter(s, q);
    if (last == p) le = 0;  // (an empty match at p is no match: the chain moves to p + 1)
    while (q < w.rend) {
      const uint32_t e = T.step(s, wbyte(w, q));
      if (e == 0) return last - p;
      s = e;
      ++q;
      enter(e, q);
    }
    if (!w.eof) ovf = 1;
    return last - p;
  }
  const uint64_t l1 = w.lend < w.rend ? w.lend : w.rend;
  while (q < l1) {
    uint32_t e = T.step(s, w.lds[q - w.base]);
    if (e == 0) return last - p;
    s = e;
    ++q;
    if (e >= T.accb) {
      last = q;
      le = e;
    }
  }
  while (q < w.rend) {
    uint32_t e = T.step(s, w.g[q]);
    if (e == 0) return last - p;
    s = e;
    ++q;
    if (e >= T.accb) {
      last = q;
      le = e;
    }
  }
  if (!w.eof) ovf = 1;  // a live walk ran into the end of this shard's readable bytes
  return last - p;
}

// A plain walk from p (walk<FMT>) that also finds where a failed walk lets
// the FIND chain go on (w.dom, tables.hpp dom): `skip` = the first position
// q > p whose state does not dominate the start state, or one past the byte
// the walk died on, or the position where it stopped.  If the walk from p
// accepts nowhere, no walk from a position in (p, skip) accepts either: its
// accepted strings would be accepted by p's walk from the dominating state it
// is in there.
template <int FMT>
__device__ __forceinline__ uint64_t walk_dom(const Tab<FMT>& T, const Win& w, uint64_t p, uint32_t& le, uint32_t& ovf,
                                             uint64_t& skip)
{
  uint32_t s = T.start;
  uint64_t q = p, last = p;
  le = 0;
  skip = 0;
  auto dom = [&w](uint32_t e) { return (w.dom[e >> (w.log_row + 5)] >> ((e >> w.log_row) & 31)) & 1u; };
  const uint64_t l1 = w.lend < w.rend ? w.lend : w.rend;
  while (q < w.rend) {
    const uint32_t e = T.step(s, q < l1 ? (uint32_t)w.lds[q - w.base] : (uint32_t)w.g[q]);
    if (e == 0) {
      if (!skip) skip = q + 1;
      return last - p;
    }
    s = e;
    ++q;
    if (e >= T.accb) {
      last = q;
      le = e;
    }
    if (!skip && !dom(e)) skip = q;
  }
  if (!w.eof) ovf = 1;  // a live walk ran into the end of this shard's readable bytes
  if (!skip) skip = q;
  return last - p;
}

// Where the FIND chain goes on after a walk from c that is known to accept
// nowhere (fix_kernel's resolved open walks; w.dom set): walk_dom's skip,
// looking no further than lim.
template <int FMT>
__device__ __forceinline__ uint64_t dom_restart(const Tab<FMT>& T, const Win& w, uint64_t c, uint64_t lim)
{
  uint32_t s = T.start;
  uint64_t q = c;
  while (q < lim && q < w.rend) {
    const uint32_t e = T.step(s, (uint32_t)w.g[q]);
    if (e == 0) return q + 1;
    s = e;
    ++q;
    if (!((w.dom[e >> (w.log_row + 5)] >> ((e >> w.log_row) & 31)) & 1u)) return q;
  }
  return q > c + 1 ? q : c + 1;
}

struct Ctx {
  const uint32_t* caps;
  uint32_t log_row;
  int64_t delta;
};

// (a match whose last accept is REDO, kCapRedo, is neither counted nor
// written: the chain steps over it, lib/matcher.cpp:732-738)
struct CountEm {
  uint64_t cnt = 0, dg = 0, dc = 0;
  __device__ __forceinline__ void put(const Ctx& c, uint64_t pos, uint64_t len, uint32_t le, int sign)
  {
    uint64_t st = pos + (uint64_t)c.delta;
    uint64_t cap = c.caps[le >> c.log_row];
    if (cap == kCapRedo) return;
    uint64_t d1 = st * 31 + len, d2 = (st + 1) * cap;
    if (sign > 0) {
      ++cnt;
      dg += d1;
      dc += d2;
    } else {
      --cnt;
      dg -= d1;
      dc -= d2;
    }
  }
};

struct WriteEm {
  uint64_t idx;
  uint64_t capacity;
  uint64_t* start;
  uint32_t* len;
  uint32_t* cap;
  uint32_t overflow = 0;
  __device__ __forceinline__ void put(const Ctx& c, uint64_t pos, uint64_t l, uint32_t le, int)
  {
    const uint32_t a = c.caps[le >> c.log_row];
    if (a == kCapRedo) return;
    if (idx < capacity) {
      start[idx] = pos + (uint64_t)c.delta;
      len[idx] = (uint32_t)l;
      if (cap) cap[idx] = a;  // (NULL: 12-byte records, one accept index)
    } else {
      overflow = 1;
    }
    ++idx;
  }
};

// One step of the FIND chain from p: the longest match at p (emitted with
// `sign`, then the chain continues at its end) or p+1.
// Mode kWalkCtx with option N: an empty match at p is reported (the chain
// still moves to p+1, lib/matcher.cpp:682-728).
// Loop-needle tables (w.lb) and cap != 0: a failed walk from a byte of C
// means no needle in the rest of its C-run, so no position of the run starts
// a match: the chain skips to the run's end (at most to cap), which keeps the
// serial re-walks of fix_kernel linear over long runs without a needle.
// Tables with dominated restarts (w.dom) and cap != 0: a failed plain walk
// moves the chain to walk_dom's skip (at most to cap), so a needle-free run
// costs one walk, not one per position.
template <int FMT, class Em, int W = kWalkPlain>
__device__ __forceinline__ uint64_t chain_step(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t p, Em& em,
                                               int sign, uint32_t& ovf, uint64_t cap = 0)
{
  uint32_t le;
  if constexpr (W == kWalkPlain) {
    if (cap && w.dom) {
      uint64_t skip;
      const uint64_t len = walk_dom<FMT>(T, w, p, le, ovf, skip);
      if (len) {
        em.put(c, p, len, le, sign);
        return p + len;
      }
      return skip < cap ? skip : (cap > p + 1 ? cap : p + 1);
    }
  }
  const uint64_t len = walk<FMT, W>(T, w, p, le, ovf);
  if constexpr (W == kWalkLook) {
    // a TAIL moved the end of a walk whose TAKE failed (option W: at_we):
    // no match, and FIND goes on one past that end (lib/matcher.cpp:621-637,
    // adv_(cur_ + 1))
    if (len && !le) return p + len + 1;
  }
  if (len) {
    em.put(c, p, len, le, sign);
    return p + len;
  }
  if constexpr (W != kWalkCtx) {
    auto in_c = [&w](uint32_t b) { return (w.lb[b >> 5] >> (b & 31)) & 1u; };
    if (cap && w.lb && p < w.rend && in_c(w.g[p])) {
      uint64_t q = p + 1;
      while (q < cap && q < w.rend && in_c(w.g[q])) ++q;
      return q;
    }
  }
  if constexpr (W == kWalkCtx) {
    if (le && w.nul) em.put(c, p, 0, le, sign);
  }
  return p + 1;
}

// Re-enter [.., e) at xn instead of xo.  Adds (true - speculative) matches to em.
// Returns true if the chains met (exit unchanged), else sets nexit.  A merge
// whose chains cross more than `budget` bytes without meeting sets `over` and
// stops (the result is then invalid: UGPU_FLAG_BUDGET).
template <int FMT, int W = kWalkPlain>
__device__ __forceinline__ bool merge(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t xo, uint64_t xn,
                                      uint64_t e, CountEm& em, uint64_t& nexit, uint32_t& ovf,
                                      uint64_t budget = ~0ull, uint32_t* over = nullptr)
{
  uint64_t po = xo, pn = xn;
  const uint64_t lim = (xo < xn ? xo : xn) + budget < (xo < xn ? xo : xn) ? ~0ull : (xo < xn ? xo : xn) + budget;
  for (;;) {
    if (po == pn) return true;
    if (over && (po > lim || pn > lim)) {
      *over = 1;
      return true;
    }
    if (po >= e && pn >= e) {
      nexit = pn;
      return false;
    }
    if (po < pn)
      po = chain_step<FMT, CountEm, W>(T, w, c, po, em, -1, ovf, e);
    else
      pn = chain_step<FMT, CountEm, W>(T, w, c, pn, em, +1, ovf, e);
  }
}

__device__ __forceinline__ uint64_t lowbits(uint64_t k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }

__device__ __forceinline__ uint64_t clampu(uint64_t v, uint64_t a, uint64_t b) { return v < a ? a : (v > b ? b : v); }

__device__ __forceinline__ uint64_t wave_sum(uint64_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace ugpu
