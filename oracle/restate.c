/*
 * oracle/restate.c -- TEST INFRASTRUCTURE: CPU restatement of the reference
 * FIND path, used as the parity checker for the HIP engine.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product (ugrep_amd/) never links or calls it.
 *
 * Pinned against the reference itself: tests/golden/ holds outputs of
 * oracle/_ref/ref_harness (the reference libreflex compiled from
 * /root/reference/lib) and tests/test_oracle.py checks this file against them.
 *
 * What is restated:
 *   orc_dfa_build -- opcode words -> dense next[state][byte] table.  For each
 *     state block and byte it emulates the interpreter's descending range scan
 *     (lib/matcher.cpp:467-502) over the goto words whose format is
 *     include/reflex/pattern.h:1155-1247 (GOTO lo<<24|hi<<16|idx, HALT
 *     0x00FFFFFF, LONG idx 0xFFFE + next word, TAKE 0xFE..).  TAKE at the head
 *     of a block (lib/pattern.cpp:2945-2952) makes the state accepting; so
 *     does REDO (0xFD000000, a negative pattern's accept, ugrep -N
 *     '(?^...)'), with the accept ORC_REDO.  TAIL/HEAD (lookahead, indices
 *     below ORC_MAXLOOK) are kept per state as bit masks (look[]); meta edges
 *     other than META_BOL / META_EOL and the word boundaries META_WBB ..
 *     META_EWE (pattern.h:933-943), REDO in a table with meta edges, and
 *     lookahead with meta edges or REDO are rejected (ORC_UNSUPPORTED); meta
 *     edges are kept per state in block order (orc_find_a).
 *   orc_find -- the FIND driver of Matcher::match (lib/matcher.cpp:42-750) for
 *     tables without meta/lookahead, options A/N/W off: from p walk the DFA,
 *     remember the last TAKE (:139-150, :207-217), stop on HALT/EOF (:448-459,
 *     :528-541); emit the longest non-empty match and resume at its end
 *     (:681, :735-737), otherwise retry at p+1 (:635-661, :692-713).  With
 *     lookahead (:157-175) every state entry runs its block in order: TAKE
 *     (last = here), then each TAIL la (last = the position HEAD la recorded
 *     in this walk, if any), then each HEAD la (record here); the records are
 *     cleared per walk (:104).  A match
 *     whose last accept is REDO is not emitted and the search resumes at its
 *     end (:732-738 "ignore accept and continue"; an empty one moves to p+1
 *     as any empty match, :682-713).  The adv_
 *     prefilters (lib/matcher.cpp:797-954, lib/matcher_avx2.cpp) only skip
 *     positions that cannot start a match and are not restated -- except for
 *     tables with meta edges, where the Pattern's predictor can also reject
 *     positions the DFA matches at (anchored patterns without option N, "a$|ab";
 *     oracle/ref_harness.cpp mode "P", tests/golden/make_anchor_golden.py):
 *     orc_find_a restates the DFA semantics (the reference with its predictor
 *     off), and the golden fixtures record both.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "gen.h"

#define ORC_OK 0
#define ORC_UNSUPPORTED 1
#define ORC_INVAL 2
#define ORC_NOMEM 3

#define ORC_MAXMETA 4
#define ORC_MAXLOOK 8 /* lookahead indices per table (TAIL/HEAD words) */
#define ORC_REDO 0xffffffffu /* the accept of a REDO state (never an accept index: those have 24 bits) */
typedef struct orc_dfa
{
  uint32_t nstates; /* including dead state 0 */
  uint32_t start;
  uint32_t *next;   /* [nstates][256] */
  uint32_t *accept; /* [nstates], 0 = not accepting */
  uint32_t *meta;   /* [nstates][ORC_MAXMETA]: (META - META_MIN) << 24 | target state, in block order; 0 = none */
  int anchored;     /* some state has a meta edge */
  uint32_t *look;   /* [nstates]: TAIL la -> bit la, HEAD la -> bit 8 + la */
  int lookahead;    /* some state has TAIL/HEAD words */
} orc_dfa;

static int is_goto(uint32_t w) { return (uint32_t)(w << 8) >= (w & 0xff000000u); }
static int is_meta(uint32_t w) { return (w & 0x00ff0000u) == 0 && (w >> 24) > 0; }

void orc_dfa_free(orc_dfa *d)
{
  if (!d)
    return;
  free(d->next);
  free(d->accept);
  free(d->meta);
  free(d->look);
  free(d);
}

int orc_dfa_build(const uint32_t *opc, uint32_t nop, orc_dfa **out)
{
  uint32_t *id, *queue, nq = 0, qh = 0, ns = 1, cap = 64;
  orc_dfa *d;
  if (!opc || nop == 0 || !out)
    return ORC_INVAL;
  *out = NULL;
  id = (uint32_t *)calloc(nop, sizeof(uint32_t)); /* pc -> state id (0 = not a state) */
  queue = (uint32_t *)malloc(nop * sizeof(uint32_t));
  d = (orc_dfa *)calloc(1, sizeof(orc_dfa));
  if (!id || !queue || !d)
    goto nomem;
  d->next = (uint32_t *)calloc((size_t)cap * 256, sizeof(uint32_t));
  d->accept = (uint32_t *)calloc(cap, sizeof(uint32_t));
  d->meta = (uint32_t *)calloc((size_t)cap * ORC_MAXMETA, sizeof(uint32_t));
  d->look = (uint32_t *)calloc(cap, sizeof(uint32_t));
  if (!d->next || !d->accept || !d->meta || !d->look)
    goto nomem;
  id[0] = ns++;
  queue[nq++] = 0;
  d->start = 1;
  while (qh < nq)
  {
    uint32_t pc = queue[qh++];
    uint32_t s = id[pc];
    uint32_t g = pc;
    int c;
    if (s >= cap)
    {
      uint32_t ncap = cap * 2;
      uint32_t *nn = (uint32_t *)realloc(d->next, (size_t)ncap * 256 * sizeof(uint32_t));
      uint32_t *na;
      if (!nn)
        goto nomem;
      d->next = nn;
      na = (uint32_t *)realloc(d->accept, ncap * sizeof(uint32_t));
      if (!na)
        goto nomem;
      d->accept = na;
      {
        uint32_t *nm = (uint32_t *)realloc(d->meta, (size_t)ncap * ORC_MAXMETA * sizeof(uint32_t));
        if (!nm)
          goto nomem;
        d->meta = nm;
        memset(d->meta + (size_t)cap * ORC_MAXMETA, 0, (size_t)(ncap - cap) * ORC_MAXMETA * sizeof(uint32_t));
      }
      {
        uint32_t *nl = (uint32_t *)realloc(d->look, ncap * sizeof(uint32_t));
        if (!nl)
          goto nomem;
        d->look = nl;
        memset(d->look + cap, 0, (ncap - cap) * sizeof(uint32_t));
      }
      memset(d->next + (size_t)cap * 256, 0, (size_t)(ncap - cap) * 256 * sizeof(uint32_t));
      memset(d->accept + cap, 0, (ncap - cap) * sizeof(uint32_t));
      cap = ncap;
    }
    /* block header: [REDO|TAKE]? TAIL* HEAD*, then meta edges (not goto
       words: the interpreter tests them in block order before the byte edges,
       lib/matcher.cpp:193-450); META_BOL (0x109), META_EOL (0x10a) and the
       word boundaries 0x101-0x108, include/reflex/pattern.h:933-943 */
    {
      uint32_t nm = 0;
      while (g < nop && !is_goto(opc[g]))
      {
        uint32_t w = opc[g], op = w >> 24;
        if (op == 0xfe)
          d->accept[s] = w & 0xffffff;
        else if (w == 0xfd000000u)
          d->accept[s] = ORC_REDO; /* REDO (lib/pattern.cpp:2945-2947): precedes any TAKE */
        else if (is_meta(w) && op >= 0x01 && op <= 0x0a && nm < ORC_MAXMETA)
        {
          uint32_t idx = w & 0xffff, tgt = idx == 0xfffe ? (g + 1 < nop ? opc[g + 1] & 0xffffff : nop) : idx;
          if (idx == 0xffff || tgt >= nop)
            goto inval;
          if (id[tgt] == 0)
          {
            id[tgt] = ns++;
            queue[nq++] = tgt;
          }
          d->meta[(size_t)s * ORC_MAXMETA + nm++] = op << 24 | id[tgt];
          d->anchored = 1;
          if (idx == 0xfffe)
            ++g;
        }
        else if ((op == 0xfc || op == 0xfb) && (w & 0xffffff) < ORC_MAXLOOK)
        {
          /* TAIL / HEAD (pattern.h:1167-1174, lookahead_of: the low 16 bits) */
          d->look[s] |= (op == 0xfc ? 1u : 0x100u) << (w & 0xffff);
          d->lookahead = 1;
        }
        else
          goto unsupported; /* other metas, lookahead indices past ORC_MAXLOOK */
        ++g;
      }
    }
    if (g >= nop)
      goto inval;
    /* per byte: first goto word in block order with lo <= c <= hi */
    for (c = 0; c < 256; ++c)
    {
      uint32_t k = g;
      for (;;)
      {
        uint32_t w, lo, hi, idx, tgt;
        if (k >= nop)
          goto inval;
        w = opc[k];
        if (!is_goto(w) || is_meta(w))
          goto unsupported;
        lo = w >> 24;
        hi = (w >> 16) & 0xff;
        if ((uint32_t)c < lo || (uint32_t)c > hi)
        {
          /* a LONG goto's continuation word never matches a byte (it follows a
             goto with a higher lo, lib/pattern.cpp:2980-2983): step over it */
          k += (w & 0xffff) == 0xfffe ? 2 : 1;
          continue;
        }
        idx = w & 0xffff;
        if (idx == 0xffff)
          break; /* HALT: dead */
        if (idx == 0xfffe)
        {
          if (k + 1 >= nop)
            goto inval;
          tgt = opc[k + 1] & 0xffffff;
        }
        else
          tgt = idx;
        if (tgt >= nop)
          goto inval;
        if (id[tgt] == 0)
        {
          id[tgt] = ns++;
          queue[nq++] = tgt;
        }
        d->next[(size_t)s * 256 + c] = id[tgt];
        break;
      }
    }
  }
  d->nstates = ns;
  /* a meta edge whose target consumes bytes: the interpreter then tries the
     target's byte edges on the next byte first and falls back to the state's
     own through its backtrack point (lib/matcher.cpp:405-423, :513-523) -- two
     walks at once, outside this restatement's (and the engine's) one-state
     model.  Targets without byte edges only contribute accepts. */
  {
    uint32_t s, k, b;
    for (s = 1; s < ns; ++s)
      for (k = 0; k < ORC_MAXMETA; ++k)
      {
        uint32_t e = d->meta[(size_t)s * ORC_MAXMETA + k], t = e & 0xffffff;
        if (e == 0)
          break;
        for (b = 0; b < 256; ++b)
          if (d->next[(size_t)t * 256 + b] != 0)
            goto unsupported;
      }
    /* REDO with meta edges, lookahead with meta edges or REDO: not restated
       (the engine refuses them too) */
    if (d->lookahead && d->anchored)
      goto unsupported;
    if (d->anchored || d->lookahead)
      for (s = 1; s < ns; ++s)
        if (d->accept[s] == ORC_REDO)
          goto unsupported;
  }
  free(id);
  free(queue);
  *out = d;
  return ORC_OK;
unsupported:
  free(id);
  free(queue);
  orc_dfa_free(d);
  return ORC_UNSUPPORTED;
inval:
  free(id);
  free(queue);
  orc_dfa_free(d);
  return ORC_INVAL;
nomem:
  free(id);
  free(queue);
  orc_dfa_free(d);
  return ORC_NOMEM;
}

uint32_t orc_dfa_nstates(const orc_dfa *d) { return d->nstates; }

/* One FIND step at p (< n): returns match length (0 = none) and the accept. */
/* a state's block on entry at q in a walk from p (lookahead tables):
   TAKE, then TAIL la ascending, then HEAD la ascending (lib/matcher.cpp:139-175) */
static inline void orc_enter(const orc_dfa *d, uint32_t s, uint64_t p, uint64_t q, uint64_t *last, uint32_t *a,
                             int64_t *lap)
{
  uint32_t lk = d->look[s], la;
  if (d->accept[s])
  {
    *last = q;
    *a = d->accept[s];
  }
  for (la = 0; la < ORC_MAXLOOK; ++la)
    if (((lk >> la) & 1u) && lap[la] >= 0)
      *last = p + (uint64_t)lap[la];
  for (la = 0; la < ORC_MAXLOOK; ++la)
    if ((lk >> (8 + la)) & 1u)
      lap[la] = (int64_t)(q - p);
}

static inline uint64_t orc_step(const orc_dfa *d, const uint8_t *buf, uint64_t n, uint64_t p, uint32_t *acc)
{
  uint32_t s = d->start;
  uint64_t q = p, last = p;
  uint32_t a = 0;
  if (d->lookahead)
  {
    int64_t lap[ORC_MAXLOOK];
    int k;
    for (k = 0; k < ORC_MAXLOOK; ++k)
      lap[k] = -1;
    orc_enter(d, s, p, q, &last, &a, lap);
    while (q < n)
    {
      uint32_t t = d->next[(size_t)s * 256 + buf[q]];
      if (t == 0)
        break;
      s = t;
      ++q;
      orc_enter(d, s, p, q, &last, &a, lap);
    }
    *acc = a;
    return last - p;
  }
  while (q < n)
  {
    uint32_t t = d->next[(size_t)s * 256 + buf[q]];
    if (t == 0)
      break;
    s = t;
    ++q;
    if (d->accept[s])
    {
      last = q;
      a = d->accept[s];
    }
  }
  *acc = a;
  return last - p;
}

/*
 * Scan buf[start..n): count, digest = sum(start*31+len), dcap = sum((start+1)*cap)
 * with start positions offset by `bias`.  If list != NULL, writes up to
 * list_cap (start,len,cap) triples.  Returns the number of matches.
 */
uint64_t orc_find(const orc_dfa *d, const uint8_t *buf, uint64_t n, uint64_t start, uint64_t bias,
                  uint64_t *digest, uint64_t *dcap, uint64_t *list, uint64_t list_cap)
{
  uint64_t p = start, cnt = 0, dg = 0, dc = 0;
  while (p < n)
  {
    uint32_t a;
    uint64_t len = orc_step(d, buf, n, p, &a);
    if (len > 0 && a == ORC_REDO)
    {
      p += len; /* a negative pattern's match: consumed, not reported */
    }
    else if (len > 0)
    {
      uint64_t st = p + bias;
      if (list && cnt < list_cap)
      {
        list[3 * cnt] = st;
        list[3 * cnt + 1] = len;
        list[3 * cnt + 2] = a;
      }
      ++cnt;
      dg += st * 31 + len;
      dc += (st + 1) * a;
      p += len;
    }
    else
    {
      ++p;
    }
  }
  if (digest)
    *digest = dg;
  if (dcap)
    *dcap = dc;
  return cnt;
}

/* ---- option W (ugrep -w, src/ugrep.cpp:8616-8618) ----
 * Matcher::match with opt_.W (lib/matcher.cpp:76, :107, :142, :208, :664): a
 * walk starts at p only if at_wb() holds there, and a TAKE counts only if
 * at_we() holds at the match end (include/reflex/matcher.h:1194-1237, WITH_SPAN
 * forms); otherwise the search moves to p+1 as for no match.  A REDO accept
 * (ugrep -N) counts without at_we, and a match whose last accept is REDO is
 * stepped over unreported, as without W.  iswword is the
 * Unicode 15.1 Word table (matcher.h:457-1192), the same ranges as \w: the
 * data file is shared with the product's compiler (it is pinned to the
 * reference by tools/gen_unicode_ranges.py, and this restatement by the W
 * goldens of tests/test_oracle.py).  Bytes at and past n read as 0 (the
 * reference buffer's NUL terminator). */
#include "../ugrep_amd/csrc/unicode_ranges.inc"

static int orc_iswword(uint32_t c)
{
  int lo = 0, hi = (int)(sizeof(k_word_ranges) / sizeof(k_word_ranges[0])) - 1;
  while (lo <= hi)
  {
    int mid = (lo + hi) / 2;
    if (c < k_word_ranges[mid][0])
      hi = mid - 1;
    else if (c > k_word_ranges[mid][1])
      lo = mid + 1;
    else
      return 1;
  }
  return 0;
}

static inline uint32_t orc_rd(const uint8_t *buf, uint64_t n, uint64_t k) { return k < n ? buf[k] : 0; }

/* reflex::utf8(const char*) (include/reflex/utf8.h:138-215), restricted form */
static uint32_t orc_utf8(const uint8_t *buf, uint64_t n, uint64_t k)
{
  uint32_t c = orc_rd(buf, n, k), c1, c2, c3;
  if (c < 0x80)
    return c;
  c1 = orc_rd(buf, n, k + 1);
  if (c < 0xC0 || (c == 0xC0 && c1 != 0x80) || c == 0xC1 || (c1 & 0xC0) != 0x80)
    return 0xFFFD;
  c1 &= 0x3F;
  if (c < 0xE0)
    return ((c & 0x1F) << 6) | c1;
  c2 = orc_rd(buf, n, k + 2);
  if ((c == 0xE0 && c1 < 0x20) || (c2 & 0xC0) != 0x80)
    return 0xFFFD;
  c2 &= 0x3F;
  if (c < 0xF0)
    return ((c & 0x0F) << 12) | (c1 << 6) | c2;
  c3 = orc_rd(buf, n, k + 3);
  if ((c == 0xF0 && c1 < 0x10) || (c == 0xF4 && c1 >= 0x10) || c >= 0xF5 || (c3 & 0xC0) != 0x80)
    return 0xFFFD;
  return ((c & 0x07) << 18) | (c1 << 12) | (c2 << 6) | (c3 & 0x3F);
}

static int orc_isalnum(uint32_t c) { return (c >= '0' && c <= '9') || ((c | 0x20) >= 'a' && (c | 0x20) <= 'z'); }

/* at_wb() before position p (matcher.h:1194-1216) */
static int orc_at_wb(const uint8_t *buf, uint64_t n, uint64_t p)
{
  uint32_t c;
  if (p == 0)
    return 1; /* BOB */
  c = buf[p - 1];
  if (c == '\n')
    return 1;
  if (c == '_')
    return 0;
  if ((c & 0xC0) == 0x80)
  {
    uint64_t k = p - 1;
    if (k > 0 && (buf[--k] & 0xC0) == 0x80)
      if (k > 0 && (buf[--k] & 0xC0) == 0x80)
        if (k > 0)
          --k;
    return !orc_iswword(orc_utf8(buf, n, k));
  }
  return !orc_isalnum(c);
}

/* at_we() at match end q (matcher.h:1217-1237); q == n is EOF */
static int orc_at_we(const uint8_t *buf, uint64_t n, uint64_t q)
{
  uint32_t c;
  if (q >= n)
    return 1;
  c = buf[q];
  if (c == '_')
    return 0;
  if ((c & 0xC0) == 0xC0)
    return !orc_iswword(orc_utf8(buf, n, q));
  return !orc_isalnum(c);
}

static inline uint64_t orc_step_w(const orc_dfa *d, const uint8_t *buf, uint64_t n, uint64_t p, uint32_t *acc)
{
  uint32_t s = d->start, a = 0;
  uint64_t q = p, last = p;
  *acc = 0;
  if (!orc_at_wb(buf, n, p))
    return 0;
  if (d->lookahead)
  {
    /* lookahead under W: orc_enter's block with the TAKE tested by at_we
       (lib/matcher.cpp:142, :208); TAIL / HEAD unchanged (:157-175) */
    int64_t lap[ORC_MAXLOOK];
    int k;
    uint32_t lk;
    for (k = 0; k < ORC_MAXLOOK; ++k)
      lap[k] = -1;
    for (;;)
    {
      lk = d->look[s];
      if (d->accept[s] && orc_at_we(buf, n, q))
      {
        last = q;
        a = d->accept[s];
      }
      for (k = 0; k < ORC_MAXLOOK; ++k)
        if (((lk >> k) & 1u) && lap[k] >= 0)
          last = p + (uint64_t)lap[k];
      for (k = 0; k < ORC_MAXLOOK; ++k)
        if ((lk >> (8 + k)) & 1u)
          lap[k] = (int64_t)(q - p);
      if (q >= n)
        break;
      {
        uint32_t t = d->next[(size_t)s * 256 + buf[q]];
        if (t == 0)
          break;
        s = t;
        ++q;
      }
    }
    *acc = a;
    return last - p;
  }
  while (q < n)
  {
    uint32_t t = d->next[(size_t)s * 256 + buf[q]];
    if (t == 0)
      break;
    s = t;
    ++q;
    /* (a REDO accept does not test at_we, lib/matcher.cpp:151-156, :218-225) */
    if (d->accept[s] && (d->accept[s] == ORC_REDO || orc_at_we(buf, n, q)))
    {
      last = q;
      a = d->accept[s];
    }
  }
  *acc = a;
  return last - p;
}

/* orc_find with option W (whole buffer buf[0..n), search from start) */
uint64_t orc_find_w(const orc_dfa *d, const uint8_t *buf, uint64_t n, uint64_t start, uint64_t *digest,
                    uint64_t *dcap, uint64_t *list, uint64_t list_cap)
{
  uint64_t p = start, cnt = 0, dg = 0, dc = 0;
  while (p < n)
  {
    uint32_t a;
    uint64_t len = orc_step_w(d, buf, n, p, &a);
    if (len > 0 && a == 0)
    {
      /* lookahead under W: a TAIL moved the end of a walk whose TAKE failed
         at_we -- no match (cap_ 0), and FIND goes on one past that end
         (lib/matcher.cpp:621-637: adv_(cur_ + 1)) */
      p += len + 1;
    }
    else if (len > 0 && a == ORC_REDO)
    {
      /* a match whose last accept is REDO: not reported, the search goes on
         at its end (lib/matcher.cpp:736-743) */
      p += len;
    }
    else if (len > 0)
    {
      if (list && cnt < list_cap)
      {
        list[3 * cnt] = p;
        list[3 * cnt + 1] = len;
        list[3 * cnt + 2] = a;
      }
      ++cnt;
      dg += p * 31 + len;
      dc += (p + 1) * a;
      p += len;
    }
    else
      ++p;
  }
  if (digest)
    *digest = dg;
  if (dcap)
    *dcap = dc;
  return cnt;
}

/* ---- line anchors (META_BOL ^, META_EOL $) and option N (empty matches) ----
 * The interpreter (lib/matcher.cpp:42-750) fixes `bol` at the walk start
 * (:93, at_bol(): the byte before is '\n', or the position is the buffer
 * begin, where got_ is '\n' under WITH_SPAN, include/reflex/absmatcher.h:1571-1580)
 * and, at each state, fetches the next byte ch and tests the state's meta edges
 * in block order (:294-316): META_BOL holds when bol, META_EOL when ch is
 * '\n', EOF, or '\r' followed by '\n'.  The first edge that holds is followed
 * without consuming ch (at most 5 in a row); a TAKE met there is an accept at
 * the current position (:207-217); then the walk goes on with the byte edges
 * (the backtrack point, :405-440).  Empty matches (:682-728): without option N
 * the search moves to p+1; with N the empty match is reported and the search
 * moves to p+1, except at the end of the input. */
/* Word boundaries (lib/matcher.cpp:317-404, include/reflex/matcher.h:1238-1319,
 * WITH_SPAN forms), tested after the interpreter fetched ch = buf[q] (pos_ =
 * q + 1; at EOF ch = EOF and pos_ = q).  Of the match begin p (txt_, len_ = 0
 * during FIND): at_wb() as for option W, at_bw() = a word character at p.  Of
 * the position: at_ew(ch) = a word character before q (k = pos_ + (ch == EOF)
 * = q + 1, byte buf[k - 2], got_ = BOB when q == 0), at_we(ch, pos_) = no word
 * character at q, where a lead byte's code point is read from buf[pos_] --
 * one byte past it. */
static int orc_at_bw(const uint8_t *buf, uint64_t n, uint64_t p)
{
  uint32_t c = orc_rd(buf, n, p);
  if (c == '_')
    return 1;
  if ((c & 0xC0) == 0xC0)
    return orc_iswword(orc_utf8(buf, n, p));
  return orc_isalnum(c);
}

static int orc_at_ew(const uint8_t *buf, uint64_t n, uint64_t q)
{
  uint64_t k = q + 1;
  uint32_t c;
  (void)n;
  if (k <= 1)
    return 0; /* got_ = BOB */
  c = buf[k - 2];
  if (c == '\n')
    return 0;
  if (c == '_')
    return 1;
  if ((c & 0xC0) == 0x80 && k > 2)
  {
    k -= 3;
    if ((buf[k] & 0xC0) == 0x80)
      if (k > 0 && (buf[--k] & 0xC0) == 0x80)
        if (k > 0)
          --k;
    return orc_iswword(orc_utf8(buf, n, k));
  }
  return orc_isalnum(c);
}

static int orc_at_we_meta(const uint8_t *buf, uint64_t n, uint64_t q)
{
  uint32_t c;
  if (q >= n)
    return 1; /* EOF */
  c = buf[q];
  if (c == '_')
    return 0;
  if ((c & 0xC0) == 0xC0)
    return !orc_iswword(orc_utf8(buf, n, q + 1));
  return !orc_isalnum(c);
}

/* at_wb() as the meta edges call it during a walk from p: got_ = buf[p - 1],
 * but a continuation byte there is decoded back from cur_ - 1 (matcher.h:
 * 1202-1210), and cur_ is the end of the walk's last accept so far (TAKE sets
 * it, lib/matcher.cpp:207-217), p before any */
static int orc_at_wb_cur(const uint8_t *buf, uint64_t n, uint64_t p, uint64_t cur)
{
  uint32_t c;
  if (p == 0)
    return 1; /* got_ = '\n' at the buffer begin (set_current, absmatcher.h:1571-1580) */
  c = buf[p - 1];
  if (c == '\n')
    return 1;
  if (c == '_')
    return 0;
  if ((c & 0xC0) == 0x80 && cur > 0)
  {
    uint64_t k = cur - 1;
    if (k > 0 && (buf[--k] & 0xC0) == 0x80)
      if (k > 0 && (buf[--k] & 0xC0) == 0x80)
        if (k > 0)
          --k;
    return !orc_iswword(orc_utf8(buf, n, k));
  }
  return !orc_isalnum(c);
}

/* walk context of a walk from p whose last accept ended at cur (p before
   any): bit 0 bol, bit 1 at_wb, bit 2 at_bw */
static int orc_walk_ctx(const uint8_t *buf, uint64_t n, uint64_t p, uint64_t cur)
{
  int bol = p == 0 || buf[p - 1] == '\n';
  return bol | orc_at_wb_cur(buf, n, p, cur) << 1 | orc_at_bw(buf, n, p) << 2;
}

/* the accept index at q of a walk from p in state s (cur: the end of its last
   accept so far, p before any), meta edges followed as above */
static uint32_t orc_accept_at(const orc_dfa *d, uint32_t s, const uint8_t *buf, uint64_t n, uint64_t p, uint64_t cur,
                              uint64_t q)
{
  uint32_t cap = d->accept[s];
  int wctx, bol, wb, bw, eol, ew, we;
  int jumps;
  if (d->meta[(size_t)s * ORC_MAXMETA] == 0)
    return cap; /* no meta edge: the contexts are not needed */
  wctx = orc_walk_ctx(buf, n, p, cur);
  bol = wctx & 1, wb = (wctx >> 1) & 1, bw = (wctx >> 2) & 1;
  eol = q >= n || buf[q] == '\n' || (buf[q] == '\r' && q + 1 < n && buf[q + 1] == '\n');
  ew = orc_at_ew(buf, n, q), we = orc_at_we_meta(buf, n, q);
  for (jumps = 0; jumps < 5; ++jumps)
  {
    uint32_t t = 0, k;
    for (k = 0; k < ORC_MAXMETA; ++k)
    {
      uint32_t e = d->meta[(size_t)s * ORC_MAXMETA + k], m = e >> 24;
      int holds;
      if (e == 0)
        break;
      switch (m)
      {
        case 0x01: holds = bw == wb; break;   /* META_WBB at_wbb() */
        case 0x02: holds = we == ew; break;   /* META_WBE at_wbe(ch) */
        case 0x03: holds = bw != wb; break;   /* META_NWB at_nwb() */
        case 0x04: holds = we != ew; break;   /* META_NWE at_nwe(ch) */
        case 0x05: holds = bw && wb; break;   /* META_BWB at_bwb() */
        case 0x06: holds = !bw && !wb; break; /* META_EWB at_ewb() */
        case 0x07: holds = !we && !ew; break; /* META_BWE at_bwe(ch) */
        case 0x08: holds = we && ew; break;   /* META_EWE at_ewe(ch) */
        case 0x09: holds = bol; break;
        default: holds = eol; break;
      }
      if (holds)
      {
        t = e & 0xffffff;
        break;
      }
    }
    if (t == 0)
      break;
    if (d->accept[t])
      cap = d->accept[t];
    s = t;
  }
  return cap;
}

int orc_dfa_anchored(const orc_dfa *d) { return d->anchored; }

/* orc_find for tables with ^ / $ edges, with option N (nul) on or off; the
   buffer begin (position 0) is a begin of line */
uint64_t orc_find_a(const orc_dfa *d, const uint8_t *buf, uint64_t n, uint64_t start, int nul, uint64_t *digest,
                    uint64_t *dcap, uint64_t *list, uint64_t list_cap)
{
  uint64_t p = start, cnt = 0, dg = 0, dc = 0;
  while (p < n)
  {
    uint32_t s = d->start, a = 0, c;
    uint64_t q = p, last = p;
    int hit = 0;
    if ((c = orc_accept_at(d, s, buf, n, p, p, q)) != 0)
    {
      hit = 1;
      a = c;
    }
    while (q < n)
    {
      uint32_t t = d->next[(size_t)s * 256 + buf[q]];
      if (t == 0)
        break;
      s = t;
      ++q;
      if ((c = orc_accept_at(d, s, buf, n, p, last, q)) != 0)
      {
        hit = 1;
        last = q;
        a = c;
      }
    }
    if (hit && (last > p || nul))
    {
      if (list && cnt < list_cap)
      {
        list[3 * cnt] = p;
        list[3 * cnt + 1] = last - p;
        list[3 * cnt + 2] = a;
      }
      ++cnt;
      dg += p * 31 + (last - p);
      dc += (p + 1) * a;
    }
    p = last > p ? last : p + 1;
  }
  if (digest)
    *digest = dg;
  if (dcap)
    *dcap = dc;
  return cnt;
}

/* Chain exit of a segment: the first chain position >= e starting from entry x. */
uint64_t orc_chain_exit(const orc_dfa *d, const uint8_t *buf, uint64_t n, uint64_t x, uint64_t e)
{
  uint64_t p = x;
  while (p < e && p < n)
  {
    uint32_t a;
    uint64_t len = orc_step(d, buf, n, p, &a);
    p += len ? len : 1;
  }
  return p;
}

/* ---- multi-threaded newline-split variant (CPU baseline "port") ---- */
typedef struct
{
  const orc_dfa *d;
  const uint8_t *buf;
  uint64_t a, b;
  uint64_t cnt, dg, dc;
} orc_job;

static void *orc_job_run(void *arg)
{
  orc_job *j = (orc_job *)arg;
  j->cnt = orc_find(j->d, j->buf + j->a, j->b - j->a, 0, j->a, &j->dg, &j->dc, NULL, 0);
  return NULL;
}

/* Splits at newlines (exact for patterns that cannot match '\n'). */
uint64_t orc_find_mt(const orc_dfa *d, const uint8_t *buf, uint64_t n, int threads, uint64_t *digest, uint64_t *dcap)
{
  orc_job jobs[256];
  pthread_t th[256];
  uint64_t cut[257];
  uint64_t cnt = 0, dg = 0, dc = 0;
  int i;
  if (threads < 1)
    threads = 1;
  if (threads > 256)
    threads = 256;
  cut[0] = 0;
  cut[threads] = n;
  for (i = 1; i < threads; ++i)
  {
    uint64_t c = n / threads * i;
    if (c < cut[i - 1])
      c = cut[i - 1];
    while (c < n && c > 0 && buf[c - 1] != '\n')
      ++c;
    cut[i] = c;
  }
  for (i = 0; i < threads; ++i)
  {
    jobs[i].d = d;
    jobs[i].buf = buf;
    jobs[i].a = cut[i];
    jobs[i].b = cut[i + 1];
    pthread_create(&th[i], NULL, orc_job_run, &jobs[i]);
  }
  for (i = 0; i < threads; ++i)
  {
    pthread_join(th[i], NULL);
    cnt += jobs[i].cnt;
    dg += jobs[i].dg;
    dc += jobs[i].dc;
  }
  if (digest)
    *digest = dg;
  if (dcap)
    *dcap = dc;
  return cnt;
}

void orc_gen(int kind, uint64_t seed, uint64_t off, uint8_t *buf, uint64_t len)
{
  gen_fill(kind, seed, off, buf, len);
}

/*
 * Binary-file detection.
 *
 * orc_isutf8 -- reflex::isutf8(s, s + n), restated from the reference's scalar
 *   loop (lib/simd.cpp:391-418): skip ASCII > 0; a lead must be c2..f4 and is
 *   followed by 1, 2 or 3 continuation bytes (80..bf) by its range (c2, e0,
 *   f0); NUL and everything else fail.  The SIMD paths (simd.cpp:174-300,
 *   simd_avx2.cpp:82-150) accept the same language; tests/test_oracle.py pins
 *   this against the compiled reference on the golden cases.
 * orc_utf8_first_bad -- the first failing position under the same language,
 *   in the local form the GPU kernel uses (a byte needs a continuation iff one
 *   of the 3 bytes before it is a lead announcing one; the end needs none):
 *   n + 1 when valid, n for a sequence cut off by the end.
 * orc_init_window -- GrepWorker::init_is_binary's trim of a trailing UTF-8
 *   sequence (src/ugrep.cpp:3998-4015): returns -1 for "binary", else the
 *   number of bytes to judge.
 */
int orc_isutf8(const uint8_t *s, uint64_t n)
{
  const uint8_t *e = s + n;
  while (s < e)
  {
    int8_t c = 0;
    while (s < e && (c = (int8_t)*s) > 0)
      ++s;
    if (s++ >= e)
      break;
    if (c < -62 || c > -12 || s >= e || (*s++ & 0xc0) != 0x80)
      return 0;
    if (c >= -32 && (s >= e || (*s++ & 0xc0) != 0x80))
      return 0;
    if (c >= -16 && (s >= e || (*s++ & 0xc0) != 0x80))
      return 0;
  }
  return 1;
}

uint64_t orc_utf8_first_bad(const uint8_t *s, uint64_t n)
{
  uint64_t i;
  for (i = 0; i <= n; ++i)
  {
    int need = (i >= 1 && s[i - 1] >= 0xc0) || (i >= 2 && s[i - 2] >= 0xe0) || (i >= 3 && s[i - 3] >= 0xf0);
    if (i == n)
      return need ? n : n + 1;
    uint8_t c = s[i];
    int cont = (c & 0xc0) == 0x80;
    int valid = (c >= 0x01 && c <= 0x7f) || cont || (c >= 0xc2 && c <= 0xf4);
    if (!valid || need != cont)
      return i;
  }
  return n + 1;
}

int64_t orc_init_window(const uint8_t *buf, uint64_t avail)
{
  if (avail == 0)
    return 0;
  if ((buf[avail - 1] & 0x80) == 0x80)
  {
    uint64_t k = avail < 4 ? avail : 4;
    while (k > 0 && (buf[--avail] & 0xc0) == 0x80)
      --k;
    if ((buf[avail] & 0xc0) != 0xc0)
      return -1;
  }
  return (int64_t)avail;
}
