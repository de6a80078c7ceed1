/*
 * oracle/gen.h -- TEST INFRASTRUCTURE (oracle side). Host restatement of the
 * synthetic corpus generators used by the benchmark configs.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * anything under oracle/.  The product has its own device-side generator
 * (ugrep_amd/csrc/gen.hip); tests check that both produce identical bytes.
 *
 * Corpus model: the stream is cut into independent 64-byte CELLS; cell c is a
 * pure function of (seed, c) so that GPUs generate any shard in parallel and the
 * host regenerates any slice for golden digests.  Words/tokens flow across cell
 * boundaries when a cell does not end in a separator, so matches do cross cell,
 * tile, block and shard boundaries.
 *
 * Kinds:
 *   GEN_WORDS    (C2)  words of U{1..10} letters [a-z], single spaces, cell
 *                      ends in '\n' with p=1/2.
 *   GEN_PLANTED  (C2') letters from [a-z]\{b,f}; with p=1/64 a cell carries one
 *                      planted "foo"/"bar"/"baz" at offset < 61: the match count
 *                      for foo|bar|baz equals the planted count (known answer).
 *   GEN_CODE     (C3)  C-like tokens: identifiers (55%), numbers (10%),
 *                      operators (25%), spaces (10%).
 *   GEN_UTF8     (C4)  UTF-8 words: ASCII, Latin-1, Greek, Cyrillic, CJK, plus
 *                      '€' and punctuation; multibyte chars never cross cells.
 */
#ifndef UGREP_ORACLE_GEN_H
#define UGREP_ORACLE_GEN_H

#include <stdint.h>
#include <string.h>

#define GEN_WORDS   1
#define GEN_PLANTED 2
#define GEN_CODE    3
#define GEN_UTF8    4

#define GEN_CELL 64

static inline uint64_t gen_sm64(uint64_t *s)
{
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline int gen_put_utf8(uint8_t *out, int pos, uint32_t cp)
{
  /* returns bytes written, 0 if it does not fit in the cell */
  if (cp < 0x80) { if (pos + 1 > GEN_CELL) return 0; out[pos] = (uint8_t)cp; return 1; }
  if (cp < 0x800) {
    if (pos + 2 > GEN_CELL) return 0;
    out[pos] = (uint8_t)(0xC0 | (cp >> 6)); out[pos + 1] = (uint8_t)(0x80 | (cp & 0x3F)); return 2;
  }
  if (pos + 3 > GEN_CELL) return 0;
  out[pos] = (uint8_t)(0xE0 | (cp >> 12)); out[pos + 1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
  out[pos + 2] = (uint8_t)(0x80 | (cp & 0x3F)); return 3;
}

/* Generate the 64 bytes of cell `cell`. */
static inline void gen_cell(int kind, uint64_t seed, uint64_t cell, uint8_t out[GEN_CELL])
{
  static const char planted_alpha[] = "acdeghijklmnopqrstuvwxyz";           /* 24 letters */
  static const char id_first[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz_"; /* 53 */
  static const char id_rest[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz_0123456789"; /* 63 */
  static const char ops[] = "(){};,=+-*/<>.";                             /* 14 */
  static const char punct[] = ".,;:!?";                                   /* 6 */
  uint64_t s = seed ^ (cell * 0xD1B54A32D192ED03ull);
  uint64_t x = gen_sm64(&s);
  int pos = 0;
  int i;
  if (kind == GEN_WORDS || kind == GEN_PLANTED)
  {
    while (pos < GEN_CELL)
    {
      uint64_t r = gen_sm64(&s);
      int wl = 1 + (int)(r % 10);
      uint64_t r2 = gen_sm64(&s);
      for (i = 0; i < wl && pos < GEN_CELL; ++i)
      {
        uint32_t sl = (uint32_t)((r2 >> (6 * i)) & 63);
        out[pos++] = kind == GEN_WORDS ? (uint8_t)('a' + sl % 26) : (uint8_t)planted_alpha[sl % 24];
      }
      if (pos < GEN_CELL)
        out[pos++] = ' ';
    }
    if (kind == GEN_PLANTED && ((x >> 1) & 63) == 0)
    {
      static const char *const words[3] = { "foo", "bar", "baz" };
      uint32_t off = (uint32_t)((x >> 8) % 61);
      const char *w = words[(x >> 16) % 3];
      out[off] = (uint8_t)w[0]; out[off + 1] = (uint8_t)w[1]; out[off + 2] = (uint8_t)w[2];
    }
    if (x & 1)
      out[GEN_CELL - 1] = '\n';
    return;
  }
  if (kind == GEN_CODE)
  {
    while (pos < GEN_CELL)
    {
      uint64_t r = gen_sm64(&s);
      uint32_t t = (uint32_t)(r % 100);
      if (t < 55)
      {
        int len = 1 + (int)((r >> 8) % 16);
        uint64_t r2 = gen_sm64(&s);
        uint64_t r3 = gen_sm64(&s);
        for (i = 0; i < len && pos < GEN_CELL; ++i)
        {
          uint32_t sl = (uint32_t)(((i < 10 ? r2 >> (6 * i) : r3 >> (6 * (i - 10)))) & 63);
          out[pos++] = i == 0 ? (uint8_t)id_first[sl % 53] : (uint8_t)id_rest[sl % 63];
        }
      }
      else if (t < 65)
      {
        int len = 1 + (int)((r >> 8) % 6);
        uint64_t r2 = gen_sm64(&s);
        for (i = 0; i < len && pos < GEN_CELL; ++i)
          out[pos++] = (uint8_t)('0' + ((r2 >> (6 * i)) & 63) % 10);
      }
      else if (t < 90)
      {
        out[pos++] = (uint8_t)ops[(r >> 8) % 14];
      }
      else
      {
        out[pos++] = ' ';
      }
      if (t < 65 && pos < GEN_CELL && ((r >> 16) & 1))
        out[pos++] = ' ';
    }
    if (x & 1)
      out[GEN_CELL - 1] = '\n';
    return;
  }
  /* GEN_UTF8 */
  while (pos < GEN_CELL)
  {
    uint64_t r = gen_sm64(&s);
    uint32_t t = (uint32_t)(r % 100);
    if (t < 90)
    {
      int len = 1 + (int)((r >> 8) % 8);
      uint64_t r2 = gen_sm64(&s);
      for (i = 0; i < len; ++i)
      {
        uint32_t sl = (uint32_t)((r2 >> (7 * i)) & 127);
        uint32_t cp;
        int n;
        if (t < 40)
          cp = (sl & 64) ? 'A' + sl % 26 : 'a' + sl % 26;
        else if (t < 55)
        {
          cp = 0xC0 + (sl & 63);
          if (cp == 0xD7 || cp == 0xF7)
            cp = 0xE9;
        }
        else if (t < 70)
          cp = 0x3B1 + sl % 25;
        else if (t < 80)
          cp = 0x430 + (sl & 31);
        else
          cp = 0x4E00 + ((uint32_t)((r2 >> (7 * i)) & 0xFFFF) % 0x5000);
        n = gen_put_utf8(out, pos, cp);
        if (n == 0)
          break;
        pos += n;
      }
    }
    else if (t < 95)
    {
      if ((r >> 8) & 1)
      {
        int n = gen_put_utf8(out, pos, 0x20AC); /* € */
        if (n == 0)
          break;
        pos += n;
      }
      else
      {
        out[pos++] = (uint8_t)punct[(r >> 9) % 6];
      }
    }
    if (pos < GEN_CELL)
      out[pos++] = ' ';
  }
  while (pos < GEN_CELL)
    out[pos++] = ' ';
  if ((x & 1) && out[GEN_CELL - 1] < 0x80)
    out[GEN_CELL - 1] = '\n';
}

/* Fill buf[0..len) with bytes [off, off+len) of the corpus stream. */
static inline void gen_fill(int kind, uint64_t seed, uint64_t off, uint8_t *buf, uint64_t len)
{
  uint8_t cellbuf[GEN_CELL];
  uint64_t end = off + len;
  uint64_t p = off;
  while (p < end)
  {
    uint64_t cell = p / GEN_CELL;
    uint64_t cs = cell * GEN_CELL;
    uint64_t a = p - cs;
    uint64_t b = end - cs < GEN_CELL ? end - cs : GEN_CELL;
    gen_cell(kind, seed, cell, cellbuf);
    memcpy(buf + (p - off), cellbuf + a, (size_t)(b - a));
    p = cs + b;
  }
}

#endif
