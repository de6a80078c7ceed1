// device_common.hpp -- device building blocks shared by the scan kernels:
// flattened DFA table lookup, the exact FIND walk, match emitters, and the
// chain step/merge used to stitch speculative pieces.
#pragma once
#include "scan_kernels.hpp"

namespace ugpu {

// ---------------------------------------------------------------- tables
template <int FMT>
struct Tab {
  const uint16_t* trans;
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

// bytes [base, lend) are staged in LDS; anything else is read from global
struct Win {
  const uint8_t* lds;
  uint64_t base, lend;
  const uint8_t* g;
  uint64_t rend;
  uint32_t eof;
};

// Longest match starting at p (0 = none).  `le` = entry of the last accepting
// state (its row identifies the accept index).  Mirrors the reference walk:
// TAKE on entering an accepting state (lib/matcher.cpp:207-217), stop on HALT
// (:528-541) or EOF (:460-465).
template <int FMT>
__device__ __forceinline__ uint64_t walk(const Tab<FMT>& T, const Win& w, uint64_t p, uint32_t& le, uint32_t& ovf)
{
  uint32_t s = T.start;
  uint64_t q = p, last = p;
  le = 0;
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

struct Ctx {
  const uint32_t* caps;
  uint32_t log_row;
  int64_t delta;
};

struct CountEm {
  uint64_t cnt = 0, dg = 0, dc = 0;
  __device__ __forceinline__ void put(const Ctx& c, uint64_t pos, uint64_t len, uint32_t le, int sign)
  {
    uint64_t st = pos + (uint64_t)c.delta;
    uint64_t cap = c.caps[le >> c.log_row];
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
    if (idx < capacity) {
      start[idx] = pos + (uint64_t)c.delta;
      len[idx] = (uint32_t)l;
      cap[idx] = c.caps[le >> c.log_row];
    } else {
      overflow = 1;
    }
    ++idx;
  }
};

// One step of the FIND chain from p: the longest match at p (emitted with
// `sign`, then the chain continues at its end) or p+1.
template <int FMT, class Em>
__device__ __forceinline__ uint64_t chain_step(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t p, Em& em,
                                               int sign, uint32_t& ovf)
{
  uint32_t le;
  const uint64_t len = walk<FMT>(T, w, p, le, ovf);
  if (len) {
    em.put(c, p, len, le, sign);
    return p + len;
  }
  return p + 1;
}

// Re-enter [.., e) at xn instead of xo.  Adds (true - speculative) matches to em.
// Returns true if the chains met (exit unchanged), else sets nexit.
template <int FMT>
__device__ __forceinline__ bool merge(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t xo, uint64_t xn,
                                      uint64_t e, CountEm& em, uint64_t& nexit, uint32_t& ovf)
{
  uint64_t po = xo, pn = xn;
  for (;;) {
    if (po == pn) return true;
    if (po >= e && pn >= e) {
      nexit = pn;
      return false;
    }
    if (po < pn)
      po = chain_step<FMT>(T, w, c, po, em, -1, ovf);
    else
      pn = chain_step<FMT>(T, w, c, pn, em, +1, ovf);
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
