// scan_kernels.hip -- CDNA4 (gfx950) kernels of the FIND engine.  See
// scan_kernels.hpp for the chain/stitch scheme.
//
// Reference hot loops replaced here:
//   * needle prefilter simd_advance_pattern_pinN_*_avx2 (lib/matcher_avx2.cpp:
//     303-799) / simd_advance_string_* (lib/matcher_avx512bw.cpp:281-463):
//     per-lane SWAR test of the segment's 64 staged bytes against the DFA's
//     first/second-byte terms -> 64-bit candidate mask (filter_mask);
//   * DFA opcode interpreter (lib/matcher.cpp:125-546): one dependent LDS
//     lookup per byte in the flattened table (walk);
//   * FIND restart/accept logic (lib/matcher.cpp:621-746): chain_step.
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

// One step of the FIND chain from p (< e).  With the prefilter (FILT), positions
// whose byte cannot start a match are skipped via the candidate mask of the
// lane's 64-byte segment [sa, sa+64): their step is p+1 with no match.
template <int FMT, bool FILT, class Em>
__device__ __forceinline__ uint64_t chain_step(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t p,
                                               uint64_t sa, uint64_t e, uint64_t mask, Em& em, int sign,
                                               uint32_t& ovf)
{
  uint64_t c0 = p;
  if constexpr (FILT) {
    uint64_t off = p - sa;
    uint64_t m = off < 64 ? (mask & (~0ull << off)) : 0ull;
    if (m == 0) return e;
    c0 = sa + (uint64_t)__builtin_ctzll(m);
  }
  uint32_t le;
  uint64_t len = walk<FMT>(T, w, c0, le, ovf);
  if (len) {
    em.put(c, c0, len, le, sign);
    return c0 + len;
  }
  return c0 + 1;
}

template <int FMT, bool FILT, class Em>
__device__ __forceinline__ uint64_t run_seg(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t x, uint64_t sa,
                                            uint64_t e, uint64_t mask, Em& em, uint32_t& ovf)
{
  uint64_t p = x;
  while (p < e) p = chain_step<FMT, FILT>(T, w, c, p, sa, e, mask, em, +1, ovf);
  return p;
}

// Re-enter [.., e) at xn instead of xo.  Adds (true - speculative) matches to em.
// Returns true if the chains met (exit unchanged), else sets nexit.
template <int FMT, bool FILT>
__device__ __forceinline__ bool merge(const Tab<FMT>& T, const Win& w, const Ctx& c, uint64_t xo, uint64_t xn,
                                      uint64_t sa, uint64_t e, uint64_t mask, CountEm& em, uint64_t& nexit,
                                      uint32_t& ovf)
{
  uint64_t po = xo, pn = xn;
  for (;;) {
    if (po == pn) return true;
    if (po >= e && pn >= e) {
      nexit = pn;
      return false;
    }
    if (po < pn)
      po = chain_step<FMT, FILT>(T, w, c, po, sa, e, mask, em, -1, ovf);
    else
      pn = chain_step<FMT, FILT>(T, w, c, pn, sa, e, mask, em, +1, ovf);
  }
}

// SWAR candidate mask of a 64-byte LDS segment: bit i set iff byte i may start
// a match, i.e. B[i] in A, or B[i] in B and B[i+1] in C (tables.hpp).  A set
// test is an OR over (mask, value) terms, each an exact per-byte zero test
// ((t & 0x7f..) + 0x7f..) | t  (bit 7 = byte nonzero, no borrow leakage).
// `nxt` holds the 4 bytes after the segment (the pair test reads byte 64).
// The term counts are compile-time (filter code FC, see fcode()).
constexpr int fcode(int na, int nb, int nc) { return 1 + na * 9 + nb * 3 + nc; }

struct Filter {
  uint32_t tm[12], tv[12];
};

__device__ __forceinline__ uint32_t nz_bytes(uint32_t t) { return ((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t; }

// bit 7 of each byte set iff the byte matches NO term of the set [o, o+N)
template <int N>
__device__ __forceinline__ uint32_t no_match(const Filter& F, int o, uint32_t x)
{
  uint32_t r = 0xffffffffu;
#pragma unroll
  for (int i = 0; i < N; ++i) r &= nz_bytes((x & F.tm[o + i]) ^ F.tv[o + i]);
  return r;
}

template <int FC>
__device__ __forceinline__ uint64_t filter_mask(const uint8_t* seg, uint32_t nxt, const Filter& F)
{
  constexpr int NA = (FC - 1) / 9, NB = ((FC - 1) / 3) % 3, NC = (FC - 1) % 3;
  const uint4* v = reinterpret_cast<const uint4*>(seg);
  uint32_t wd[17];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint4 x = v[i];
    wd[4 * i] = x.x;
    wd[4 * i + 1] = x.y;
    wd[4 * i + 2] = x.z;
    wd[4 * i + 3] = x.w;
  }
  wd[16] = nxt;
  uint32_t lo = 0, hi = 0;
  uint32_t noC_next = NC ? no_match<NC>(F, 8, wd[0]) : 0u;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t noBC = 0xffffffffu;
    if constexpr (NB > 0) {
      const uint32_t noC = noC_next;
      noC_next = NC ? no_match<NC>(F, 8, wd[j + 1]) : 0u;
      // byte i of the shifted word = C-test of byte i+1
      const uint32_t noCs = __builtin_amdgcn_alignbyte(noC_next, noC, 1);
      noBC = no_match<NB>(F, 4, wd[j]) | noCs;
    }
    const uint32_t cand = ~(no_match<NA>(F, 0, wd[j]) & noBC) & 0x80808080u;
    const uint32_t nib = (((cand >> 7) * 0x00204081u) >> 21) & 0xfu;
    if (j < 8)
      lo |= nib << (4 * j);
    else
      hi |= nib << (4 * (j - 8));
  }
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t lowbits(uint64_t k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }

__device__ __forceinline__ uint64_t clampu(uint64_t v, uint64_t a, uint64_t b) { return v < a ? a : (v > b ? b : v); }

__device__ __forceinline__ uint4 load_chunk(const uint8_t* g, uint64_t pos, uint64_t rend)
{
  // A 16-byte aligned chunk holding at least one readable byte lies in a mapped
  // page, so it is loaded whole; bytes >= rend are never consulted.
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  if (pos < rend) {
    v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(g + pos));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- scan kernel
template <int FMT, int FC, bool WRITE>
__global__ __launch_bounds__(kBlock) void scan_kernel(ScanParams P)
{
  constexpr bool FILT = FC != 0;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint64_t* ex = reinterpret_cast<uint64_t*>(smem + kTile + kHalo);
  uint64_t* red = ex + kBlock;  // 3 * 4 u64 reduction scratch
  uint16_t* ltrans = reinterpret_cast<uint16_t*>(red + 16);
  uint8_t* lcls = reinterpret_cast<uint8_t*>(ltrans + P.ntrans_pad);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;

  // stage the transition table (and class map) once per block
  {
    const uint4* src = reinterpret_cast<const uint4*>(P.trans);
    uint4* dst = reinterpret_cast<uint4*>(ltrans);
    for (uint32_t i = tid; i < P.ntrans_pad / 8; i += kBlock) dst[i] = src[i];
    if constexpr (FMT == 1) {
      if (tid < 16) reinterpret_cast<uint4*>(lcls)[tid] = reinterpret_cast<const uint4*>(P.cls)[tid];
    }
  }
  const Tab<FMT> T{ltrans, lcls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  Filter F;
  if constexpr (FILT) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      F.tm[i] = P.tm[i];
      F.tv[i] = P.tv[i];
    }
  }

  const uint64_t b = blockIdx.x;
  uint64_t tb = P.t0 + b * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t blo = clampu(tb * kTile, P.lo, P.hi);
  const uint64_t bhi = clampu(te * kTile, P.lo, P.hi);
  uint64_t x0 = WRITE ? P.entries[b] : blo;

  Win w;
  w.lds = tile;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0;
  CountEm tot;
  uint64_t wbase = WRITE ? P.out_base[b] : 0;
  uint32_t wover = 0;

  uint4 pf[4], ph = make_uint4(0, 0, 0, 0);
  auto prefetch = [&](uint64_t t) {
    const uint64_t ts = t * kTile;
#pragma unroll
    for (int k = 0; k < 4; ++k) pf[k] = load_chunk(P.g, ts + 16ull * (tid + k * kBlock), P.rend);
    if (tid < kHalo / 16) ph = load_chunk(P.g, ts + kTile + 16ull * tid, P.rend);
  };
  if (tb < te) prefetch(tb);

  for (uint64_t t = tb; t < te; ++t) {
    const uint64_t ts = t * kTile;
    __syncthreads();  // previous tile fully consumed
    {
      uint4* d = reinterpret_cast<uint4*>(tile);
#pragma unroll
      for (int k = 0; k < 4; ++k) d[tid + k * kBlock] = pf[k];
      if (tid < kHalo / 16) d[kTile / 16 + tid] = ph;
    }
    __syncthreads();
    if (t + 1 < te) prefetch(t + 1);

    w.base = ts;
    w.lend = ts + kTile + kHalo;
    const uint64_t sa = ts + (uint64_t)tid * kSeg;
    const uint64_t s = clampu(sa, blo, bhi);
    const uint64_t e = clampu(sa + kSeg, blo, bhi);
    uint64_t mask = 0;
    if (P.ablate == 1) {  // keep x0 consistent so fix_kernel has nothing to stitch
      tot.cnt += tile[tid];
      x0 = clampu(ts + kTile, blo, bhi);
      continue;
    }
    if constexpr (FILT) {
      const uint32_t nxt = *reinterpret_cast<const uint32_t*>(tile + tid * kSeg + kSeg);
      mask = filter_mask<FC>(tile + tid * kSeg, nxt, F);
      mask &= lowbits(e - sa) & ~lowbits(s - sa);
    }
    if (P.ablate == 2) {
      tot.cnt += __popcll(mask);
      x0 = clampu(ts + kTile, blo, bhi);
      continue;
    }
    uint64_t x = (tid == 0) ? x0 : s;
    CountEm la;
    const uint64_t xe = run_seg<FMT, FILT>(T, w, C, x, sa, e, mask, la, ovf);
    // The true chain enters lane k at lane k-1's exit.  It differs from the
    // speculative entry s_k only where some lane's chain left its segment past
    // the segment end (a match crossing the boundary).
    if (__syncthreads_or(xe > e)) {
      ex[tid] = xe;
      // resolve the true chain entry of every lane (rounds propagate left->right)
      for (;;) {
        __syncthreads();
        const uint64_t nx = (tid == 0) ? x0 : ex[tid - 1];
        const bool ch = nx != x;
        __syncthreads();
        if (ch) {
          uint64_t ne;
          if (!merge<FMT, FILT>(T, w, C, x, nx, sa, e, mask, la, ne, ovf)) ex[tid] = ne;
          x = nx;
        }
        if (!__syncthreads_or(ch)) break;
      }
      x0 = ex[kBlock - 1];
    } else {
      x0 = clampu(ts + kTile, blo, bhi);  // == exit of the last lane
    }
    if constexpr (WRITE) {
      // exclusive prefix of the lanes' match counts, then re-walk and store
      uint64_t v = la.cnt, incl = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      if (lane == 63) red[wid] = incl;
      __syncthreads();
      uint64_t off = 0, all = 0;
#pragma unroll
      for (int k = 0; k < kBlock / 64; ++k) {
        off += (k < wid) ? red[k] : 0;
        all += red[k];
      }
      WriteEm we{wbase + off + incl - v, P.out_capacity, P.out_start, P.out_len, P.out_cap};
      run_seg<FMT, FILT>(T, w, C, x, sa, e, mask, we, ovf);
      wover |= we.overflow;
      wbase += all;
      __syncthreads();  // red reused next tile
    } else {
      tot.cnt += la.cnt;
      tot.dg += la.dg;
      tot.dc += la.dc;
    }
  }

  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (wover) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  if constexpr (!WRITE) {
    const uint64_t c = wave_sum(tot.cnt), d = wave_sum(tot.dg), dc = wave_sum(tot.dc);
    __syncthreads();
    if (lane == 0) {
      red[wid] = c;
      red[4 + wid] = d;
      red[8 + wid] = dc;
    }
    __syncthreads();
    if (tid == 0) {
      BlockRec r;
      r.entry = blo;
      r.exit = x0;
      r.cnt = red[0] + red[1] + red[2] + red[3];
      r.dg = red[4] + red[5] + red[6] + red[7];
      r.dc = red[8] + red[9] + red[10] + red[11];
      r.pad0 = r.pad1 = r.pad2 = 0;
      P.recs[b] = r;
    }
  }
}

// ---------------------------------------------------------------- fix kernel
// One workgroup re-enters every block whose speculative entry differs from its
// predecessor's exit (merge over the block's byte range, bytes from global),
// repeating until no exit changes; then reduces the totals and produces the
// exact block entries and output bases for the OFFSETS pass.
template <int FMT>
__global__ __launch_bounds__(kFixThreads) void fix_kernel(ScanParams P)
{
  __shared__ uint64_t ent[kMaxGrid], exi[kMaxGrid];
  __shared__ uint64_t wred[3][kFixThreads / 64];
  __shared__ uint64_t wscan[kFixThreads / 64];
  constexpr int PER = kMaxGrid / kFixThreads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = (int)P.grid;
  const Tab<FMT> T{P.trans, P.cls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  Win w;
  w.lds = nullptr;
  w.base = 0;
  w.lend = 0;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0;

  uint64_t cnt[PER], dg[PER], dc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = tid * PER + j;
    if (b < G) {
      BlockRec r = P.recs[b];
      ent[b] = r.entry;
      exi[b] = r.exit;
      cnt[j] = r.cnt;
      dg[j] = r.dg;
      dc[j] = r.dc;
    } else {
      cnt[j] = dg[j] = dc[j] = 0;
    }
  }
  uint32_t rounds = 0;
  for (;;) {
    __syncthreads();
    uint64_t nx[PER];
    bool ch[PER], any = false;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int b = tid * PER + j;
      ch[j] = false;
      if (b > 0 && b < G) {
        nx[j] = exi[b - 1];
        ch[j] = nx[j] != ent[b];
        any |= ch[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (!ch[j]) continue;
      const uint64_t b = tid * PER + j;
      uint64_t tb = P.t0 + b * P.tpb;
      uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
      if (tb > te) tb = te;
      const uint64_t blo = clampu(tb * kTile, P.lo, P.hi);
      const uint64_t bhi = clampu(te * kTile, P.lo, P.hi);
      (void)blo;
      CountEm d;
      uint64_t ne;
      if (!merge<FMT, 0>(T, w, C, ent[b], nx[j], 0, bhi, 0, d, ne, ovf)) exi[b] = ne;
      ent[b] = nx[j];
      cnt[j] += d.cnt;
      dg[j] += d.dg;
      dc[j] += d.dc;
    }
    if (!__syncthreads_or(any)) break;
    ++rounds;
  }
  // totals + exclusive scan of block counts
  uint64_t mc = 0, md = 0, mdc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    mc += cnt[j];
    md += dg[j];
    mdc += dc[j];
  }
  uint64_t incl = mc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const uint64_t sd = wave_sum(md), sdc = wave_sum(mdc);
  if (lane == 63) wscan[wid] = incl;
  if (lane == 0) {
    wred[1][wid] = sd;
    wred[2][wid] = sdc;
  }
  __syncthreads();
  uint64_t off = 0;
  for (int k = 0; k < wid; ++k) off += wscan[k];
  uint64_t run = off + incl - mc;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = tid * PER + j;
    if (b < G) {
      P.out_base_out[b] = run;
      P.entries_out[b] = ent[b];
      run += cnt[j];
    }
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (tid == 0) {
    uint64_t c = 0, d = 0, e = 0;
    for (int k = 0; k < kFixThreads / 64; ++k) {
      c += wscan[k];
      d += wred[1][k];
      e += wred[2][k];
    }
    DevTotals* t = P.totals;
    t->count = c;
    t->digest = d;
    t->dcap = e;
    t->entry = ent[0];
    t->exit = exi[G - 1];
    t->rounds = rounds;
  }
}

// Shard-boundary stitch (multi-GPU): re-enter [lo, hi) at new_entry.
template <int FMT>
__global__ void chain_fix_kernel(ScanParams P, uint64_t old_entry, uint64_t new_entry)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const Tab<FMT> T{P.trans, P.cls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  Win w;
  w.lds = nullptr;
  w.base = 0;
  w.lend = 0;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0;
  CountEm d;
  uint64_t ne = 0;
  bool met = merge<FMT, 0>(T, w, C, old_entry, new_entry, 0, P.hi, 0, d, ne, ovf);
  DevTotals* t = P.totals;
  t->count = d.cnt;
  t->digest = d.dg;
  t->dcap = d.dc;
  t->entry = new_entry;
  t->exit = met ? ~0ull : ne;  // ~0 = exit unchanged
  t->flags = ovf ? UGPU_FLAG_HALO : 0;
  t->rounds = met ? 1 : 0;
}

// ---------------------------------------------------------------- launchers
template <int FMT, int FC, bool WRITE>
static hipError_t launch_one(const ScanParams& P, size_t smem, hipStream_t stream)
{
  static size_t attr_smem = 65536;
  if (smem > attr_smem) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&scan_kernel<FMT, FC, WRITE>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_smem = smem;
  }
  hipLaunchKernelGGL((scan_kernel<FMT, FC, WRITE>), dim3(P.grid), dim3(kBlock), smem, stream, P);
  return hipGetLastError();
}

// filter codes with instantiated kernels: NA + NB in {1, 2}, NC in {0, 1, 2} (tables.cpp)
#define UGPU_FOR_FCODES(X) \
  X(fcode(1, 0, 0)) X(fcode(2, 0, 0)) X(fcode(0, 1, 0)) X(fcode(0, 1, 1)) X(fcode(0, 1, 2)) X(fcode(1, 1, 0)) \
  X(fcode(1, 1, 1)) X(fcode(1, 1, 2)) X(fcode(0, 2, 0)) X(fcode(0, 2, 1)) X(fcode(0, 2, 2))

template <bool WRITE>
static hipError_t launch_byte(const ScanParams& P, int fc, size_t smem, hipStream_t stream)
{
  switch (fc) {
#define X(c) \
  case c: return launch_one<0, c, WRITE>(P, smem, stream);
    UGPU_FOR_FCODES(X)
#undef X
    default: return launch_one<0, 0, WRITE>(P, smem, stream);
  }
}

hipError_t launch_scan(const ScanParams& P, uint32_t format, bool filter, bool write, size_t smem,
                       hipStream_t stream)
{
  const int fc = filter ? fcode((int)P.nA, (int)P.nB, (int)P.nC) : 0;
  if (format == 0) return write ? launch_byte<true>(P, fc, smem, stream) : launch_byte<false>(P, fc, smem, stream);
  return write ? launch_one<1, 0, true>(P, smem, stream) : launch_one<1, 0, false>(P, smem, stream);
}

hipError_t launch_fix(const ScanParams& P, uint32_t format, hipStream_t stream)
{
  if (format == 0)
    hipLaunchKernelGGL(fix_kernel<0>, dim3(1), dim3(kFixThreads), 0, stream, P);
  else
    hipLaunchKernelGGL(fix_kernel<1>, dim3(1), dim3(kFixThreads), 0, stream, P);
  return hipGetLastError();
}

hipError_t launch_chain_fix(const ScanParams& P, uint32_t format, uint64_t old_entry, uint64_t new_entry,
                            hipStream_t stream)
{
  if (format == 0)
    hipLaunchKernelGGL(chain_fix_kernel<0>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  else
    hipLaunchKernelGGL(chain_fix_kernel<1>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  return hipGetLastError();
}

template <int FMT, int FC>
static hipError_t occ_one(size_t smem, int* n)
{
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, scan_kernel<FMT, FC, false>, kBlock, smem);
}

hipError_t scan_occupancy(uint32_t format, bool filter, size_t smem, int* n)
{
  // all filter variants share the same resource shape; the common C2 one answers
  if (format == 0) return filter ? occ_one<0, fcode(0, 1, 2)>(smem, n) : occ_one<0, 0>(smem, n);
  return occ_one<1, 0>(smem, n);
}

size_t scan_smem_bytes(uint32_t ntrans_pad, uint32_t format)
{
  size_t b = kTile + kHalo + sizeof(uint64_t) * (kBlock + 16) + sizeof(uint16_t) * ntrans_pad;
  if (format == 1) b += 256;
  return (b + 15) & ~size_t(15);
}

}  // namespace ugpu
