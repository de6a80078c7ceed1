// xg_kernel.hip -- FIND over restart-local tables whose walk "gap" is a
// function of the DFA state (tables.hpp, "gap transducer"): UTF-8 word
// patterns such as \w+ or \S+ (BASELINE config C4), and many literal or
// token patterns.
//
// What it replaces: the reference's FIND loop (lib/matcher.cpp:42-750) and its
// DFA walk (:125-546) for these tables; results are the same (count,
// digest = sum(31 start + len), dcap = sum((start + 1) cap)).
//
// Same lane/tile/wave scheme as xi_kernel.hip (1 KiB lane segments read
// directly from HBM, sync-byte exact lanes, tails to the next sync byte, edge
// tiles in a one-wave kernel), with a different per-byte step: a byte costs a
// class lookup (class tables) and one u16 transition lookup in LDS, and the
// match bookkeeping is incremental -- every accept adds its gap + 1 bytes to
// the current match, the first accept of a walk (tracked by one bit per lane)
// counts the match and its start q + 1 - (gap + 1).  So no walk start or last
// accept registers, and no work at the death of a walk:
//   count = #F, sum start = sum_F (q + 1) - sum_F L, sum len = sum L.
#include "device_common.hpp"
#include "tables.hpp"

namespace ugpu {

namespace {

constexpr int kGS = 1024;          // lane segment bytes
constexpr int kGTile = 64 * kGS;   // wave tile
constexpr int kGBlk = 64;          // bytes per block (4 x 16 B per lane, double buffered)
constexpr int kGLd = kGBlk / 16;
constexpr int kGBlocks = kGS / kGBlk;
#ifndef UGPU_XG_WAVES
#define UGPU_XG_WAVES 16
#endif
constexpr int kGWaves = UGPU_XG_WAVES;  // waves per workgroup: one staged table per CU
constexpr int kGMaxEntries = 65536;  // u16 table entries (128 KB)

__device__ __forceinline__ uint4 gload16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
  return uint4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t grsrc(const uint8_t* base, uint64_t readable)
{
  const uint32_t n = readable < 0x7fffff00ull ? (uint32_t)readable : 0x7fffff00u;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)n), 0x00020000);
}

__device__ __forceinline__ uint32_t gsel4(const uint4& v, uint32_t j)
{
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// Tables in LDS: transitions (u16), class x 2 (FMT 1), sync flags.
template <int FMT>
struct GTab {
  const uint16_t* xg;
  const uint8_t* c2;
  const uint8_t* sy;
  uint32_t rowmask;
  uint32_t start_row;
  // entry after byte k of dword w from entry m
  template <int K>
  __device__ __forceinline__ uint32_t step(uint32_t m, uint32_t w) const
  {
    if constexpr (FMT == 1) {
      const uint32_t c = c2[(w >> (8 * K)) & 0xffu];
      return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(xg) + (((m & rowmask) << 1) | c));
    } else {
      return xg[__builtin_amdgcn_perm(m, w, 0x0c0c0500u | (uint32_t)K)];  // (m & 0xff00) | byte
    }
  }
  __device__ __forceinline__ uint32_t stepb(uint32_t m, uint32_t b) const
  {
    if constexpr (FMT == 1)
      return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(xg) +
                                                (((m & rowmask) << 1) | c2[b]));
    else
      return xg[(m & 0xff00u) | b];
  }
  __device__ __forceinline__ bool in_walk(uint32_t m) const { return (m & rowmask) != start_row; }
};

// Lane sums (lane-relative positions r): cnt = #F, sq = sum_F (r + 1),
// sfl = sum_F L, sl = sum L.
struct GSum {
  uint32_t cnt = 0, sq = 0, sfl = 0, sl = 0;
};

__device__ __forceinline__ void gfold(const GSum& a, uint64_t base, uint64_t& cnt, uint64_t& sst, uint64_t& len)
{
  cnt += a.cnt;
  // sum of starts r + 1 - L; signed: in a tail chunk a match may start before the chunk base
  sst += (uint64_t)a.cnt * base + (uint64_t)(int64_t)(int32_t)(a.sq - a.sfl);
  len += a.sl;
}

// One byte of the main loop.  MASK: events of the lane's head (up to and
// including its first sync byte) are dropped.  off1 = the byte's offset in its
// block + 1 (a constant once unrolled): sq gets f (off1) here and f bb per block.
template <int FMT, int K, bool MASK>
__device__ __forceinline__ void gbyte(const GTab<FMT>& T, uint32_t w, uint32_t& m, uint32_t& acc, GSum& s,
                                      uint32_t bb, uint32_t off1, bool& synced, uint32_t& fs)
{
  const uint32_t e = T.template step<K>(m, w);
  // bit 2 (XG_A): the new state accepts; d2 bit 2: the walk died here
  const uint32_t d2 = e << 2;
  uint32_t f = e & (d2 | ~acc) & XG_A;  // first accept of the walk (XG_A or 0; a death restarts it)
  acc = e | (acc & ~d2);                // bit 2: the walk has accepted
  uint32_t L = (e >> XG_LSHIFT) & 7u;
  if constexpr (MASK) {
    const uint32_t y = T.sy[(w >> (8 * K)) & 0xffu];
    if (!synced) {
      f = 0;
      L = 0;
      if (y) fs = bb + off1 - 1;
    }
    synced = synced || y != 0;
  }
  s.cnt += f;  // (sums of f are 4x: XG_A == 4)
  s.sq += __umul24(f, off1);
  s.sfl += __umul24(f, L);
  s.sl += L;
  m = e;
}

// acc: bit 2 = the walk has accepted (main-loop form; the tail's form is bit 0)
template <int FMT, bool MASK>
__device__ __forceinline__ void gblock(const GTab<FMT>& T, const uint4 (&v)[kGLd], uint32_t& m, uint32_t& acc,
                                       GSum& s4, bool& synced, uint32_t& fs, uint32_t bb)
{
  GSum& s = s4;  // cnt, sq and sfl are scaled by 4 (f = XG_A or 0); sl is exact
  const uint32_t c0 = s.cnt;
#pragma unroll
  for (int k = 0; k < kGLd; ++k) {
    const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t o1 = 16u * k + 4u * j + 1u;
      gbyte<FMT, 0, MASK>(T, w[j], m, acc, s, bb, o1, synced, fs);
      gbyte<FMT, 1, MASK>(T, w[j], m, acc, s, bb, o1 + 1, synced, fs);
      gbyte<FMT, 2, MASK>(T, w[j], m, acc, s, bb, o1 + 2, synced, fs);
      gbyte<FMT, 3, MASK>(T, w[j], m, acc, s, bb, o1 + 3, synced, fs);
    }
  }
  s.sq += __umul24(s.cnt - c0, bb);  // the block's starts at offset bb
}

__device__ __forceinline__ uint32_t gdist(uint64_t lim, uint64_t base)  // lim - base clamped to [0, 64]
{
  return lim > base ? (lim - base < 64 ? (uint32_t)(lim - base) : 64u) : 0u;
}

// Tail of a lane from tile offset o (its segment end): walk until a sync
// byte has been read.  Returns the coverage end (as xi_kernel's xtail).
template <int FMT>
__device__ __forceinline__ uint64_t gtail(const GTab<FMT>& T, const uint8_t* g, uint64_t ts, uint32_t o,
                                          uint32_t& m, uint32_t& acc, uint64_t& cnt, uint64_t& sst,
                                          uint64_t& len, uint64_t hi, uint64_t rend, uint32_t at_eof, uint32_t& ovf,
                                          bool act)
{
  // (sums per 16-byte chunk, folded into 64-bit totals at the chunk's base:
  // a tail may run far when sync bytes are rare, e.g. \D over text)
  uint64_t xit = ~0ull, last = 0;
  const uint64_t rend16 = (rend + 15) & ~uint64_t(15);
  uint4 vn = gload16(grsrc(g + ts, rend16 > ts ? rend16 - ts : 0), o);
  for (uint64_t c = 0; __ballot(act); c += 16) {
    const uint4 v = vn;
    const uint64_t cb = ts + c + 16;
    vn = gload16(grsrc(g + cb, rend16 > cb ? rend16 - cb : 0), o);
    const uint64_t base = ts + o + c;
    const uint32_t dh = gdist(hi, base), dr = gdist(rend, base);
    GSum s;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      bool go = act;
      const bool walk = T.in_walk(m);
      if (go && k >= dh && !walk) {  // nothing crosses into this byte: the chain is here
        xit = base + k;
        act = go = false;
      }
      if (go && k >= dr) {  // readable end: at EOF the walk ends there
        if (!at_eof && walk) ovf |= 1;
        xit = k >= dh ? (last > hi ? last : hi) : base + k;
        act = go = false;
      }
      const uint32_t b = (gsel4(v, k >> 2) >> (8 * (k & 3))) & 0xffu;
      const uint32_t e = T.stepb(m, b);
      if (go) {
        const uint32_t t = e >> 2;
        const uint32_t f = t & (e | ~acc) & 1u;
        const uint32_t L = (e >> XG_LSHIFT) & 7u;
        if (k >= dh && (e & XT_DEAD)) {  // the walk crossing hi died here
          xit = last > hi ? last : hi;
          act = false;
        } else {
          s.cnt += f;
          s.sq += __umul24(f, k + 1);
          s.sfl += __umul24(f, L);
          s.sl += L;
          if (t & 1u) last = base + k + 1;
          acc = t | (acc & ~e);
          if (k < dh && T.sy[b]) {
            xit = base + k + 1;
            act = false;
          }
        }
        m = e;
      }
    }
    gfold(s, base, cnt, sst, len);
  }
  return xit;
}

// Exact per-byte processing of one lane of an edge tile (xi_kernel's
// xslow_lane rules: bytes before wlo are outside; fresh entry at `fresh`;
// other lanes count after their first sync byte; tails to the next sync
// byte; past hi only the crossing walk).
template <int FMT>
__device__ __forceinline__ uint64_t gslow_lane(const GTab<FMT>& T, const uint8_t* g, uint64_t ts, uint32_t seg,
                                               uint32_t slen, uint64_t wlo, uint64_t hi, uint64_t fresh,
                                               uint64_t rend, uint32_t at_eof, uint64_t& cnt, uint64_t& sst,
                                               uint64_t& len, uint64_t& fs, uint32_t& ovf)
{
  bool act = ts + seg + slen > wlo && ts + seg < hi;
  bool synced = false;
  uint32_t m = T.start_row, acc = 0;
  uint64_t xit = ~0ull, last = 0;
  const uint64_t rend16 = (rend + 15) & ~uint64_t(15);
  uint4 vn = gload16(grsrc(g + ts, rend16 > ts ? rend16 - ts : 0), seg);
  for (uint64_t c = 0; __ballot(act); c += 16) {
    const uint4 v = vn;
    const uint64_t cb = ts + c + 16;
    vn = gload16(grsrc(g + cb, rend16 > cb ? rend16 - cb : 0), seg);
    const uint64_t base = ts + seg + c;
    const uint32_t dh = gdist(hi, base), dr = gdist(rend, base), dl = gdist(wlo, base);
    const uint32_t df = fresh >= base && fresh - base < 16 ? (uint32_t)(fresh - base) : 0xffffffffu;
    const uint32_t dseg = c >= (uint64_t)slen ? 0u : (uint32_t)(slen - c);
    GSum s;  // this chunk's sums, relative to base
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      bool go = act && k >= dl;
      if (go && k == df) {
        m = T.start_row;
        acc = 0;
        synced = true;
      }
      if (go && !synced && k >= dseg) act = go = false;  // no sync in the segment: covered by a tail
      const bool walk = T.in_walk(m);
      if (go && k >= dh && !(synced && walk)) {
        if (synced) xit = base + k;
        act = go = false;
      }
      if (go && k >= dr) {
        if (synced) {
          if (!at_eof && walk) ovf |= 1;
          xit = k >= dh ? (last > hi ? last : hi) : base + k;
        }
        act = go = false;
      }
      const uint32_t b = (gsel4(v, k >> 2) >> (8 * (k & 3))) & 0xffu;
      const uint32_t e = T.stepb(m, b);
      if (go) {
        const uint32_t t = e >> 2;
        const uint32_t f = t & (e | ~acc) & 1u;
        const uint32_t L = (e >> XG_LSHIFT) & 7u;
        if (k >= dh && (e & XT_DEAD)) {
          xit = last > hi ? last : hi;
          act = false;
        } else if (synced) {
          s.cnt += f;
          s.sq += __umul24(f, k + 1);
          s.sfl += __umul24(f, L);
          s.sl += L;
          if (t & 1u) last = base + k + 1;
          if (k < dh && T.sy[b] && k >= dseg) {  // the tail ends at a sync byte
            xit = base + k + 1;
            act = false;
          }
        } else if (T.sy[b]) {
          synced = true;
          fs = base + k;
        }
        acc = t | (acc & ~e);
        m = e;
      }
    }
    gfold(s, base, cnt, sst, len);
  }
  return xit;
}

__device__ __forceinline__ uint64_t gwave_min64(uint64_t m)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(m, o, 64);
    m = y < m ? y : m;
  }
  return m;
}

__device__ __forceinline__ uint64_t gwave_max_set(uint64_t v)
{
  uint64_t m = v == ~0ull ? 0ull : v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(m, o, 64);
    m = y > m ? y : m;
  }
  return m;
}


// stage the tables of P into LDS (all threads of the block)
template <int FMT>
__device__ __forceinline__ GTab<FMT> gstage(const ScanParams& P, uint16_t* xg, uint8_t* c2, uint8_t* sy, int tid,
                                            int nthreads)
{
  const uint4* src = reinterpret_cast<const uint4*>(P.xg);
  uint4* dst = reinterpret_cast<uint4*>(xg);
  for (uint32_t i = tid; i < P.ntrans_pad / 8; i += nthreads) dst[i] = src[i];
  for (int i = tid; i < 256; i += nthreads) {
    c2[i] = (uint8_t)(2 * P.cls[i]);
    sy[i] = P.xg_sync[i];
  }
  __syncthreads();
  GTab<FMT> T;
  T.xg = xg;
  T.c2 = c2;
  T.sy = sy;
  T.rowmask = ~((1u << P.log_row) - 1u);
  T.start_row = P.start;
  return T;
}

}  // namespace

template <int FMT>
__global__ __launch_bounds__(kGWaves * 64) void xg_kernel(ScanParams P)
{
  __shared__ __attribute__((aligned(16))) uint16_t gxg[kGMaxEntries];
  __shared__ uint8_t gc2[256], gsy[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const GTab<FMT> T = gstage<FMT>(P, gxg, gc2, gsy, tid, kGWaves * 64);

  const uint64_t gw = (uint64_t)blockIdx.x * kGWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kGTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kGTile, P.lo, P.hi);
  const uint32_t n = (uint32_t)(te - tb);
  const bool first_wave = wlo == P.lo;
  const uint32_t seg = (uint32_t)lane * kGS;

  uint64_t cnt = 0, sst = 0, len = 0;
  uint64_t entry = first_wave ? wlo : ~0ull, exit = whi;
  uint32_t ovf = 0;
  bool has_edge = false;
  const uint64_t rend16 = (P.rend + 15) & ~uint64_t(15);

  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t ts = (tb + i) * (uint64_t)kGTile;
    const __amdgpu_buffer_rsrc_t rs = grsrc(P.g + ts, rend16 > ts ? rend16 - ts : 0);
    const bool edge_lo = ts < wlo;
    const bool edge_hi = whi == P.hi && i + 1 == n;
    if (edge_lo || edge_hi) {  // xg_edge_kernel completes this wave's record
      has_edge = true;
      continue;
    }
    bool synced = first_wave && i == 0 && lane == 0 && ts == wlo;  // fresh entry at the tile start
    uint32_t fs = ~0u, m = T.start_row, acc = 0;
    GSum s4;  // main loop: cnt, sq and sfl x4
    uint4 cur[kGLd], nxt[kGLd];
#pragma unroll
    for (int k = 0; k < kGLd; ++k) cur[k] = gload16(rs, seg + 16u * k);
    for (uint32_t b = 0; b < (uint32_t)kGBlocks; ++b) {
      const uint32_t nb = b + 1 < (uint32_t)kGBlocks ? b + 1 : b;
#pragma unroll
      for (int k = 0; k < kGLd; ++k) nxt[k] = gload16(rs, seg + nb * kGBlk + 16u * k);
      if (__ballot(!synced))
        gblock<FMT, true>(T, cur, m, acc, s4, synced, fs, b * kGBlk);
      else
        gblock<FMT, false>(T, cur, m, acc, s4, synced, fs, b * kGBlk);
#pragma unroll
      for (int k = 0; k < kGLd; ++k) cur[k] = nxt[k];
    }
    GSum s;
    s.cnt = s4.cnt >> 2;
    s.sq = s4.sq >> 2;
    s.sfl = s4.sfl >> 2;
    s.sl = s4.sl;
    if (!synced) s = GSum();  // covered by an earlier tail
    acc = (acc >> 2) & 1u;    // the tail keeps the accepted bit in bit 0
    gfold(s, ts + seg, cnt, sst, len);
    const uint64_t xit =
        gtail<FMT>(T, P.g, ts, seg + kGS, m, acc, cnt, sst, len, P.hi, P.rend, P.at_eof, ovf, synced);
    const uint64_t f = synced && fs != ~0u ? ts + seg + fs : ~0ull;
    if (entry == ~0ull) {
      const uint64_t mn = gwave_min64(f);
      if (mn != ~0ull) entry = mn + 1;
    }
    const uint64_t mx = gwave_max_set(xit);
    if (mx) exit = mx;
  }
  if (entry == ~0ull && !has_edge) entry = exit;
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  const uint64_t c = wave_sum(cnt), sm = wave_sum(sst), l = wave_sum(len);
  if (lane == 0) {
    const uint64_t s_rep = sm + c * (uint64_t)P.delta;
    BlockRec rec;
    rec.entry = n ? entry : wlo;
    rec.exit = n ? exit : wlo;
    rec.cnt = c;
    rec.dg = 31 * s_rep + l;
    rec.dc = (uint64_t)P.cap1 * (s_rep + c);
    rec.pad0 = rec.pad1 = rec.pad2 = 0;
    P.recs[gw] = rec;
  }
}

struct GEdges {
  uint64_t tile[2], wave[2];
  uint32_t n;
};

// Edge tiles: 1024 lanes of 64-byte segments (see xi_kernel.hip).
constexpr int kGEdgeThreads = 1024;
constexpr uint32_t kGEdgeSeg = kGTile / kGEdgeThreads;

struct GBlockRed {
  uint64_t v[kGEdgeThreads / 64][5];
};

template <int FMT>
__global__ __launch_bounds__(kGEdgeThreads) void xg_edge_kernel(ScanParams P, GEdges E)
{
  __shared__ __attribute__((aligned(16))) uint16_t gxg[kGMaxEntries];
  __shared__ uint8_t gc2[256], gsy[256];
  __shared__ GBlockRed R;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const GTab<FMT> T = gstage<FMT>(P, gxg, gc2, gsy, tid, kGEdgeThreads);
  const uint32_t seg = (uint32_t)tid * kGEdgeSeg;
  uint32_t ovf = 0;
  for (uint32_t k = 0; k < E.n; ++k) {
    const uint64_t gw = E.wave[k];
    uint64_t tb = P.t0 + gw * P.tpb;
    uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
    if (tb > te) tb = te;
    const uint64_t wlo = clampu(tb * kGTile, P.lo, P.hi);
    const uint64_t t = E.tile[k], ts = t * (uint64_t)kGTile;
    const uint64_t fresh = wlo == P.lo && t == tb ? wlo : ~0ull;
    uint64_t fs = ~0ull, cnt = 0, sst = 0, len = 0;
    const uint64_t xit =
        gslow_lane<FMT>(T, P.g, ts, seg, kGEdgeSeg, wlo, P.hi, fresh, P.rend, P.at_eof, cnt, sst, len, fs, ovf);
    const uint64_t c = wave_sum(cnt), sm = wave_sum(sst), l = wave_sum(len);
    const uint64_t mx = gwave_max_set(xit), mf = gwave_min64(fs);
    if (lane == 0) {
      R.v[wid][0] = c;
      R.v[wid][1] = sm;
      R.v[wid][2] = l;
      R.v[wid][3] = mf;
      R.v[wid][4] = mx;
    }
    __syncthreads();
    if (tid == 0) {
      uint64_t rc = 0, rs = 0, rl = 0, rf = ~0ull, rx = 0;
      for (int w = 0; w < kGEdgeThreads / 64; ++w) {
        rc += R.v[w][0];
        rs += R.v[w][1];
        rl += R.v[w][2];
        rf = R.v[w][3] < rf ? R.v[w][3] : rf;
        rx = R.v[w][4] > rx ? R.v[w][4] : rx;
      }
      BlockRec r = P.recs[gw];
      const uint64_t s_rep = rs + rc * (uint64_t)P.delta;
      r.cnt += rc;
      r.dg += 31 * s_rep + rl;
      r.dc += (uint64_t)P.cap1 * (s_rep + rc);
      if (t + 1 == te && rx) r.exit = rx;
      if (r.entry == ~0ull) r.entry = rf != ~0ull ? rf + 1 : r.exit;
      P.recs[gw] = r;
    }
    __syncthreads();
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
}

hipError_t launch_xg(const ScanParams& P, hipStream_t stream)
{
  GEdges E{};
  const uint64_t unit = kGTile;
  if (P.lo % unit != 0) {
    E.tile[E.n] = P.t0;
    E.wave[E.n] = 0;
    ++E.n;
  }
  if (P.t1 > P.t0 && !(E.n == 1 && E.tile[0] == P.t1 - 1)) {
    E.tile[E.n] = P.t1 - 1;
    E.wave[E.n] = (P.t1 - 1 - P.t0) / P.tpb;
    ++E.n;
  }
  if (P.log_row == 8) {
    hipLaunchKernelGGL(xg_kernel<0>, dim3(P.grid), dim3(kGWaves * 64), 0, stream, P);
    hipLaunchKernelGGL(xg_edge_kernel<0>, dim3(1), dim3(kGEdgeThreads), 0, stream, P, E);
  } else {
    hipLaunchKernelGGL(xg_kernel<1>, dim3(P.grid), dim3(kGWaves * 64), 0, stream, P);
    hipLaunchKernelGGL(xg_edge_kernel<1>, dim3(1), dim3(kGEdgeThreads), 0, stream, P, E);
  }
  return hipGetLastError();
}

hipError_t xg_occupancy(uint32_t format, int* n)
{
  if (format == 0) return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xg_kernel<0>, kGWaves * 64, 0);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xg_kernel<1>, kGWaves * 64, 0);
}

uint32_t xg_unit() { return kGTile; }
uint32_t xg_waves() { return kGWaves; }
uint32_t xg_max_entries() { return kGMaxEntries; }

}  // namespace ugpu
