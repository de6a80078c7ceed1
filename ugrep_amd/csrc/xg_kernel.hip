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
// tiles in a one-wave kernel).  Per byte: a column lookup (u8) and one u16
// transition lookup in LDS, on the product transducer of tables.hpp (xg2):
// states (DFA state, "the walk has accepted"), so each entry carries its byte's
// events outright -- L = gap + 1 of an accept (every accept adds L bytes to the
// current match), F = the first accept of a walk (the match starts at
// q + 1 - L):
//   count = #F, sum start = sum_F (q + 1) - sum_F L, sum len = sum L.
// The table is class-major with an odd dword stride per column, so lanes in
// different states reading one column (or one state reading different
// columns) hit different LDS banks.  Events are packed four bytes to a dword
// and summed with v_dot4_u32_u8; the main loop keeps no per-byte
// bookkeeping beyond the three VALU of the lookup itself.
#include "device_common.hpp"
#include "tables.hpp"

namespace ugpu {

namespace {

// Each lane walks UGPU_XG_NCH chains, over the segments of virtual lanes
// v = lane + 64 j.  Measured on C4 (8 GiB): 1 chain x 16 waves 3.07 ms, 2 x 8
// 4.44, 2 x 16 9.3, 4 x 4 10.9 (register spills): one chain per lane it is
#ifndef UGPU_XG_NCH
#define UGPU_XG_NCH 1
#endif
constexpr int kGCh = UGPU_XG_NCH;
constexpr int kGTile = 65536;            // wave tile
constexpr int kGS = kGTile / 64 / kGCh;  // segment bytes per chain
#ifndef UGPU_XG_BLK
#define UGPU_XG_BLK 64
#endif
constexpr int kGBlk = UGPU_XG_BLK;  // bytes per block (16 B loads per chain, double buffered)
constexpr int kGLd = kGBlk / 16;
constexpr int kGBlocks = kGS / kGBlk;
#ifndef UGPU_XG_WAVES
#define UGPU_XG_WAVES 16
#endif
constexpr int kGWaves = UGPU_XG_WAVES;  // waves per workgroup: one staged table per CU
// LDS: the table (up to ~158 KB: C4's \w+ has 99 columns x 794 product states)
// plus 512 B of byte columns and sync flags, dynamic
constexpr uint32_t kGMaxTableBytes = 160u * 1024 - 512 - 1024;

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

// Tables in LDS: transitions (u16, class-major), columns and sync flags per byte.
struct GTab {
  const uint8_t* xg;   // byte address of the table
  const uint8_t* col;  // column of each byte
  const uint8_t* sy;   // sync-byte flags
  uint32_t stride;     // bytes per column
  // entry after byte b from entry m (the row offset of m is m >> XG2_ROWSHIFT)
  __device__ __forceinline__ uint32_t step(uint32_t m, uint32_t b) const
  {
    const uint32_t c = col[b];
    return *reinterpret_cast<const uint16_t*>(xg + __umul24(c, stride) + (m >> XG2_ROWSHIFT));
  }
  __device__ __forceinline__ static bool in_walk(uint32_t m) { return (m >> XG2_ROWSHIFT) != 0; }
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

// Events of four entries packed into one dword (bits 0-2 L, bit 3 F per byte),
// summed into s with the dword's position weights wq = (q + 1) of each byte.
__device__ __forceinline__ void gevents(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3, uint32_t keep,
                                        uint32_t wq, GSum& s)
{
  const uint32_t ev = (__builtin_amdgcn_perm(e1, e0, 0x0c0c0400u) | __builtin_amdgcn_perm(e3, e2, 0x04000c0cu)) & keep;
  const uint32_t Lb = ev & 0x07070707u;
  const uint32_t Fb = (ev >> 3) & 0x01010101u;
  s.cnt = __builtin_amdgcn_udot4(Fb, 0x01010101u, s.cnt, false);
  s.sq = __builtin_amdgcn_udot4(Fb, wq, s.sq, false);
  s.sfl = __builtin_amdgcn_udot4(Fb, Lb, s.sfl, false);
  s.sl = __builtin_amdgcn_udot4(Lb, 0x01010101u, s.sl, false);
}

// One dword of the main loop (block offset of its byte 0: bo; block offset in
// the segment: bb).  MASK: events up to and including the lane's first sync
// byte are dropped (the previous lane's tail counts them); fs gets that byte's
// segment offset.
template <bool MASK>
__device__ __forceinline__ void gdword(const GTab& T, uint32_t w, uint32_t& m, GSum& s, uint32_t bo, uint32_t bb,
                                       bool& synced, uint32_t& fs)
{
  const uint32_t e0 = T.step(m, w & 0xffu);
  const uint32_t e1 = T.step(e0, (w >> 8) & 0xffu);
  const uint32_t e2 = T.step(e1, (w >> 16) & 0xffu);
  const uint32_t e3 = T.step(e2, w >> 24);
  m = e3;
  uint32_t keep = 0xffffffffu;
  if constexpr (MASK) {
    const uint32_t y = (uint32_t)T.sy[w & 0xffu] | (uint32_t)T.sy[(w >> 8) & 0xffu] << 8 |
                       (uint32_t)T.sy[(w >> 16) & 0xffu] << 16 | (uint32_t)T.sy[w >> 24] << 24;
    const uint32_t t = y & (0u - y);  // bit 0 of the first sync byte k
    if (!synced) {
      keep = ~((t << 8) - 1u);  // bytes after k (none when there is no sync byte)
      if (y) fs = bb + bo + ((uint32_t)__builtin_ctz(y) >> 3);
    }
    synced = synced || y != 0u;
  }
  const uint32_t wq = (bo + 1) | ((bo + 2) << 8) | ((bo + 3) << 16) | ((bo + 4) << 24);
  gevents(e0, e1, e2, e3, keep, wq, s);
}

// One block of kGBlk bytes of every chain, from registers, block offset bb
// within the chains' segments; the chains advance a dword each in turn, so
// their lookups overlap.  Position weights are block-relative (< 256),
// bb * #F is added after.
template <bool MASK>
__device__ __forceinline__ void gblock(const GTab& T, const uint4 (&v)[kGCh][kGLd], uint32_t (&m)[kGCh],
                                       GSum (&s)[kGCh], bool (&synced)[kGCh], uint32_t (&fs)[kGCh], uint32_t bb)
{
  uint32_t c0[kGCh];
#pragma unroll
  for (int j = 0; j < kGCh; ++j) c0[j] = s[j].cnt;
#pragma unroll
  for (int k = 0; k < kGLd; ++k) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
#pragma unroll
      for (int j = 0; j < kGCh; ++j) {
        const uint32_t w = d == 0 ? v[j][k].x : d == 1 ? v[j][k].y : d == 2 ? v[j][k].z : v[j][k].w;
        gdword<MASK>(T, w, m[j], s[j], 16u * k + 4u * d, bb, synced[j], fs[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kGCh; ++j) s[j].sq += __umul24(s[j].cnt - c0[j], bb);  // the block's starts at offset bb
}

__device__ __forceinline__ uint32_t gdist(uint64_t lim, uint64_t base)  // lim - base clamped to [0, 64]
{
  return lim > base ? (lim - base < 64 ? (uint32_t)(lim - base) : 64u) : 0u;
}

// Tail of a lane from tile offset o (its segment end): walk until a sync
// byte has been read.  Returns the coverage end (as xi_kernel's xtail).
__device__ __forceinline__ uint64_t gtail(const GTab& T, const uint8_t* g, uint64_t ts, uint32_t o, uint32_t& m,
                                          uint64_t& cnt, uint64_t& sst, uint64_t& len, uint64_t hi, uint64_t rend,
                                          uint32_t at_eof, uint32_t& ovf, bool act)
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
      const bool walk = GTab::in_walk(m);
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
      const uint32_t e = T.step(m, b);
      if (go) {
        const uint32_t L = e & XG2_L, f = (e >> 3) & 1u;
        if (k >= dh && (e & XG2_D)) {  // the walk crossing hi died here
          xit = last > hi ? last : hi;
          act = false;
        } else {
          s.cnt += f;
          s.sq += __umul24(f, k + 1);
          s.sfl += __umul24(f, L);
          s.sl += L;
          if (L) last = base + k + 1;
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
__device__ __forceinline__ uint64_t gslow_lane(const GTab& T, const uint8_t* g, uint64_t ts, uint32_t seg,
                                               uint32_t slen, uint64_t wlo, uint64_t hi, uint64_t fresh, uint64_t rend,
                                               uint32_t at_eof, uint64_t& cnt, uint64_t& sst, uint64_t& len,
                                               uint64_t& fs, uint32_t& ovf)
{
  bool act = ts + seg + slen > wlo && ts + seg < hi;
  bool synced = false;
  uint32_t m = 0;
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
        m = 0;
        synced = true;
      }
      if (go && !synced && k >= dseg) act = go = false;  // no sync in the segment: covered by a tail
      const bool walk = GTab::in_walk(m);
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
      const uint32_t e = T.step(m, b);
      if (go) {
        const uint32_t L = e & XG2_L, f = (e >> 3) & 1u;
        if (k >= dh && (e & XG2_D)) {
          xit = last > hi ? last : hi;
          act = false;
        } else if (synced) {
          s.cnt += f;
          s.sq += __umul24(f, k + 1);
          s.sfl += __umul24(f, L);
          s.sl += L;
          if (L) last = base + k + 1;
          if (k < dh && T.sy[b] && k >= dseg) {  // the tail ends at a sync byte
            xit = base + k + 1;
            act = false;
          }
        } else if (T.sy[b]) {
          synced = true;
          fs = base + k;
        }
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

// stage the tables of P into LDS (all threads of the block): table, then the
// byte columns and sync flags
__device__ __forceinline__ GTab gstage(const ScanParams& P, uint8_t* smem, int tid, int nthreads)
{
  uint16_t* xg = reinterpret_cast<uint16_t*>(smem);
  uint8_t* sy = smem + 2 * (size_t)P.xg_entries;
  uint8_t* col = sy + 256;
  const uint4* src = reinterpret_cast<const uint4*>(P.xg);
  uint4* dst = reinterpret_cast<uint4*>(xg);
  for (uint32_t i = tid; i < P.xg_entries / 8; i += nthreads) dst[i] = src[i];
  for (int i = tid; i < 256; i += nthreads) {
    col[i] = P.xg_cls[i];
    sy[i] = P.xg_sync[i];
  }
  __syncthreads();
  GTab T;
  T.xg = reinterpret_cast<const uint8_t*>(xg);
  T.col = col;
  T.sy = sy;
  T.stride = P.xg_stride;
  return T;
}

}  // namespace

__global__ __launch_bounds__(kGWaves * 64) void xg_kernel(ScanParams P)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const GTab T = gstage(P, gsm, tid, kGWaves * 64);

  const uint64_t gw = (uint64_t)blockIdx.x * kGWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kGTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kGTile, P.lo, P.hi);
  const uint32_t n = (uint32_t)(te - tb);
  const bool first_wave = wlo == P.lo;

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
    bool synced[kGCh];
    uint32_t fs[kGCh], m[kGCh], seg[kGCh];
    GSum s[kGCh];
    uint4 cur[kGCh][kGLd], nxt[kGCh][kGLd];
#pragma unroll
    for (int j = 0; j < kGCh; ++j) {
      seg[j] = (uint32_t)(lane + 64 * j) * kGS;
      synced[j] = first_wave && i == 0 && lane == 0 && j == 0 && ts == wlo;  // fresh entry at the tile start
      fs[j] = ~0u;
      m[j] = 0;
#pragma unroll
      for (int k = 0; k < kGLd; ++k) cur[j][k] = gload16(rs, seg[j] + 16u * k);
    }
    for (uint32_t b = 0; b < (uint32_t)kGBlocks; ++b) {
      const uint32_t nb = b + 1 < (uint32_t)kGBlocks ? b + 1 : b;
#pragma unroll
      for (int j = 0; j < kGCh; ++j)
#pragma unroll
        for (int k = 0; k < kGLd; ++k) nxt[j][k] = gload16(rs, seg[j] + nb * kGBlk + 16u * k);
      bool any = false;
#pragma unroll
      for (int j = 0; j < kGCh; ++j) any = any || !synced[j];
      if (__ballot(any))
        gblock<true>(T, cur, m, s, synced, fs, b * kGBlk);
      else
        gblock<false>(T, cur, m, s, synced, fs, b * kGBlk);
#pragma unroll
      for (int j = 0; j < kGCh; ++j)
#pragma unroll
        for (int k = 0; k < kGLd; ++k) cur[j][k] = nxt[j][k];
    }
    uint64_t f = ~0ull, xmax = 0;
#pragma unroll
    for (int j = 0; j < kGCh; ++j) {
      if (!synced[j]) s[j] = GSum();  // covered by an earlier tail
      gfold(s[j], ts + seg[j], cnt, sst, len);
      const uint64_t xit =
          gtail(T, P.g, ts, seg[j] + kGS, m[j], cnt, sst, len, P.hi, P.rend, P.at_eof, ovf, synced[j]);
      if (synced[j] && fs[j] != ~0u && ts + seg[j] + fs[j] < f) f = ts + seg[j] + fs[j];
      if (xit != ~0ull && xit > xmax) xmax = xit;
    }
    if (entry == ~0ull) {
      const uint64_t mn = gwave_min64(f);
      if (mn != ~0ull) entry = mn + 1;
    }
    const uint64_t mx = gwave_max_set(xmax ? xmax : ~0ull);
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

__global__ __launch_bounds__(kGEdgeThreads) void xg_edge_kernel(ScanParams P, GEdges E)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  __shared__ GBlockRed R;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const GTab T = gstage(P, gsm, tid, kGEdgeThreads);
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
        gslow_lane(T, P.g, ts, seg, kGEdgeSeg, wlo, P.hi, fresh, P.rend, P.at_eof, cnt, sst, len, fs, ovf);
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
  const size_t smem = xg_smem_bytes(P.xg_entries);
  hipError_t e;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(xg_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)smem)) != hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(xg_edge_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(xg_kernel, dim3(P.grid), dim3(kGWaves * 64), smem, stream, P);
  hipLaunchKernelGGL(xg_edge_kernel, dim3(1), dim3(kGEdgeThreads), smem, stream, P, E);
  return hipGetLastError();
}

size_t xg_smem_bytes(uint32_t entries) { return 2 * (size_t)entries + 512; }

hipError_t xg_occupancy(uint32_t entries, int* n)
{
  const size_t smem = xg_smem_bytes(entries);
  if (2 * (size_t)entries > kGMaxTableBytes) {
    *n = 0;
    return hipSuccess;
  }
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(xg_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xg_kernel, kGWaves * 64, smem);
}

uint32_t xg_unit() { return kGTile; }
uint32_t xg_waves() { return kGWaves; }

}  // namespace ugpu
