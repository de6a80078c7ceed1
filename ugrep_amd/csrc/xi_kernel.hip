// xi_kernel.hip -- FIND over "immediate" restart-local tables (tables.hpp):
// token patterns such as identifiers, numbers or ASCII words, where every walk
// accepts on each byte it reads, so a match is exactly one walk of the DFA.
//
// What it replaces: the reference's per-match FIND loop (lib/matcher.cpp:
// 42-750) with its DFA opcode walk (:125-546) for such patterns; results are
// the same (count, digest = sum(31 start + len), dcap = sum((start + 1) cap)).
//
// Layout.  A wave owns contiguous 64 KiB tiles; lane l walks its own 1 KiB
// segment [ts + 1024 l, ts + 1024 (l + 1)), reading it from HBM with 16-byte
// loads (64 B per block, double buffered in registers).  The walk runs on the
// byte-id table of tables.hpp staged in LDS: one v_perm (address = id << 8 |
// byte) and one ds_read_u8 per byte; the id read carries the events of that
// byte (ST: a match starts, IN: the byte lies in a match, Y: sync byte).
//
// Exact lanes without fix-ups.  A sync byte kills every walk and starts none,
// so after it every FIND chain is in the start state.  Lane l counts the
// events strictly after the first sync byte of its segment (the "head" is
// masked) and, past its segment end, keeps walking until it has read the
// first sync byte of what follows (its "tail").  Consecutive lanes thus tile
// the chain exactly, and so do consecutive tiles and waves: a wave's record
// enters at its first sync byte + 1 and exits after its last tail's sync
// byte, so fix_kernel finds nothing to merge.  Only the chain entry of the
// whole range (P.lo, fresh) and its end (P.hi: matches starting before hi,
// the exit is the first chain position >= hi) need the exact per-byte rules
// of xi_slow_tile, run for the at most two tiles that hold lo (unaligned) or hi.
//
// Deferred accounting.  The main loop does no per-byte bookkeeping: four ids
// are packed into one dword and summed with v_dot4_u32_u8 -- the number of
// starts, their positions inside the 64-byte block (weights 0..63) and the
// number of IN bytes -- and folded once per block.  Then
//   count = #ST, sum start = sum of ST positions, sum len = #IN,
//   digest = 31 sum start + sum len, dcap = cap1 (sum start + count).
#include "device_common.hpp"
#include "tables.hpp"

namespace ugpu {

namespace {

#ifndef UGPU_XI_SEG
#define UGPU_XI_SEG 1024
#endif
#ifndef UGPU_XI_WGLDS
// LDS per workgroup (table + padding), capping xi_kernel at 3 workgroups (12
// waves) per CU: measured on C3 16 GiB, 3 waves per SIMD beat 4 (4.49 vs 5.39
// ms) and 2 (5.64).  Tables above 208 rows exceed it (2 workgroups per CU).
#define UGPU_XI_WGLDS 53248
#endif
constexpr int kXS = UGPU_XI_SEG;   // lane segment bytes
constexpr int kXTile = 64 * kXS;   // wave tile
#ifndef UGPU_XI_BLK
#define UGPU_XI_BLK 64
#endif
constexpr int kXBlk = UGPU_XI_BLK;  // bytes per block, read by back-to-back 16-byte loads
constexpr int kXLd = kXBlk / 16;    // 16-byte loads per lane per block
constexpr int kXBlocks = kXS / kXBlk;
constexpr int kXWaves = 4;         // waves per workgroup (one staged table)

__device__ __forceinline__ uint4 xload16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
  return uint4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xrsrc(const uint8_t* base, uint64_t readable)
{
  const uint32_t n = readable < 0x7fffff00ull ? (uint32_t)readable : 0x7fffff00u;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)n), 0x00020000);
}

// Two layouts were measured against this one on C3 (16 GiB, 4.33 ms): rows
// 260 bytes apart so that different ids use different LDS banks (one more VALU
// per byte: 5.72 ms, bank-conflict cycles 578 M vs 751 M), and 4-byte steps
// (the byte classes of 4 bytes by SWAR range tests, then one lookup of the ids
// after each byte: 5.12 ms, VALU 2.24 G vs 1.35 G instructions).  One LDS read
// per byte is the cheapest classifier.
// next id after byte k (0..3) of dword w: table row = id, column = byte
template <int K>
__device__ __forceinline__ uint32_t xnext(const uint8_t* T, uint32_t id, uint32_t w)
{
  return T[__builtin_amdgcn_perm(id, w, 0x0c0c0400u | (uint32_t)K)];
}

// Lane accumulators (lane-relative positions; ins2 = 2 x #IN bytes).  64-bit:
// a tail runs as long as there is no sync byte (a lane may cover gigabytes of
// a newline-free '.' search), the main loop adds once per block.
struct XSum {
  uint64_t cnt = 0, ins2 = 0, pos = 0;
};

// One dword of the main loop.  MASK: events up to and including the lane's
// first sync byte are dropped (the previous lane's tail counts them); fs gets
// that byte's position (dword base q0).
template <bool MASK>
__device__ __forceinline__ void xdword(const uint8_t* T, uint32_t w, uint32_t& id, uint32_t wj, uint32_t& cS,
                                       uint32_t& wS, uint32_t& cI, bool& synced, uint32_t& fs, uint32_t q0)
{
  const uint32_t i0 = xnext<0>(T, id, w);
  const uint32_t i1 = xnext<1>(T, i0, w);
  const uint32_t i2 = xnext<2>(T, i1, w);
  const uint32_t i3 = xnext<3>(T, i2, w);
  id = i3;
  uint32_t Q = i0 | (i1 << 8) | (i2 << 16) | (i3 << 24);
  if constexpr (MASK) {
    const uint32_t y = Q & 0x04040404u;
    const uint32_t t = y & (0u - y);                   // bit 2 of the first sync byte k
    const uint32_t m = synced ? 0xffffffffu : ~((t << 6) - 1u);  // bytes after k (none if no sync)
    if (!synced && y) fs = q0 + ((uint32_t)__builtin_ctz(y) >> 3);
    synced = synced || y != 0u;
    Q &= m;
  }
  const uint32_t s = Q & 0x01010101u;
  cS = __builtin_amdgcn_udot4(s, 0x01010101u, cS, false);
  wS = __builtin_amdgcn_udot4(s, wj, wS, false);
  cI = __builtin_amdgcn_udot4(Q & 0x02020202u, 0x01010101u, cI, false);
}

// One block (kXBlk bytes of the lane's segment; dot4 position weights
// 0..kXBlk-1); bb = block byte offset in the segment.  The bytes come from the
// lane's registers.
template <bool MASK, class SRC>
__device__ __forceinline__ void xblock(const uint8_t* T, const SRC& src, uint32_t& id, XSum& a, bool& synced,
                                       uint32_t& fs, uint32_t bb)
{
  uint32_t cS = 0, wS = 0, cI = 0;
#pragma unroll
  for (int k = 0; k < kXBlk / 8; ++k) {
    const uint2 v = src(k);
    const uint32_t w[2] = {v.x, v.y};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t d = (uint32_t)(2 * k + j);  // dword index in the block
      const uint32_t wj = (4 * d) | ((4 * d + 1) << 8) | ((4 * d + 2) << 16) | ((4 * d + 3) << 24);
      xdword<MASK>(T, w[j], id, wj, cS, wS, cI, synced, fs, bb + 4 * d);
    }
  }
  a.cnt += cS;
  a.pos += wS + bb * cS;
  a.ins2 += cI;
}

struct XRegs {  // the block's bytes in registers
  const uint4* v;
  __device__ __forceinline__ uint2 operator()(int k) const
  {
    return (k & 1) ? uint2{v[k >> 1].z, v[k >> 1].w} : uint2{v[k >> 1].x, v[k >> 1].y};
  }
};

// Per-byte walk of one lane (tails and the edge tiles): returns the next id and
// adds the byte's events when counting.
__device__ __forceinline__ uint32_t xbyte(const uint8_t* T, uint32_t id, uint32_t w, uint32_t k)
{
  return T[(id << 8) | ((w >> (8 * k)) & 0xffu)];
}

__device__ __forceinline__ uint32_t xsel4(const uint4& v, uint32_t j)
{
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// Tail of a lane: from tile offset `o` (its segment end) walk until a sync
// byte has been read, counting everything; bytes from global, 16 at a time.
// Past the range end hi only the walk crossing hi goes on.  Returns the chain
// position where the lane's coverage ends: after the sync byte, the first
// chain position >= hi, or the readable end; ~0 for lanes not active.
__device__ __forceinline__ uint32_t xdist(uint64_t lim, uint64_t base)  // lim - base clamped to [0, 64]
{
  return lim > base ? (lim - base < 64 ? (uint32_t)(lim - base) : 64u) : 0u;
}

__device__ __forceinline__ uint64_t xtail(const uint8_t* T, const uint8_t* g, uint64_t ts, uint32_t o,
                                          uint32_t seg, uint32_t& id, XSum& a, uint64_t hi, uint64_t rend,
                                          uint32_t at_eof, uint32_t& ovf, bool act)
{
  uint64_t xit = ~0ull;
  const uint64_t rend16 = (rend + 15) & ~uint64_t(15);
  // (the resource moves with c: tails may be longer than 32-bit offsets; the
  // next 16 bytes load while these are walked; per-byte work is 32-bit,
  // relative to the chunk)
  uint4 vn = xload16(xrsrc(g + ts, rend16 > ts ? rend16 - ts : 0), o);
  for (uint64_t c = 0; __ballot(act); c += 16) {
    const uint4 v = vn;
    const uint64_t cb = ts + c + 16;
    vn = xload16(xrsrc(g + cb, rend16 > cb ? rend16 - cb : 0), o);
    const uint64_t base = ts + o + c;  // position of byte 0 of this chunk
    const uint32_t dh = xdist(hi, base), dr = xdist(rend, base);
    uint32_t cn = 0, ps = 0, in2 = 0, stop = 0xffffffffu;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      bool go = act;
      if (go && k >= dh && !(id & XI_IN)) {  // no walk crosses into this byte: the chain is here
        stop = k;
        act = go = false;
      }
      if (go && k >= dr) {  // readable end: at EOF the walk ends there
        if (!at_eof && (id & XI_IN)) ovf |= 1;
        stop = k;
        act = go = false;
      }
      const uint32_t e = xbyte(T, id, xsel4(v, k >> 2), k & 3);
      if (go) {
        if (k >= dh) {
          if ((e & XI_ST) || !(e & XI_IN)) {  // the walk crossing hi ended here
            stop = k;
            act = false;
          } else {
            in2 += XI_IN;
          }
        } else {
          const uint32_t st = e & XI_ST;
          cn += st;
          ps += st ? k : 0u;
          in2 += e & XI_IN;
          if (e & XI_Y) {
            stop = k + 1;
            act = false;
          }
        }
        id = e;
      }
    }
    a.cnt += cn;
    a.pos += (uint64_t)cn * (o + c - seg) + ps;
    a.ins2 += in2;
    if (stop != 0xffffffffu) xit = base + stop;
  }
  return xit;
}

// Exact per-byte processing of one lane for the tiles holding the range
// edges: bytes before wlo are outside the range; the chain enters fresh at
// `fresh` (P.lo for the first wave, ~0 otherwise); other lanes count after
// their first sync byte; past the segment a counting lane goes on to the next
// sync byte, past hi only the walk crossing hi.  Returns the lane's coverage
// end as xtail does (~0: the lane covers nothing) and its first sync byte in fs.
__device__ __forceinline__ uint64_t xslow_lane(const uint8_t* T, const uint8_t* g, uint64_t ts, uint32_t seg,
                                               uint32_t slen, uint64_t wlo, uint64_t hi, uint64_t fresh,
                                               uint64_t rend, uint32_t at_eof, XSum& a, uint64_t& fs, uint32_t& ovf)
{
  bool act = ts + seg + slen > wlo && ts + seg < hi;
  bool synced = false;
  uint32_t id = 0;
  uint64_t xit = ~0ull;
  const uint64_t rend16 = (rend + 15) & ~uint64_t(15);
  uint4 vn = xload16(xrsrc(g + ts, rend16 > ts ? rend16 - ts : 0), seg);
  for (uint64_t c = 0; __ballot(act); c += 16) {
    const uint4 v = vn;
    const uint64_t cb = ts + c + 16;
    vn = xload16(xrsrc(g + cb, rend16 > cb ? rend16 - cb : 0), seg);
    const uint64_t base = ts + seg + c;  // position of byte 0 of this chunk
    const uint32_t dh = xdist(hi, base), dr = xdist(rend, base), dl = xdist(wlo, base);
    const uint32_t df = fresh >= base && fresh - base < 16 ? (uint32_t)(fresh - base) : 0xffffffffu;
    const uint32_t dseg = c >= (uint64_t)slen ? 0u : (uint32_t)(slen - c);  // bytes left in the segment
    uint32_t cn = 0, ps = 0, in2 = 0, stop = 0xffffffffu, fsk = 0xffffffffu;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      bool go = act && k >= dl;
      if (go && k == df) {
        id = 0;
        synced = true;
      }
      if (go && !synced && k >= dseg) act = go = false;  // no sync in the segment: covered by a tail
      if (go && k >= dh && !(synced && (id & XI_IN))) {
        if (synced) stop = k;
        act = go = false;
      }
      if (go && k >= dr) {
        if (synced) {
          if (!at_eof && (id & XI_IN)) ovf |= 1;
          stop = k;
        }
        act = go = false;
      }
      const uint32_t e = xbyte(T, id, xsel4(v, k >> 2), k & 3);
      if (go) {
        if (k >= dh) {
          if ((e & XI_ST) || !(e & XI_IN)) {
            stop = k;
            act = false;
          } else {
            in2 += XI_IN;
          }
        } else if (synced) {
          const uint32_t st = e & XI_ST;
          cn += st;
          ps += st ? k : 0u;
          in2 += e & XI_IN;
          if ((e & XI_Y) && k >= dseg) {  // the tail ends at a sync byte
            stop = k + 1;
            act = false;
          }
        } else if (e & XI_Y) {
          synced = true;
          fsk = k;
        }
        id = e;
      }
    }
    a.cnt += cn;
    a.pos += (uint64_t)cn * c + ps;
    a.ins2 += in2;
    if (stop != 0xffffffffu) xit = base + stop;
    if (fsk != 0xffffffffu) fs = base + fsk;
  }
  return xit;
}

__device__ __forceinline__ uint64_t wave_min64(uint64_t m)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(m, o, 64);
    m = y < m ? y : m;
  }
  return m;
}

// max over lanes, ~0 entries ignored (0 when none)
__device__ __forceinline__ uint64_t wave_max_set(uint64_t v)
{
  uint64_t m = v == ~0ull ? 0ull : v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(m, o, 64);
    m = y > m ? y : m;
  }
  return m;
}

__device__ __forceinline__ void xfold(const XSum& a, uint64_t base, uint64_t& cnt, uint64_t& sst, uint64_t& len)
{
  cnt += a.cnt;
  sst += a.cnt * base + a.pos;
  len += a.ins2 >> 1;
}

}  // namespace

// ROWS = table capacity (ids); a static LDS array lets the table address fold
// into the ds_read offset field (an extern array costs an add per byte)
#ifndef UGPU_XI_MINW
#define UGPU_XI_MINW 4  // waves per SIMD the register budget must allow (4: 128 VGPRs, no spills)
#endif
template <int ROWS>
__global__ __launch_bounds__(kXWaves * 64, UGPU_XI_MINW) void xi_kernel(ScanParams P)
{
  __shared__ __attribute__((aligned(16))) uint8_t xsm[ROWS * 256];
  constexpr int kPad = UGPU_XI_WGLDS - ROWS * 256 > 64 ? UGPU_XI_WGLDS - ROWS * 256 : 64;
  __shared__ uint8_t xpad[kPad];
  if (P.zero) xpad[threadIdx.x & 63] = 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  {
    const uint4* src = reinterpret_cast<const uint4*>(P.xid);
    uint4* dst = reinterpret_cast<uint4*>(xsm);
    for (uint32_t i = tid; i < P.xid_rows * 16; i += kXWaves * 64) dst[i] = src[i];
  }
  __syncthreads();
  const uint8_t* T = xsm;

  const uint64_t gw = (uint64_t)blockIdx.x * kXWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kXTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kXTile, P.lo, P.hi);
  const uint32_t n = (uint32_t)(te - tb);
  const bool first_wave = wlo == P.lo;  // the chain enters the range here, fresh
  const uint32_t seg = (uint32_t)lane * kXS;

  uint64_t cnt = 0, sst = 0, len = 0;  // lane totals (absolute positions)
  uint64_t entry = first_wave ? wlo : ~0ull, exit = whi;
  uint32_t ovf = 0;
  bool has_edge = false;

  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t ts = (tb + i) * (uint64_t)kXTile;
    // (a buffer load past num_records zeroes the whole dword: round the readable
    // end up to the 16-byte granule; bytes past rend are never used)
    const uint64_t rend16 = (P.rend + 15) & ~uint64_t(15);
    const __amdgpu_buffer_rsrc_t rs = xrsrc(P.g + ts, rend16 > ts ? rend16 - ts : 0);
    const bool edge_lo = ts < wlo;                   // (first wave, unaligned lo)
    const bool edge_hi = whi == P.hi && i + 1 == n;  // the range end lies in this tile
    const uint64_t fresh = first_wave && i == 0 ? wlo : ~0ull;
    XSum a;
    uint64_t xit, f;
    if (edge_lo || edge_hi) {  // xi_edge_kernel completes this wave's record
      has_edge = true;
      continue;
    } else {
      // ---- fast tile: every lane segment lies inside [wlo, whi) ----
      bool synced = fresh == ts && lane == 0;  // fresh entry at the tile start
      uint32_t fs = ~0u, id = 0;
      // Direct loads: lane l reads its own segment, 16 bytes per load, block
      // b+1 in flight while block b is walked.
      uint4 cur[kXLd], nxt[kXLd];
      const XRegs src{cur};
#pragma unroll
      for (int k = 0; k < kXLd; ++k) cur[k] = xload16(rs, seg + 16u * k);
      for (uint32_t b = 0; b < (uint32_t)kXBlocks; ++b) {
        const uint32_t nb = b + 1 < (uint32_t)kXBlocks ? b + 1 : b;
#pragma unroll
        for (int k = 0; k < kXLd; ++k) nxt[k] = xload16(rs, seg + nb * kXBlk + 16u * k);
        if (P.ablate == 6) {
          id ^= src(0).x ^ src(3).y;  // loads only (benchmarking; wrong counts)
        } else if (__ballot(!synced)) {
          xblock<true>(T, src, id, a, synced, fs, b * kXBlk);
        } else {
          xblock<false>(T, src, id, a, synced, fs, b * kXBlk);
        }
#pragma unroll
        for (int k = 0; k < kXLd; ++k) cur[k] = nxt[k];
      }
      // a lane that never met a sync byte counts nothing: an earlier tail covers it
      if (!synced) a = XSum();
      xit = xtail(T, P.g, ts, seg + kXS, seg, id, a, P.hi, P.rend, P.at_eof, ovf, synced && P.ablate != 6);
      f = synced && fs != ~0u ? ts + seg + fs : ~0ull;
    }
    if (entry == ~0ull) {  // the wave's chain starts after its first sync byte
      const uint64_t m = wave_min64(f);
      if (m != ~0ull) entry = m + 1;
    }
    const uint64_t mx = wave_max_set(xit);
    if (mx) exit = mx;
    xfold(a, ts + seg, cnt, sst, len);
  }
  if (entry == ~0ull && !has_edge) entry = exit;  // no sync byte in the range: the previous tail covers it
  if (P.ablate == 6) {  // loads-only benchmark: keep the records chained
    entry = wlo;
    exit = whi;
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  const uint64_t c = wave_sum(cnt), s = wave_sum(sst), l = wave_sum(len);
  if (lane == 0) {
    const uint64_t s_rep = s + c * (uint64_t)P.delta;  // reported starts
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

// The tiles holding the range edges (P.lo unaligned, P.hi), done by one wave
// after xi_kernel with the exact per-byte rules of xslow_lane; each completes
// its wave's record (sums added, exit and a missing entry set).  Kept out of
// xi_kernel: the per-byte edge code needs many more registers than the main loop.
struct XEdges {
  uint64_t tile[2], wave[2];
  uint32_t n;
};

// Edge tiles run with 1024 lanes of 64-byte segments (the segment length only
// matters inside the tile: lanes still count after their first sync byte and
// their tails end at the next one), so the per-byte walk is 16x shorter than
// with the main kernel's 1 KiB segments.
constexpr int kEdgeThreads = 1024;
constexpr uint32_t kEdgeSeg = kXTile / kEdgeThreads;

// block-wide sums / min / max (16 waves)
struct XBlockRed {
  uint64_t v[kEdgeThreads / 64][5];
};

__device__ __forceinline__ void xblock_reduce(XBlockRed& R, uint64_t c, uint64_t s, uint64_t l, uint64_t fsmin,
                                              uint64_t xmax, uint64_t out[5])
{
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  c = wave_sum(c);
  s = wave_sum(s);
  l = wave_sum(l);
  if (lane == 0) {
    R.v[wid][0] = c;
    R.v[wid][1] = s;
    R.v[wid][2] = l;
    R.v[wid][3] = fsmin;
    R.v[wid][4] = xmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = out[1] = out[2] = 0;
    out[3] = ~0ull;
    out[4] = 0;
    for (int w = 0; w < kEdgeThreads / 64; ++w) {
      out[0] += R.v[w][0];
      out[1] += R.v[w][1];
      out[2] += R.v[w][2];
      out[3] = R.v[w][3] < out[3] ? R.v[w][3] : out[3];
      out[4] = R.v[w][4] > out[4] ? R.v[w][4] : out[4];
    }
  }
  __syncthreads();
}

template <int ROWS>
__global__ __launch_bounds__(kEdgeThreads) void xi_edge_kernel(ScanParams P, XEdges E)
{
  __shared__ __attribute__((aligned(16))) uint8_t xsm[ROWS * 256];
  __shared__ XBlockRed R;
  const int tid = threadIdx.x;
  {
    const uint4* src = reinterpret_cast<const uint4*>(P.xid);
    uint4* dst = reinterpret_cast<uint4*>(xsm);
    for (uint32_t i = tid; i < P.xid_rows * 16; i += kEdgeThreads) dst[i] = src[i];
  }
  __syncthreads();
  const uint8_t* T = xsm;
  const uint32_t seg = (uint32_t)tid * kEdgeSeg;
  uint32_t ovf = 0;
  for (uint32_t k = 0; k < E.n; ++k) {
    const uint64_t gw = E.wave[k];
    uint64_t tb = P.t0 + gw * P.tpb;
    uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
    if (tb > te) tb = te;
    const uint64_t wlo = clampu(tb * kXTile, P.lo, P.hi);
    const uint64_t t = E.tile[k], ts = t * (uint64_t)kXTile;
    const uint64_t fresh = wlo == P.lo && t == tb ? wlo : ~0ull;
    XSum a;
    uint64_t fs = ~0ull;
    const uint64_t xit = xslow_lane(T, P.g, ts, seg, kEdgeSeg, wlo, P.hi, fresh, P.rend, P.at_eof, a, fs, ovf);
    uint64_t cnt = 0, sst = 0, len = 0;
    xfold(a, ts + seg, cnt, sst, len);
    uint64_t r[5];
    xblock_reduce(R, cnt, sst, len, wave_min64(fs), wave_max_set(xit), r);
    if (tid == 0) {
      BlockRec rec = P.recs[gw];
      const uint64_t s_rep = r[1] + r[0] * (uint64_t)P.delta;
      rec.cnt += r[0];
      rec.dg += 31 * s_rep + r[2];
      rec.dc += (uint64_t)P.cap1 * (s_rep + r[0]);
      if (t + 1 == te && r[4]) rec.exit = r[4];  // the wave's last tile: its coverage end is the exit
      if (rec.entry == ~0ull) rec.entry = r[3] != ~0ull ? r[3] + 1 : rec.exit;
      P.recs[gw] = rec;
    }
    __syncthreads();
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
}

hipError_t launch_xi(const ScanParams& P, size_t smem, hipStream_t stream)
{
  (void)smem;
  // edge tiles: the first tile when lo is not tile aligned, the last tile
  XEdges E{};
  const uint64_t unit = kXTile;
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
  if (P.xid_rows <= 16) {
    hipLaunchKernelGGL(xi_kernel<16>, dim3(P.grid), dim3(kXWaves * 64), 0, stream, P);
    hipLaunchKernelGGL(xi_edge_kernel<16>, dim3(1), dim3(kEdgeThreads), 0, stream, P, E);
  } else if (P.xid_rows <= 64) {
    hipLaunchKernelGGL(xi_kernel<64>, dim3(P.grid), dim3(kXWaves * 64), 0, stream, P);
    hipLaunchKernelGGL(xi_edge_kernel<64>, dim3(1), dim3(kEdgeThreads), 0, stream, P, E);
  } else {
    hipLaunchKernelGGL(xi_kernel<256>, dim3(P.grid), dim3(kXWaves * 64), 0, stream, P);
    hipLaunchKernelGGL(xi_edge_kernel<256>, dim3(1), dim3(kEdgeThreads), 0, stream, P, E);
  }
  return hipGetLastError();
}

hipError_t xi_occupancy(size_t smem, int* n)
{
  const uint32_t rows = (uint32_t)(smem / 256);
  if (rows <= 16) return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xi_kernel<16>, kXWaves * 64, 0);
  if (rows <= 64) return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xi_kernel<64>, kXWaves * 64, 0);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xi_kernel<256>, kXWaves * 64, 0);
}

uint32_t xi_unit() { return kXTile; }
uint32_t xi_waves() { return kXWaves; }

}  // namespace ugpu
