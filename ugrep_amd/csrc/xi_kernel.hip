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

constexpr int kXS = 1024;          // lane segment bytes
constexpr int kXTile = 64 * kXS;   // wave tile
constexpr int kXBlk = 64;          // bytes per block (4 x 16 B per lane)
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

// 16 dwords (one 64-byte block); bb = block byte offset in the segment
template <bool MASK>
__device__ __forceinline__ void xblock(const uint8_t* T, const uint4 (&v)[4], uint32_t& id, XSum& a, bool& synced,
                                       uint32_t& fs, uint32_t bb)
{
  uint32_t cS = 0, wS = 0, cI = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t d = (uint32_t)(4 * k + j);  // dword index in the block
      const uint32_t wj = (4 * d) | ((4 * d + 1) << 8) | ((4 * d + 2) << 16) | ((4 * d + 3) << 24);
      xdword<MASK>(T, w[j], id, wj, cS, wS, cI, synced, fs, bb + 4 * d);
    }
  }
  a.cnt += cS;
  a.pos += wS + bb * cS;
  a.ins2 += cI;
}

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
__device__ __forceinline__ uint64_t xtail(const uint8_t* T, const uint8_t* g, uint64_t ts, uint32_t o,
                                          uint32_t seg, uint32_t& id, XSum& a, uint64_t hi, uint64_t rend,
                                          uint32_t at_eof, uint32_t& ovf, bool act)
{
  uint64_t xit = ~0ull;
  const uint64_t rend16 = (rend + 15) & ~uint64_t(15);
  // (the resource moves with c: tails may be longer than 32-bit offsets; the
  // next 16 bytes load while these are walked)
  uint4 vn = xload16(xrsrc(g + ts, rend16 > ts ? rend16 - ts : 0), o);
  for (uint64_t c = 0; __ballot(act); c += 16) {
    const uint4 v = vn;
    const uint64_t cb = ts + c + 16;
    vn = xload16(xrsrc(g + cb, rend16 > cb ? rend16 - cb : 0), o);
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint64_t r = o + c + k;  // tile-relative position
      const uint64_t q = ts + r;
      bool go = act;
      if (go && q >= hi && !(id & XI_IN)) {  // no walk crosses into q: the chain is at q
        xit = q;
        act = go = false;
      }
      if (go && q >= rend) {  // readable end: at EOF the walk ends there
        if (!at_eof && (id & XI_IN)) ovf |= 1;
        xit = q;
        act = go = false;
      }
      const uint32_t e = xbyte(T, id, xsel4(v, k >> 2), k & 3);
      if (go) {
        if (q >= hi) {
          if ((e & XI_ST) || !(e & XI_IN)) {  // the walk crossing hi ended at q
            xit = q;
            act = false;
          } else {
            a.ins2 += XI_IN;
          }
        } else {
          const uint32_t st = e & XI_ST;
          a.cnt += st;
          a.pos += st ? r - seg : 0ull;
          a.ins2 += e & XI_IN;
          if (e & XI_Y) {
            xit = q + 1;
            act = false;
          }
        }
        id = e;
      }
    }
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
                                               uint64_t wlo, uint64_t hi, uint64_t fresh, uint64_t rend,
                                               uint32_t at_eof, XSum& a, uint64_t& fs, uint32_t& ovf)
{
  bool act = ts + seg + kXS > wlo && ts + seg < hi;
  bool synced = false;
  uint32_t id = 0;
  uint64_t xit = ~0ull;
  const uint64_t rend16 = (rend + 15) & ~uint64_t(15);
  uint4 vn = xload16(xrsrc(g + ts, rend16 > ts ? rend16 - ts : 0), seg);
  for (uint64_t c = 0; __ballot(act); c += 16) {
    const uint4 v = vn;
    const uint64_t cb = ts + c + 16;
    vn = xload16(xrsrc(g + cb, rend16 > cb ? rend16 - cb : 0), seg);
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint64_t r = c + k;  // segment-relative position
      const uint64_t q = ts + seg + r;
      bool go = act && q >= wlo;
      if (go && q == fresh) {
        id = 0;
        synced = true;
      }
      if (go && !synced && r >= (uint64_t)kXS) act = go = false;  // no sync in the segment: covered by a tail
      if (go && q >= hi && !(synced && (id & XI_IN))) {
        if (synced) xit = q;
        act = go = false;
      }
      if (go && q >= rend) {
        if (synced) {
          if (!at_eof && (id & XI_IN)) ovf |= 1;
          xit = q;
        }
        act = go = false;
      }
      const uint32_t e = xbyte(T, id, xsel4(v, k >> 2), k & 3);
      if (go) {
        if (q >= hi) {
          if ((e & XI_ST) || !(e & XI_IN)) {
            xit = q;
            act = false;
          } else {
            a.ins2 += XI_IN;
          }
        } else if (synced) {
          const uint32_t st = e & XI_ST;
          a.cnt += st;
          a.pos += st ? r : 0ull;
          a.ins2 += e & XI_IN;
          if ((e & XI_Y) && r >= (uint64_t)kXS) {  // the tail ends at a sync byte
            xit = q + 1;
            act = false;
          }
        } else if (e & XI_Y) {
          synced = true;
          fs = q;
        }
        id = e;
      }
    }
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

__global__ __launch_bounds__(kXWaves * 64) void xi_kernel(ScanParams P)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t xsm[];
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
    if (edge_lo || edge_hi) {
      uint64_t fs = ~0ull;
      xit = xslow_lane(T, P.g, ts, seg, wlo, P.hi, fresh, P.rend, P.at_eof, a, fs, ovf);
      f = fs;
    } else {
      // ---- fast tile: every lane segment lies inside [wlo, whi) ----
      bool synced = fresh == ts && lane == 0;  // fresh entry at the tile start
      uint32_t fs = ~0u, id = 0;
      uint4 cur[4], nxt[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) cur[k] = xload16(rs, seg + 16u * k);
      for (uint32_t b = 0; b < (uint32_t)kXBlocks; ++b) {
        const uint32_t nb = b + 1 < (uint32_t)kXBlocks ? b + 1 : b;
#pragma unroll
        for (int k = 0; k < 4; ++k) nxt[k] = xload16(rs, seg + nb * kXBlk + 16u * k);
        if (P.ablate == 6) {
          id ^= cur[0].x ^ cur[1].y ^ cur[2].z ^ cur[3].w;  // loads only (benchmarking; wrong counts)
        } else if (__ballot(!synced)) {
          xblock<true>(T, cur, id, a, synced, fs, b * kXBlk);
        } else {
          xblock<false>(T, cur, id, a, synced, fs, b * kXBlk);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
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
  if (entry == ~0ull) entry = exit;  // no sync byte in the whole range: the previous tail covers it
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

hipError_t launch_xi(const ScanParams& P, size_t smem, hipStream_t stream)
{
  hipLaunchKernelGGL(xi_kernel, dim3(P.grid), dim3(kXWaves * 64), smem, stream, P);
  return hipGetLastError();
}

hipError_t xi_occupancy(size_t smem, int* n)
{
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xi_kernel, kXWaves * 64, smem);
}

uint32_t xi_unit() { return kXTile; }
uint32_t xi_waves() { return kXWaves; }

}  // namespace ugpu
