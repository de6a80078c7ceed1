// dense_kernel.hip -- wave-persistent FIND kernel for patterns without a
// selective prefilter (C3 identifiers, C4 Unicode \w+: a match every few bytes).
//
// Replaces the reference's DFA opcode interpreter (lib/matcher.cpp:125-546) and
// FIND restart logic (:621-746) for such tables: there is no needle to skip to,
// so every byte goes through one DFA transition.
//
// Each wave owns a contiguous range of wave-tiles (64 lane segments of S bytes)
// and processes them in order, with no workgroup barrier after table staging:
//   1. the next tile (+ a 64-byte halo) arrives by coalesced 16 B/lane buffer
//      loads into registers while the current one is walked, and is written to
//      the wave's LDS buffer afterwards (S/4 odd: lanes at the same offset of
//      their segments read distinct banks);
//   2. every lane runs the FIND chain of its segment speculatively from the
//      segment start.  Restart-local tables (tables.hpp: C3, C4) use the FIND
//      transducer: all lanes in lockstep, bytes read a dword at a time, one
//      table lookup per byte that both continues and restarts walks
//      (lockstep_lane).  Other tables run the general walk with restarts
//      folded into selects (run_lane);
//   3. fix-up rounds: the true chain enters lane l at lane l-1's exit (DPP).
//      For restart-local tables a lane whose entry differs just drops the
//      speculative matches that start before the true entry (xt_correct);
//      otherwise both chains are re-walked in lock step until they meet
//      (merge_rel);
//   4. match counts and digests are summed tile-relative in 32 bits and folded
//      into 64-bit totals once per tile.
// Per-wave chain records (entry, exit, counts) are stitched by fix_kernel.
#include "device_common.hpp"

#include <type_traits>

namespace ugpu {

namespace {

constexpr int kDHalo = 64;  // bytes staged past the tile end (walks crossing the tile end)
constexpr uint32_t kLaneRounds = 16;  // in-wave fix-up rounds before UGPU_FLAG_BUDGET

template <int S>
struct DGeo {
  static_assert(S % 4 == 0 && (S / 4) % 2 == 1, "segment stride must be an odd number of dwords");
  static constexpr int kTileB = 64 * S;                           // wave-tile bytes
  static constexpr int kLoads = (kTileB + kDHalo + 1023) / 1024;  // 16 B/lane load instructions per tile
  static constexpr int kBuf = kLoads * 1024;                      // LDS bytes per wave
};

// Tile-relative match sums of one lane (positions < 2^16 past the tile start
// in practice; every sum wraps mod 2^32 and the per-tile totals fit).
//   cnt = #matches, sst = sum p, dsum = sum (31 p + len)
// so that with base = absolute position of tile offset 0:
//   digest += 31 base cnt + dsum,  dcap += cap1 (cnt (base + 1) + sst)
struct RelSums {
  uint32_t cnt = 0, sst = 0, dsum = 0;
  uint64_t scap = 0, sstcap = 0;  // generic accept indices only: sum cap, sum p cap
};

template <bool CAP1>
struct RelEm {
  RelSums r;
  const uint32_t* caps;
  uint32_t log_row;
  __device__ __forceinline__ void put(uint32_t p, uint32_t len, uint32_t le, int sign)
  {
    if constexpr (!CAP1) {
      if (caps[le >> log_row] == kCapRedo) return;  // (REDO: not reported; CAP1 tables have none)
    }
    const uint32_t sg = (uint32_t)sign;  // +1 / -1 (wraps)
    r.cnt += sg;
    r.sst += sg * p;
    r.dsum += sg * (31u * p + len);
    if constexpr (!CAP1) {
      const uint64_t cap = caps[le >> log_row];
      const uint64_t s64 = (uint64_t)(int64_t)sign;
      r.scap += s64 * cap;
      r.sstcap += s64 * cap * p;
    }
  }
};

// Absolute emitter for the OFFSETS pass.
struct AbsWriteEm {
  uint64_t base;  // absolute position of tile offset 0 (with delta)
  uint64_t idx, capacity;
  uint64_t* start;
  uint32_t* len;
  uint32_t* cap;
  const uint32_t* caps;
  uint32_t log_row;
  uint32_t overflow = 0;
  __device__ __forceinline__ void put(uint32_t p, uint32_t l, uint32_t le, int)
  {
    const uint32_t a = caps[le >> log_row];
    if (a == kCapRedo) return;  // (REDO: not reported)
    if (idx < capacity) {
      start[idx] = base + p;
      len[idx] = l;
      if (cap) cap[idx] = a;  // (NULL: 12-byte records, one accept index)
    } else {
      overflow = 1;
    }
    ++idx;
  }
};

// Window of one wave-tile: bytes [0, wlen) in LDS, [wlen, rlim) from global.
struct DWin {
  const uint8_t* lds;
  const uint8_t* g;  // global address of tile offset 0
  uint32_t wlen, rlim;
  uint32_t eof;
  // (an unconditional LDS read and a rare global branch: a select between the
  // two pointers would compile to a flat load)
  __device__ __forceinline__ uint32_t byte(uint32_t q) const
  {
    uint32_t v = lds[q < wlen ? q : 0u];
    if (q >= wlen) v = g[q];
    return v;
  }
};

// Longest match from p (tile-relative), the reference walk (lib/matcher.cpp:
// 207-217 TAKE, :528-541 HALT, :460-465 EOF).  Used by the fix-up and OFFSETS
// passes; the main pass inlines the same step into run_lane.
template <class TT>
__device__ __forceinline__ uint32_t walk_rel(const TT& T, const DWin& w, uint32_t p, uint32_t& le, uint32_t& ovf)
{
  uint32_t s = T.start, q = p, last = p;
  le = 0;
  for (;;) {
    if (q >= w.rlim) {
      if (!w.eof) ovf = 1;  // a live walk ran into the end of the readable bytes
      break;
    }
    const uint32_t e = T.step(s, w.byte(q));
    if (e == 0) break;
    s = e;
    ++q;
    if (e >= T.accb) {
      last = q;
      le = e;
    }
  }
  return last - p;
}

template <class TT, class Em>
__device__ __forceinline__ uint32_t step_rel(const TT& T, const DWin& w, uint32_t p, Em& em, int sign, uint32_t& ovf)
{
  uint32_t le;
  const uint32_t len = walk_rel(T, w, p, le, ovf);
  if (len) {
    em.put(p, len, le, sign);
    return p + len;
  }
  return p + 1;
}

// The speculative chain of one lane over [p, b): one transition per iteration,
// restarts folded in with selects (every lane advances every iteration).
// Chain state of one lane: walk start p, next byte q, DFA entry s, end of the
// last accept and its entry.
struct LaneWalk {
  uint32_t p, q, s, last, le;
};

// One transition for every lane whose chain is still inside its segment.
// GLOBAL = false: bytes come from LDS only, and a lane whose walk needs a byte
// past the staged window parks (returns with q >= lim); the caller finishes
// parked lanes with GLOBAL = true.  Keeping global loads out of the main loop
// matters: hipcc would otherwise wait for every outstanding load (the next
// tile's prefetch included) at each byte.
template <bool CAP1, bool GLOBAL, class TT>
__device__ __forceinline__ void run_lane(const TT& T, const DWin& w, LaneWalk& L, uint32_t b, RelEm<CAP1>& em,
                                         bool& hit_end)
{
  uint32_t p = L.p, q = L.q, s = L.s, last = L.last, le = L.le;
  const uint32_t lim = w.wlen < w.rlim ? w.wlen : w.rlim;
  const uint32_t top = lim - 1;  // lim >= 1 whenever a segment is non-empty
  // byte = the byte at q (valid when q < lim).  The byte at q+1 is read
  // alongside each transition: the next q is q+1 (alive), q (a match ended
  // just before this byte) or p+1 == q+1 (a one-byte miss), so the loop-
  // carried path holds a single LDS read (the transition); other restarts
  // (backtracking past q) re-read.
  uint32_t byte = w.lds[q < lim ? q : 0u];
  while (p < b) {
    bool inr = true;
    if (q >= lim) {  // rare: past the staged halo, or at the readable end
      inr = q < w.rlim;
      if constexpr (GLOBAL) {
        if (inr) byte = w.g[q];
      } else {
        if (inr) break;  // park
      }
      hit_end |= !inr;
    }
    const uint32_t q1 = q + 1;
    const uint32_t bn = w.lds[q1 < top ? q1 : top];
    uint32_t e = T.step(s, byte);
    e = inr ? e : 0u;
    const bool alive = e != 0;
    const bool acc = e >= T.accb;  // implies alive (accb > 0)
    last = acc ? q1 : last;
    if constexpr (!CAP1) le = acc ? e : le;
    // dead: emit [p, last) when non-empty, restart at max(last, p + 1)
    const bool m = !alive && last > p;
    if constexpr (CAP1) {
      em.r.cnt += m ? 1u : 0u;
      em.r.sst += m ? p : 0u;
      em.r.dsum += m ? __umul24(p, 30u) + last : 0u;  // 31 p + (last - p)
    } else {
      if (m) em.put(p, last - p, le, +1);
    }
    const uint32_t np = last > p + 1 ? last : p + 1;
    const uint32_t nq = alive ? q1 : np;
    byte = nq == q ? byte : bn;
    if (nq != q && nq != q1) byte = w.lds[nq < lim ? nq : 0u];  // backtrack (rare)
    p = alive ? p : np;
    q = nq;
    s = alive ? e : T.start;
    last = alive ? last : np;
  }
  L = LaneWalk{p, q, s, last, le};
}

// Re-enter a lane's segment [.., b) at xn instead of xo: walk the speculative
// (old) and the true (new) chains in lock step, subtracting the old matches and
// adding the new ones, until they meet (true: the exit is unchanged) or both
// leave the segment (false: nexit = the new exit).
template <class TT, class Em>
__device__ __forceinline__ bool merge_rel(const TT& T, const DWin& w, uint32_t xo, uint32_t xn, uint32_t b, Em& em,
                                          uint32_t& nexit, uint32_t& ovf)
{
  uint32_t po = xo, pn = xn;
  for (;;) {
    if (po == pn) return true;
    if (po >= b && pn >= b) {
      nexit = pn;
      return false;
    }
    if (po < pn)
      po = step_rel(T, w, po, em, -1, ovf);
    else
      pn = step_rel(T, w, pn, em, +1, ovf);
  }
}

__device__ __forceinline__ uint32_t dprev_lane(uint32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false); }

__device__ __forceinline__ uint32_t dscan_add(uint32_t v)
{
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

__device__ __forceinline__ void dwave_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint4 dload16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2 /* nt */);
  return uint4{v.x, v.y, v.z, v.w};
}

// Buffer resource of tile i of a wave (rel = readable bytes from the wave's
// first tile, rounded up to 16; bytes past it read as 0 and are never used).
template <int S>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dtile_rsrc(const uint8_t* wbase, uint32_t i, uint32_t rel)
{
  const uint32_t off = i * (uint32_t)DGeo<S>::kTileB;
  const uint32_t n = rel > off ? rel - off : 0u;
  const uint32_t lim = (uint32_t)(DGeo<S>::kTileB + kDHalo);
  const int nr = __builtin_amdgcn_readfirstlane((int)(n < lim ? n : lim));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wbase + off), (short)0, nr, 0x00020000);
}

// FIND transducer entries (tables.hpp xtrans): row offset | flags.
constexpr uint32_t kXtDead = 1;  // XT_DEAD: the walk died here; the row is the restart state
constexpr uint32_t kXtLive = 2;  // XT_LIVE: the restart at this byte begins a walk

// The transducer table seen as a plain DFA table by the general walks
// (fix-up, parked lanes, edge tiles, OFFSETS): a DEAD entry is the dead state.
template <int FMT>
struct XTab {
  const uint16_t* trans;
  const uint8_t* cls;
  uint32_t start, accb;
  __device__ __forceinline__ uint32_t step(uint32_t s, uint32_t b) const
  {
    const uint32_t e = FMT == 0 ? trans[s | b] : trans[s + cls[b]];
    return (e & kXtDead) ? 0u : e;
  }
};

// Lockstep FIND over one full lane segment [0, S) (lane-relative positions)
// for restart-local tables: one transducer lookup per byte for every lane,
// bytes read four at a time, no per-lane control flow (SURVEY Appendix A,
// restated for tables.hpp xtrans):
//   dead entry: emit [p, last) if last > p; the chain restarts at this byte
//               (p = last = q, or q + 1 when no walk begins here);
//   accepting entry: last = q + 1.
// Walks still alive at the segment end continue byte by byte (other lanes
// masked) until they die; a walk that reaches the staged window end `wend`
// parks for the general global-memory path.  cnt / sp / sl = number, sum of
// starts and sum of ends of the emitted matches (lane-relative).  Returns the
// lane's exit (first chain position >= S) unless parked.
template <int FMT, int S>
__device__ __forceinline__ uint32_t lockstep_lane(const uint16_t* xt, const uint8_t* lcls, const uint8_t* seg,
                                                  uint32_t wend, uint32_t start, uint32_t accb, uint32_t rowmask,
                                                  uint32_t& cnt, uint32_t& sp, uint32_t& sl, LaneWalk& park,
                                                  bool& parked, bool ablate_tail)
{
  uint32_t m = start, p = 0, last = 0;
#pragma unroll 2
  for (uint32_t i = 0; i < (uint32_t)S; i += 4) {
    const uint32_t x = *reinterpret_cast<const uint32_t*>(seg + i);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t b = (x >> (8 * k)) & 0xffu;
      const uint32_t col = FMT == 0 ? b : (uint32_t)lcls[b];
      const uint32_t e = xt[(m & rowmask) | col];
      const uint32_t q = i + k;
      const bool dead = (e & kXtDead) != 0;
      const bool em = dead && last > p;
      cnt += em ? 1u : 0u;
      sp += em ? p : 0u;
      sl += em ? last : 0u;
      const uint32_t pn = (e & kXtLive) ? q : q + 1;
      p = dead ? pn : p;
      last = e >= accb ? q + 1 : (dead ? pn : last);
      m = e;
    }
  }
  uint32_t ex = p;  // == S when no walk is open at the segment end
  bool act = p < (uint32_t)S && !ablate_tail;
  for (uint32_t q = S; __ballot(act); ++q) {
    if (act) {
      if (q >= wend) {
        park = LaneWalk{p, q, m & rowmask, last, 0};
        parked = true;
        act = false;
      } else {
        const uint32_t b = seg[q];
        const uint32_t e = xt[(m & rowmask) | (FMT == 0 ? b : (uint32_t)lcls[b])];
        if (e & kXtDead) {
          if (last > p) {
            cnt += 1;
            sp += p;
            sl += last;
          }
          const uint32_t c = last > p ? last : p + 1;  // the chain runs on from here to q
          ex = c > (uint32_t)S ? c : (uint32_t)S;
          act = false;
        } else {
          if (e >= accb) last = q + 1;
          m = e;
        }
      }
    }
  }
  return ex;
}

// Fix-up of one lane for restart-local tables: the speculative chain entered
// at `a` but the true chain enters at x (a < x).  A FIND chain passes through
// every position not strictly inside one of its matches, so when x is not
// inside a speculative match the two chains coincide from x on and the
// correction is just "drop the speculative matches starting before x"; they
// are found by re-running the transducer from a until the chain reaches x.
// Returns false when x lies strictly inside a speculative match (or the walk
// leaves the staged window): the caller falls back to merge_rel.
// All lanes with `act` run together, one byte per iteration, with selects
// only (a divergent loop with early exits cost more SALU exec-mask work than
// the walk itself).  ok = the shortcut held; the sums go to cnt/sst/dsum.
template <int FMT>
__device__ __forceinline__ bool xt_correct(const uint16_t* xt, const uint8_t* lcls, const uint8_t* lds, uint32_t wlen,
                                           uint32_t a, uint32_t x, bool act, uint32_t start, uint32_t accb,
                                           uint32_t rowmask, uint32_t& cnt, uint32_t& sst, uint32_t& dsum)
{
  uint32_t m = start, p = a, last = a, q = a;
  bool ok = true;
  uint32_t dc = 0, ds = 0, dd = 0;
  while (__ballot(act)) {
    // state at the top: chain position p (walk start) <= q
    const bool at = p >= x;        // the chain reached x: it passes through x iff p == x
    const bool out = q >= wlen;    // left the staged window
    const bool fin = act && (at || out);
    ok = fin ? (ok && at && p == x) : ok;
    act = act && !fin;
    const uint32_t b = lds[q < wlen ? q : 0u];
    const uint32_t e = xt[(m & rowmask) | (FMT == 0 ? b : (uint32_t)lcls[b])];
    const bool dead = act && (e & kXtDead) != 0;
    const bool em = dead && last > p;
    const bool inside = em && last > x;  // x strictly inside the match [p, last)
    const bool sub = em && !inside;
    dc += sub ? 1u : 0u;
    ds += sub ? p : 0u;
    dd += sub ? __umul24(p, 30u) + last : 0u;
    const bool passed = dead && q >= x;  // x lies in [last, q]: the chain runs through it
    ok = inside ? false : ok;
    act = act && !inside && !passed;
    const uint32_t pn = (e & kXtLive) ? q : q + 1;
    p = dead ? pn : p;
    last = (e >= accb) ? q + 1 : (dead ? pn : last);
    m = e;
    ++q;
  }
  if (ok) {
    cnt -= dc;
    sst -= ds;
    dsum -= dd;
  }
  return ok;
}

}  // namespace

template <int FMT, int S, bool CAP1, bool XT, bool WRITE>
__global__ __launch_bounds__((FMT == 0 ? kDWavesByte : kDWavesClass) * 64) void dense_kernel(ScanParams P)
{
  constexpr int kDWaves = FMT == 0 ? kDWavesByte : kDWavesClass;
  static_assert(!XT || CAP1, "the lockstep path sums matches for a single accept index");
  using G = DGeo<S>;
  using TT = typename std::conditional<XT, XTab<FMT>, Tab<FMT> >::type;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint8_t* buf = smem + wid * G::kBuf;
  uint16_t* ltrans = reinterpret_cast<uint16_t*>(smem + kDWaves * G::kBuf);
  uint32_t* lcaps = reinterpret_cast<uint32_t*>(ltrans + P.ntrans_pad);
  uint8_t* lcls = reinterpret_cast<uint8_t*>(lcaps + ((P.nstates + 3) & ~3u));
  {
    const uint4* src = reinterpret_cast<const uint4*>(XT ? P.xtrans : P.trans);
    uint4* dst = reinterpret_cast<uint4*>(ltrans);
    for (uint32_t i = tid; i < P.ntrans_pad / 8; i += kDWaves * 64) dst[i] = src[i];
    for (uint32_t i = tid; i < P.nstates; i += kDWaves * 64) lcaps[i] = P.caps[i];
    if constexpr (FMT == 1) {
      if (tid < 16) reinterpret_cast<uint4*>(lcls)[tid] = reinterpret_cast<const uint4*>(P.cls)[tid];
    }
  }
  __syncthreads();  // the only workgroup barrier: tables staged
  const TT T{ltrans, lcls, P.start, P.accb};
  const uint32_t rowmask = ~((1u << P.log_row) - 1u);

  const uint64_t gw = (uint64_t)blockIdx.x * kDWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * G::kTileB, P.lo, P.hi);
  const uint64_t whi = clampu(te * G::kTileB, P.lo, P.hi);
  const uint32_t n = (uint32_t)(te - tb);
  const uint64_t wb = tb * G::kTileB;
  const uint8_t* wbase = P.g + wb;
  const uint64_t rend16 = (P.rend + 15) & ~uint64_t(15);
  const uint64_t relw = rend16 > wb ? rend16 - wb : 0;
  const uint64_t span = (uint64_t)n * G::kTileB + kDHalo;
  const uint32_t rel = (uint32_t)(relw < span ? relw : span);
  const bool clip_lo = wlo != wb, clip_hi = whi != te * G::kTileB;

  uint64_t x = WRITE ? P.entries[gw] : wlo;  // true chain position (wave-uniform)
  uint64_t widx = WRITE ? P.out_base[gw] : 0;
  uint32_t ovf = 0, wover = 0;
  CountEm acc;

  uint4 c[G::kLoads];
  if (n > 0) {
    const __amdgpu_buffer_rsrc_t r0 = dtile_rsrc<S>(wbase, 0, rel);
#pragma unroll
    for (int k = 0; k < G::kLoads; ++k) c[k] = dload16(r0, 16u * lane + 1024u * k);
  }
  for (uint32_t i = 0; i < n; ++i) {
    // a wave that met chains which do not resynchronise stopped the scan: the
    // host redoes the range with the forest FIND, so the rest is wasted work
    if (__hip_atomic_load(P.flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & UGPU_FLAG_BUDGET) break;
    // stage tile i, then start loading tile i+1 (empty resource past the range)
    dwave_sync();  // every read of the previous tile is done
#pragma unroll
    for (int k = 0; k < G::kLoads; ++k) *reinterpret_cast<uint4*>(buf + 16 * lane + 1024 * k) = c[k];
    {
      const __amdgpu_buffer_rsrc_t rn = dtile_rsrc<S>(wbase, i + 1 < n ? i + 1 : n, i + 1 < n ? rel : 0u);
#pragma unroll
      for (int k = 0; k < G::kLoads; ++k) c[k] = dload16(rn, 16u * lane + 1024u * k);
    }
    dwave_sync();

    const uint64_t ts = wb + (uint64_t)i * G::kTileB;
    DWin w;
    w.lds = buf;
    w.g = P.g + ts;
    w.wlen = (uint32_t)(G::kTileB + kDHalo);
    {
      const uint64_t r = P.rend > ts ? P.rend - ts : 0;
      w.rlim = (uint32_t)(r < 0x7fffffffull ? r : 0x7fffffffull);
    }
    w.eof = P.at_eof;
    // lane segment [a, b) clipped to the wave's range
    const uint64_t sa = ts + (uint64_t)lane * S;
    const uint32_t a = (uint32_t)(clampu(sa, wlo, whi) - ts);
    const uint32_t b = (uint32_t)(clampu(sa + S, wlo, whi) - ts);
    const uint64_t tend = ts + G::kTileB;
    // true entry of lane 0 (x may lie past this tile after a very long match)
    const uint32_t x0 = (uint32_t)(x - ts < 0x7fffffffull ? x - ts : 0x7fffffffull);

    RelEm<CAP1> em;
    em.caps = lcaps;
    em.log_row = P.log_row;
    uint32_t ent = a, ex;
    bool hit_end = false;
    // interior tile: every segment whole and the staged window readable
    const bool interior = !((i == 0 && clip_lo) || (i + 1 == n && clip_hi)) && w.rlim >= w.wlen;
    if (XT && interior) {
      const uint32_t lb = (uint32_t)lane * S;
      uint32_t cnt = 0, sp = 0, sl = 0;
      LaneWalk park{};
      bool parked = false;
      ex = lb + lockstep_lane<FMT, S>(ltrans, lcls, buf + lb, w.wlen - lb, P.start, P.accb, rowmask, cnt, sp, sl, park,
                                      parked, P.ablate == 5);
      // lane-relative sums -> tile-relative: start = lb + p, 31 start + len = 30 p + end + 31 lb
      em.r.cnt = cnt;
      em.r.sst = sp + cnt * lb;
      em.r.dsum = 30u * sp + sl + 31u * lb * cnt;
      if (__ballot(parked)) {
        if (parked) {
          LaneWalk L{park.p + lb, park.q + lb, park.s, park.last + lb, 0};
          run_lane<CAP1, true>(T, w, L, b, em, hit_end);
          ex = L.p;
        }
      }
    } else {
      LaneWalk L{a, a, T.start, a, 0};
      run_lane<CAP1, false>(T, w, L, b, em, hit_end);
      if (__ballot(L.p < b)) run_lane<CAP1, true>(T, w, L, b, em, hit_end);  // parked lanes
      ex = L.p;
    }
    if (hit_end && !w.eof) ovf = 1;  // a live walk ran into the end of the readable bytes
    // fix-up rounds: lane l's true entry is lane l-1's exit.  Chains that do
    // not resynchronise move a wrong phase one lane per round: past
    // kLaneRounds the scan gives up (UGPU_FLAG_BUDGET) and the host resolves
    // the range with the forest FIND (forest.hip)
    // (only rounds that re-walk a segment count: an entry past a lane's
    // segment, e.g. the empty segments after hi, just passes through)
    for (uint32_t round = 0;;) {
      if (P.ablate == 4) break;  // benchmarking only: no fix-up (results are not matches)
      const uint32_t pv = dprev_lane(ex);
      const uint32_t nx = lane == 0 ? x0 : pv;
      const bool ch = nx != ent;
      if (!__ballot(ch)) break;
      if (__ballot(ch && ent < b) && ++round > kLaneRounds) {
        wover |= 2u;
        if (lane == 0) atomicOr(P.flags, UGPU_FLAG_BUDGET);
        break;
      }
      bool done = false;
      if constexpr (XT) {
        const bool skip = ch && nx >= b;  // the true chain skips the whole segment
        if (skip) {
          em.r = RelSums();
          ex = nx;
        }
        const bool need = ch && !skip;
        uint32_t c2 = em.r.cnt, s2 = em.r.sst, d2 = em.r.dsum;
        const bool ok = xt_correct<FMT>(ltrans, lcls, buf, w.wlen < w.rlim ? w.wlen : w.rlim, ent, nx, need, P.start,
                                        P.accb, rowmask, c2, s2, d2);
        if (need && ok) {
          em.r.cnt = c2;
          em.r.sst = s2;
          em.r.dsum = d2;
        }
        done = skip || (need && ok);
      }
      if (ch && !done) {
        uint32_t ne;
        if (!merge_rel(T, w, ent, nx, b, em, ne, ovf)) ex = ne;
      }
      if (ch) ent = nx;
    }
    if (wover & 2u) break;
    const uint32_t ex63 = (uint32_t)__builtin_amdgcn_readlane(ex, 63);
    x = (x >= tend) ? x : ts + ex63;

    const uint64_t base = ts + (uint64_t)P.delta;
    if constexpr (WRITE) {
      const uint32_t cl = em.r.cnt;
      const uint32_t incl = dscan_add(cl);
      const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
      AbsWriteEm we{base, widx + (incl - cl), P.out_capacity, P.out_start, P.out_len, P.out_cap, lcaps, P.log_row};
      uint32_t p = ent;
      while (p < b) p = step_rel(T, w, p, we, +1, ovf);
      wover |= we.overflow;
      widx += tot;
    } else {
      const uint64_t cn = em.r.cnt;
      acc.cnt += cn;
      acc.dg += 31 * cn * base + em.r.dsum;
      if constexpr (CAP1)
        acc.dc += (uint64_t)P.cap1 * (cn * (base + 1) + em.r.sst);
      else
        acc.dc += em.r.scap * (base + 1) + em.r.sstcap;
    }
  }
  if (n == 0) x = wlo;
  if (x < whi) x = whi;  // (exits are >= the range end)

  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (wover & 1u) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  if (wover & 2u) atomicOr(P.flags, UGPU_FLAG_BUDGET);
  if constexpr (!WRITE) {
    const uint64_t c0 = wave_sum(acc.cnt), d = wave_sum(acc.dg), dc = wave_sum(acc.dc);
    if (lane == 0) {
      BlockRec rec;
      rec.entry = wlo;
      rec.exit = n ? x : wlo;
      rec.cnt = c0;
      rec.dg = d;
      rec.dc = dc;
      rec.pad0 = rec.pad1 = rec.pad2 = 0;
      P.recs[gw] = rec;
    }
  }
}

// ---------------------------------------------------------------- launchers
namespace {

template <int FMT>
constexpr int seg_for() { return FMT == 0 ? kDSegByte : kDSegClass; }

template <int FMT, bool CAP1, bool XT, bool WRITE>
hipError_t dense_one(const ScanParams& P, size_t smem, hipStream_t stream)
{
  auto kern = dense_kernel<FMT, seg_for<FMT>(), CAP1, XT, WRITE>;
  static size_t attr_smem = 65536;
  if (smem > attr_smem) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    attr_smem = smem;
  }
  hipLaunchKernelGGL(kern, dim3(P.grid), dim3(dense_waves(FMT) * 64), smem, stream, P);
  return hipGetLastError();
}

template <int FMT, bool WRITE>
hipError_t dense_fmt(const ScanParams& P, size_t smem, hipStream_t stream)
{
  if (P.cap1 == 0) return dense_one<FMT, false, false, WRITE>(P, smem, stream);
  if (P.xtrans) return dense_one<FMT, true, true, WRITE>(P, smem, stream);
  return dense_one<FMT, true, false, WRITE>(P, smem, stream);
}

}  // namespace

uint32_t dense_unit(uint32_t format) { return 64u * (uint32_t)(format == 0 ? kDSegByte : kDSegClass); }

size_t dense_smem_bytes(uint32_t format, uint32_t ntrans_pad, uint32_t nstates)
{
  const size_t bufb = format == 0 ? DGeo<kDSegByte>::kBuf : DGeo<kDSegClass>::kBuf;
  size_t b = dense_waves(format) * bufb + 2 * (size_t)ntrans_pad + 4 * (size_t)((nstates + 3) & ~3u) + 256;
  return (b + 15) & ~size_t(15);
}

hipError_t launch_dense(const ScanParams& P, uint32_t format, bool write, size_t smem, hipStream_t stream)
{
  if (format == 0) return write ? dense_fmt<0, true>(P, smem, stream) : dense_fmt<0, false>(P, smem, stream);
  return write ? dense_fmt<1, true>(P, smem, stream) : dense_fmt<1, false>(P, smem, stream);
}

hipError_t dense_occupancy(uint32_t format, bool cap1, bool xt, size_t smem, int* n)
{
#define UGPU_DENSE_OCC(F, SEG, C, X) \
  hipOccupancyMaxActiveBlocksPerMultiprocessor(n, dense_kernel<F, SEG, C, X, false>, dense_waves(F) * 64, smem)
  if (format == 0)
    return !cap1 ? UGPU_DENSE_OCC(0, kDSegByte, false, false)
                 : (xt ? UGPU_DENSE_OCC(0, kDSegByte, true, true) : UGPU_DENSE_OCC(0, kDSegByte, true, false));
  return !cap1 ? UGPU_DENSE_OCC(1, kDSegClass, false, false)
               : (xt ? UGPU_DENSE_OCC(1, kDSegClass, true, true) : UGPU_DENSE_OCC(1, kDSegClass, true, false));
#undef UGPU_DENSE_OCC
}

}  // namespace ugpu
