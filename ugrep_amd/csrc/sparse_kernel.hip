// sparse_kernel.hip -- wave-persistent FIND kernel for prefiltered patterns
// (needle-like first bytes: C1 -F lorem, C2 foo|bar|baz).
//
// Replaces the reference's adv_ prefilter loop + per-candidate DFA walk
// (lib/matcher_avx2.cpp:475-527 ADV_PAT_PIN, lib/matcher.cpp:42-750) for byte
// tables whose first bytes have a small exact term cover (tables.hpp).
//
// Each wave owns a contiguous range of 4 KiB wave-tiles and walks it alone, so
// the main loop has no workgroup barrier:
//   1. 4 KiB wave-tiles arrive by coalesced non-temporal 16 B/lane loads into
//      two register sets used in turn (no LDS staging);
//   2. the prefilter reads chunk k of lane l = bytes [1024k + 16l, +16) from
//      registers -> per-byte candidate flags (3 v_perm + 4 ops per dword);
//   3. chunks with a candidate are ranked by a DPP scan and their candidates
//      appended in position order to a per-wave LDS list; when 64 are queued
//      they are walked at once, one per lane, each from its own 32-byte
//      window re-read from global memory; a walk from c is independent of the
//      chain, so all walks run in parallel;
//   4. the FIND chain over candidates is the greedy rule "keep the match at c
//      iff c >= end of the last kept match" (Appendix A: a non-candidate
//      position only steps p+1).  With an exclusive prefix-max of match ends
//      the rule is exact unless two candidate matches overlap; those batches
//      fall back to a 64-step in-wave sequential pass.
// Per-wave chain records (entry, exit, counts) are stitched by fix_kernel.
#include "device_common.hpp"

// The context-walk instantiations (word boundaries, line anchors) are built
// for UGPU_SP_CTX_OCC blocks of kSpWaves waves per CU: at 4 they hold their
// 95 VGPRs without spills (at 6: 80 VGPRs and 36 spilled) and their walks read
// the candidate's LDS window (UGPU_SP_CTX_WIN), with acap/amap in LDS
// (ScanParams::acap_lds): C2 \<(in|ut)\> 4.65 -> 4.24 ms, \bfoo\b 2.63 ->
// 2.58 ms (profiles/r05_ctx_walks_ab.json)
#ifndef UGPU_SP_CTX_OCC
#define UGPU_SP_CTX_OCC 4
#endif
#ifndef UGPU_SP_CTX_WIN
#define UGPU_SP_CTX_WIN 1
#endif

namespace ugpu {

namespace {

// Prefilter set bits of the 4 bytes of x (tables.hpp): three v_perm_b32
// byte-table lookups on the lo3 / mid3 / hi2 fields of every byte, ANDed.
// Byte i of the result holds B_g(i) at bit g, C_g(i) at bit 2+g, D_g(i) at
// bit 4+g; bits 6 and 7 are 0.
struct FTab {
  uint32_t t0lo, t0hi, t1lo, t1hi, t2;
};

__device__ __forceinline__ uint32_t bucket_bits(uint32_t x, const FTab& F)
{
  const uint32_t r0 = __builtin_amdgcn_perm(F.t0hi, F.t0lo, x & 0x07070707u);
  const uint32_t r1 = __builtin_amdgcn_perm(F.t1hi, F.t1lo, (x >> 3) & 0x07070707u);
  const uint32_t r2 = __builtin_amdgcn_perm(F.t2, F.t2, (x >> 6) & 0x03030303u);
  return r0 & r1 & r2;
}

// Candidate flags of one dword: bit g of byte i is set iff group g accepts
// bytes i, i+1, i+2.  R = set bits of the dword, Rn = of the next 4 bytes
// (0x3f3f3f3f when unknown: they pass).  alignbit(Rn, R, 10) moves byte
// i+1's bits 2,3 onto byte i's bits 0,1, alignbit(Rn, R, 20) byte i+2's bits
// 4,5; since bits 6,7 of every byte of R and Rn are 0, every other bit of the
// AND is 0.  One v_bitop3 + two v_alignbit per 4 positions.
__device__ __forceinline__ uint32_t cand_flags(uint32_t R, uint32_t Rn)
{
  return R & __builtin_amdgcn_alignbit(Rn, R, 10) & __builtin_amdgcn_alignbit(Rn, R, 20);
}

// 4-bit mask (bit i = byte i has a flag) of a cand_flags dword.
__device__ __forceinline__ uint32_t flags4(uint32_t X)
{
  return ((((X | (X >> 1)) & 0x01010101u) * 0x01020408u) >> 24);
}

// 4-bit mask (bit i = byte i is an ASCII letter) of a dword: lower-case the
// letters (| 0x20), then t >= 'a' and t <= 'z' per byte with the bytes' top
// bits as the comparison results (t <= 0x7f, so no carry crosses a byte);
// bytes >= 0x80 are no letters.
__device__ __forceinline__ uint32_t letters4(uint32_t x)
{
  const uint32_t t = (x | 0x20202020u) & 0x7f7f7f7fu;
  const uint32_t m = (t + 0x1f1f1f1fu) & ~(t + 0x05050505u) & ~x & 0x80808080u;
  return ((m >> 7) * 0x01020408u) >> 24;
}

// 16-bit mask of the ASCII letters among a lane's 16 bytes
__device__ __forceinline__ uint32_t letters16(const uint4& v)
{
  return letters4(v.x) | (letters4(v.y) << 4) | (letters4(v.z) << 8) | (letters4(v.w) << 12);
}

// Wave-wide inclusive scans by DPP row shifts + row broadcasts (no LDS round
// trip): row_shr 1,2,4,8 then row_bcast:15 (rows 1,3) and row_bcast:31 (rows 2,3).
__device__ __forceinline__ uint32_t dpp_scan_add(uint32_t v)
{
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t dpp_scan_max(uint32_t v)
{
  v = umax32(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));
  v = umax32(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));
  v = umax32(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));
  v = umax32(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));
  v = umax32(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
  v = umax32(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
  return v;
}

// value of lane-1 (wave_shr:1); lane 0 gets 0
__device__ __forceinline__ uint32_t dpp_prev_lane(uint32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false); }

__device__ __forceinline__ uint4 load16(const uint8_t* g, uint64_t pos, uint64_t last16)
{
  return *reinterpret_cast<const uint4*>(g + (pos < last16 ? pos : last16));
}

// Streaming tile loads.  Each byte is read once from HBM, so the loads carry
// the non-temporal hint (C2 16 GiB 2.93 -> 2.71 ms).  They go through a
// per-tile buffer resource (scalar base = tile start, num_records = readable
// bytes of the tile rounded up to 16): lane offsets are loop-invariant, there
// is no 64-bit address or clamp arithmetic per load, and 16-byte granules
// wholly past the readable end read as 0 (positions there are clipped, and a
// zero byte only ever fails or passes a prefilter test -- see tile_pass).
struct TileLoad {
  __amdgpu_buffer_rsrc_t rs;
};

__device__ __forceinline__ uint4 stream16(const TileLoad& L, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(L.rs, (int)off, 0, 2 /* nt */);
  return uint4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void wave_lds_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t ballot)
{
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(ballot >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ballot, 0u));
}

constexpr int kDefer = 64;                          // deferred candidates per wave (one walk batch)
constexpr int kAux = 2048;                          // per-wave aux LDS bytes
static_assert(kDefer * 8 <= kAux && 64 * 32 <= kAux, "aux region too small");

// Records staged by a COUNT pass for the OFFSETS pass (single-pass OFFSETS):
// the wave's slice of the staging arrays, filled in chain order from index 0.
struct Stage {
  uint64_t* start = nullptr;
  uint32_t* len = nullptr;
  uint32_t* cap = nullptr;
  uint64_t n = 0;       // records staged
  uint32_t over = 0;    // the slice was too small
};

// State of one wave's FIND chain over its tile range.
struct WaveChain {
  uint64_t x;      // end of the last kept match (wave-uniform): the chain resumes there
  uint32_t dn;     // deferred candidates in the list
  uint64_t widx;   // next output slot (WRITE)
  uint32_t wover;  // output capacity exceeded
  uint32_t ovf;    // a walk ran past the read window
  CountEm acc;
  Stage sg;        // COUNT pass with staging: the wave's staged records
  // COUNT pass: the first match the chain keeps (fix_kernel shortcuts) and
  // whether the chain ended in an open walk (OpenRec)
  uint32_t first, open;
  uint64_t c1, e1;
  uint32_t le1;
  // a batch left pending by flush_deferred (a walk outgrew its window), and
  // the position the tile loop resumes from (earlier candidates are consumed)
  uint32_t pend;
  uint64_t rs, ptile;  // (ptile: start of the tile the wave suspended in)
  // loop-needle tables (lb_batch): the range start, the last list entry's
  // position and run start
  uint64_t wlo;
  uint64_t lbr, lbs;
  uint64_t whi;  // the range end (dominated restarts stop there)
};

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);  // (readlane is int: no sign extension)
  return ((uint64_t)hi << 32) | lo;
}

// Greedy FIND rule over up to 64 walked candidates held one per lane in
// position order: keep the match at c iff c >= x, the end of the last kept
// match (Appendix A: a non-candidate position only steps p+1).  With the
// exclusive prefix-max of match ends (relative to x) the rule is exact unless
// two candidate matches overlap; those batches take a 64-step in-wave pass.
// COUNT: also stages the kept records (STAGE) and notes the first kept match.
template <bool WRITE, bool STAGE = false>
__device__ __forceinline__ void resolve(bool valid, uint64_t c, uint64_t len, uint32_t le, int lane, const Ctx& C,
                                        const ScanParams& P, WaveChain& w)
{
  const uint64_t x = w.x;
  const bool vm = valid && len != 0 && c >= x;
  const uint64_t endr = vm ? c + len - x : 0;  // > 0 for vm lanes
  const bool wide = __ballot(endr > 0xffffffffull) != 0;
  const uint32_t er = (uint32_t)endr, cr = vm ? (uint32_t)(c - x) : 0u;
  const uint32_t pm = dpp_prev_lane(dpp_scan_max(er));
  bool kept = vm && cr >= pm;
  if (wide || __ballot(vm && cr < pm)) {
    uint64_t xx = x;
    kept = false;
    const uint64_t e = vm ? c + len : 0ull;
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
      const uint64_t ci = __shfl(c, i, 64), ei = __shfl(e, i, 64);
      if (ei != 0 && ci >= xx) {
        if (lane == i) kept = true;
        xx = ei;
      }
    }
  }
  const uint64_t kb = __ballot(kept);
  if (!kb) return;
  // the reported ones: a kept match whose last accept is REDO moves the chain
  // but is not reported (WriteEm / CountEm skip it)
  const uint64_t rb = __ballot(kept && C.caps[le >> C.log_row] != kCapRedo);
  if constexpr (WRITE) {
    WriteEm we{w.widx + lanes_below(rb), P.out_capacity, P.out_start, P.out_len, P.out_cap};
    if (kept) we.put(C, c, len, le, +1);
    w.wover |= we.overflow;
    w.widx += __popcll(rb);
  } else {
    if (kept) w.acc.put(C, c, len, le, +1);
    if constexpr (STAGE) {
      WriteEm se{w.sg.n + lanes_below(rb), P.st_per, w.sg.start, w.sg.len, w.sg.cap};
      if (kept) se.put(C, c, len, le, +1);
      w.sg.over |= se.overflow;
      w.sg.n += __popcll(rb);
    }
    if (!w.first) {
      const int f = __builtin_ctzll(kb);
      w.first = 1;
      w.c1 = readlane64(c, f);
      w.e1 = w.c1 + readlane64(len, f);
      w.le1 = (uint32_t)__builtin_amdgcn_readlane(le, f);
    }
  }
  // kept matches are disjoint and ordered: the last one ends last
  w.x = readlane64(c + len, 63 - __builtin_clzll(kb));
}

// A walk continued by the whole wave (wave-uniform in and out).
struct CoopWalk {
  uint64_t last;  // last accept position (unchanged: none since the entry)
  uint32_t s;     // DFA entry at `lim` when the walk is still alive there
  uint32_t le;    // entry of the last accepting state
  uint32_t done;  // the walk ended: it died, or reached the end of the stream
  uint32_t ovf;   // it reached a readable end that is not the end of the stream
  uint64_t dpos;  // it died: one past the byte it died on (else 0)
};

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;

// Continue one walk -- DFA entry s before byte q, last accept `last` / `le` --
// with all 64 lanes, up to `lim` (<= rend).  A walk that outgrows its 32-byte
// window (a long match, e.g. `a+` over a run of `a`) would otherwise read one
// byte per dependent global load.  Each round stages the 1 KiB from q & ~15 in
// the wave's LDS scratch, 16 bytes per lane; every lane walks its 16 bytes
// from a guessed entry -- the walk's state run over the 4 bytes before them,
// which is exact whenever the state depends on the last few bytes only (a run
// of one byte, a `.*`-like loop) -- and the guesses are checked in lane order
// against the previous lane's exit (DPP).  The walk advances to the first lane
// whose guess was wrong, or dies in the first dying lane before it: at least
// the rest of lane 0's 16 bytes per round, up to 1 KiB.
// (noinline: called from the rare long-walk path, it keeps its registers out
// of the main loop's budget)
__device__ __forceinline__ CoopWalk coop_walk(const lds_u16* trans, uint32_t accb, const uint8_t* g,
                                                       uint64_t rend, uint32_t eof, lds_u8* scr, uint32_t s,
                                                       uint64_t q, uint64_t last, uint32_t le, uint64_t lim)
{
  const int lane = threadIdx.x & 63;
  const uint64_t last16 = (rend - 1) & ~uint64_t(15);
  CoopWalk r{last, s, le, 0u, 0u, 0ull};
  while (q < lim) {
    const uint64_t base = q & ~uint64_t(15);
    const uint64_t sa = base + 16u * (uint32_t)lane;
    uint4 v{0u, 0u, 0u, 0u};
    if (sa <= last16) v = *reinterpret_cast<const uint4*>(g + sa);
    wave_lds_sync();  // the previous round's reads are done
    {
      typedef __attribute__((address_space(3))) uint32_t lds_u32;
      lds_u32* d = reinterpret_cast<lds_u32*>(scr + 16 * lane);
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    wave_lds_sync();
    const uint64_t a = sa > q ? sa : q;
    const uint64_t z = sa + 16 < lim ? sa + 16 : lim;
    uint32_t spec = r.s;
    if (lane != 0) {
      uint32_t t = r.s;
#pragma unroll
      for (int k = 4; k > 0; --k) t = t ? (uint32_t)trans[t | scr[16 * lane - k]] : 0u;
      spec = t ? t : r.s;
    }
    uint32_t cur = spec, lel = 0;
    uint64_t lastl = 0;  // (an accept position follows a consumed byte: never 0)
    uint64_t dl = 0;
    bool died = false;
    for (uint64_t i = a; i < z; ++i) {
      const uint32_t e = trans[cur | scr[i - base]];
      if (e == 0) {
        died = true;
        dl = i + 1;
        break;
      }
      cur = e;
      if (e >= accb) {
        lastl = i + 1;
        lel = e;
      }
    }
    const uint32_t prev = dpp_prev_lane(cur);
    const bool seg = a < z;
    const uint64_t live = __ballot(seg);  // a prefix of the lanes (lane 0 owns q)
    const int nl = __popcll(live);
    const uint64_t bad = __ballot(seg && lane != 0 && spec != prev);
    const uint64_t dead = __ballot(seg && died);
    const uint64_t accm = __ballot(lastl != 0);
    const int j = bad ? __builtin_ctzll(bad) : nl;  // lanes [0, j) walked from their true entry
    const int d = dead ? __builtin_ctzll(dead) : 64;
    if (d < j) {  // the walk dies in lane d
      const uint64_t m = accm & lowbits((uint64_t)d + 1);
      if (m) {
        const int k = 63 - __builtin_clzll(m);
        r.last = readlane64(lastl, k);
        r.le = (uint32_t)__builtin_amdgcn_readlane(lel, k);
      }
      r.done = 1;
      r.dpos = readlane64(dl, d);
      return r;
    }
    const uint64_t m = accm & lowbits((uint64_t)j);
    if (m) {
      const int k = 63 - __builtin_clzll(m);
      r.last = readlane64(lastl, k);
      r.le = (uint32_t)__builtin_amdgcn_readlane(lel, k);
    }
    r.s = (uint32_t)__builtin_amdgcn_readlane(cur, j - 1);
    const uint64_t qn = base + 16u * (uint32_t)j;
    q = (j < nl || qn < lim) ? qn : lim;
  }
  if (lim >= rend) {  // alive at the end of the readable bytes: the walk ends there
    r.done = 1;
    r.ovf = eof ? 0u : 1u;
  }
  return r;
}

// Per-lane state of a walked batch (window-relative 32-bit offsets): st 0 =
// the walk ended, match [c, c + lr); 1 = alive at the window end, DFA entry s
// before byte c + qr, last accept c + lr; 2 = alive at the walk limit.
struct BatchLane {
  uint64_t c;
  uint32_t s, qr, lr, le, st;
  bool todo;  // not resolved yet
};

// Resolve a walked batch in position order up to the first lane whose walk
// outgrew its window and that the chain can still keep.  Returns that lane, or
// 64 when the whole batch is resolved.
template <bool WRITE, bool STAGE>
__device__ __forceinline__ int batch_resolve(BatchLane& L, int lane, const Ctx& C, const ScanParams& P, WaveChain& w)
{
  for (;;) {
    const uint64_t pend = __ballot(L.todo && L.st != 0);
    const int i = pend ? __builtin_ctzll(pend) : 64;
    // the candidates before lane i have their walks: resolve them
    resolve<WRITE, STAGE>(L.todo && lane < i, L.c, L.st == 0 ? (uint64_t)L.lr : 0ull, L.le, lane, C, P, w);
    if (!pend) return 64;
    L.todo = L.todo && lane > i;
    if (readlane64(L.c, i) >= w.x) return i;  // (else inside a kept match: never kept, its walk is not needed)
  }
}

// Lane i's walk outgrew its window: complete it with the whole wave
// (coop_walk) and resolve it.  A walk still alive at the walk limit: the COUNT
// pass records it as the wave's open walk (no match counted, nothing kept
// after it: fix_kernel finds its end from the next waves' records); the WRITE
// pass takes the end fix_kernel resolved when it is that walk, else walks on.
template <bool WRITE, bool STAGE>
__device__ __forceinline__ void long_lane(int i, const BatchLane& L, int lane, uint8_t* scr, const Tab<0>& T,
                                          const Ctx& C, const ScanParams& P, WaveChain& w, uint64_t lim, uint64_t gw)
{
  const uint64_t ci = readlane64(L.c, i);
  CoopWalk r{ci + (uint32_t)__builtin_amdgcn_readlane(L.lr, i), (uint32_t)__builtin_amdgcn_readlane(L.s, i),
             (uint32_t)__builtin_amdgcn_readlane(L.le, i), 0u, 0u, 0ull};
  if (__builtin_amdgcn_readlane(L.st, i) == 1)
    r = coop_walk((const lds_u16*)T.trans, T.accb, P.g, P.rend, P.at_eof, (lds_u8*)scr, r.s,
                  ci + (uint32_t)__builtin_amdgcn_readlane(L.qr, i), r.last, r.le, lim);
  // a walk alive at the range end usually ends a few bytes later (a needle
  // across the cut): walk on up to kOpenSlack bytes before calling it open
  uint64_t lim2 = lim;
  if (!r.done) {
    lim2 = lim + kOpenSlack < P.rend ? lim + kOpenSlack : P.rend;
    r = coop_walk((const lds_u16*)T.trans, T.accb, P.g, P.rend, P.at_eof, (lds_u8*)scr, r.s, lim, r.last, r.le, lim2);
  }
  w.ovf |= r.ovf;
  if (!r.done) {  // alive at lim2 (< rend), past the wave's range end
    if constexpr (!WRITE) {
      if (lane == 0) {
        OpenRec o{};
        o.c = ci;
        o.last = r.last;
        o.lim = lim2;
        o.s = r.s;
        o.le = r.le;
        P.open[gw] = o;
      }
      w.open = 1;
      if (!w.first) {
        w.first = 1;
        w.c1 = ci;
        w.e1 = kOpenEnd;
        w.le1 = 0;
      }
      w.x = kOpenEnd;
      return;
    } else {
      bool got = false;
      if (P.open && (P.recs[gw].pad2 & kRecOpen)) {
        const OpenRec o = P.open[gw];
        if (o.c == ci) {
          r.last = o.e;
          r.le = o.le_e;
          got = true;
        }
      }
      if (!got) {
        r = coop_walk((const lds_u16*)T.trans, T.accb, P.g, P.rend, P.at_eof, (lds_u8*)scr, r.s, lim2, r.last, r.le,
                      P.rend);
        w.ovf |= r.ovf;
      }
    }
  }
  resolve<WRITE, STAGE>(lane == i, L.c, r.last - ci, r.le, lane, C, P, w);
  // dominated restarts (tables.hpp dom_all): the failed walk from ci (on the
  // chain: batch_resolve hands over no candidate below w.x) crossed only
  // states that dominate the start, so no position up to the byte it died on
  // (or up to the end of the stream) starts a match: the chain resumes there,
  // at most at the range end (the exit the position-by-position chain has)
  if (P.dom_all && r.done && r.last == ci && !r.ovf) {
    const uint64_t sk = r.dpos ? r.dpos : P.rend;
    const uint64_t s2 = sk < w.whi ? sk : w.whi;
    if (s2 > w.x) w.x = s2;
  }
}

// Resolve a walked batch completely: in position order, each lane whose walk
// outgrew its window and that the chain can still keep is completed by the
// whole wave (long_lane), up to an open walk (nothing after it is kept).
template <bool WRITE, bool STAGE>
__device__ __forceinline__ void batch_finish(BatchLane& L, int lane, uint8_t* scr, const Tab<0>& T, const Ctx& C,
                                             const ScanParams& P, WaveChain& w, uint64_t lim, uint64_t gw)
{
  for (;;) {
    const int i = batch_resolve<WRITE, STAGE>(L, lane, C, P, w);
    if (i == 64) break;
    long_lane<WRITE, STAGE>(i, L, lane, scr, T, C, P, w, lim, gw);
    if (w.x == kOpenEnd) break;
  }
  wave_lds_sync();  // the aux region is reused
}

// Loop-needle tables (ScanParams::lb_cls, host_api.cpp loop_needle).  A list
// entry is a needle position, or (kLbStart set) a run start already: the
// wave's range start inside a run, and the run that reaches its range end.
constexpr uint64_t kLbStart = 1ull << 63;
__device__ __forceinline__ bool lb_in(const ScanParams& P, uint32_t b) { return (P.lb_cls[b >> 5] >> (b & 31)) & 1u; }

// The whole wave walks back from position pl (exclusive) over bytes of C, 64
// a step, not below bl: the start of the C-run that ends at pl (bl when the
// run reaches it)
__device__ __forceinline__ uint64_t lb_back_wave(const ScanParams& P, uint64_t pl, uint64_t bl, int lane)
{
  while (pl > bl) {
    const bool inr = (uint64_t)lane < pl - bl;
    const uint32_t b = inr ? (uint32_t)P.g[pl - 1 - lane] : 0u;
    const uint64_t stop = __ballot(inr && !lb_in(P, b));
    if (stop) return pl - (uint64_t)__builtin_ctzll(stop);
    if (pl - bl <= 64) return bl;
    pl -= 64;
  }
  return pl;
}

// The run starts of a batch of list entries (one per lane): each needle walks
// back over C to the previous entry (at most 64 bytes alone, then with the
// whole wave), so the walks of a batch cover the bytes between its entries
// once; a needle that reaches the previous entry is in its run.  Run starts
// never decrease along the list, so a max-scan hands each lane the start of
// the nearest entry on its left that found one (or the wave's carried run).
// A run begun before the wave's range starts at the range start: the wave's
// chain is FIND from there, as every kernel's speculative chain (fix_kernel
// stitches the true entries; the previous wave's range-end run converges with
// it within a few bytes).
__device__ __forceinline__ uint64_t lb_batch(const ScanParams& P, uint64_t e, bool listed, int lane, uint32_t dn,
                                             WaveChain& w)
{
  const bool fixed = listed && (e >> 63) != 0;
  const uint64_t n = listed ? (e & ~kLbStart) : w.lbr;
  // the previous entry's position (lane 0: the last entry of the previous batch)
  const uint32_t plo = (uint32_t)__shfl_up((int)(uint32_t)n, 1, 64);
  const uint32_t phi = (uint32_t)__shfl_up((int)(uint32_t)(n >> 32), 1, 64);
  uint64_t bound = lane == 0 ? w.lbr : (((uint64_t)phi << 32) | plo);
  if (bound < w.wlo) bound = w.wlo;
  if (bound > n) bound = n;
  uint64_t p = n;
  uint32_t steps = 0;
  if (listed && !fixed)
    while (p > bound && steps < 64 && lb_in(P, P.g[p - 1])) {
      --p;
      ++steps;
    }
  const bool longl = listed && !fixed && p > bound && lb_in(P, P.g[p - 1]);
  for (uint64_t lm = __ballot(longl); lm; lm &= lm - 1) {
    const int L = __builtin_ctzll(lm);
    const uint64_t r = lb_back_wave(P, readlane64(p, L), readlane64(bound, L), lane);
    if (lane == L) p = r;
  }
  // found: a run start of its own (a non-C byte before p, or a fixed entry)
  const bool found = fixed || (listed && p > bound) || (listed && p == bound && bound == w.wlo);
  uint64_t st = found ? p : 0;
  // inclusive max-scan over the wave (64-bit, as two 32-bit halves ordered by the high one)
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t lo2 = (uint32_t)__shfl_up((int)(uint32_t)st, d, 64);
    const uint32_t hi2 = (uint32_t)__shfl_up((int)(uint32_t)(st >> 32), d, 64);
    const uint64_t o = ((uint64_t)hi2 << 32) | lo2;
    if (lane >= d && o > st) st = o;
  }
  if (w.lbs > st) st = w.lbs;
  // carry: the batch's last entry and its run
  const int last = (int)dn - 1;
  w.lbr = readlane64(n, last);
  w.lbs = readlane64(st, last);
  return st;
}

// Walk the deferred candidates (one per lane) and resolve them.  Each lane
// copies the 32 bytes from c & ~15 into its LDS window (the tiles are gone
// from registers) and walks its candidate there.  A walk still alive at the
// window end (a long match, e.g. `a+` over a run of `a`) needs the whole wave
// (coop_walk): the main kernel then suspends the wave (w.pend: its state goes
// to P.srec) and the RESUME instantiation of the kernel, launched right
// after, completes the batch and the rest of the wave's tiles -- so the long
// path's registers never count against the main kernel's occupancy.  `lim`
// bounds every walk: the wave's range end when walks are truncated (P.open),
// else the readable end.  Option W (W = kWalkWord) and tables whose accepts
// depend on the context (W = kWalkCtx: word boundaries, line anchors) keep
// per-lane walks (walk<0, W>): option W's read the lane's window and, around
// it, global memory; the context walks read global memory.
template <bool WRITE, int ABL, int W = kWalkPlain, bool STAGE = false, bool RESUME = false, bool LB = false>
__device__ __forceinline__ void flush_deferred(const uint64_t* dl, uint8_t* scr, uint32_t dn, int lane, const Tab<0>& T,
                                            const Ctx& C, const ScanParams& P, WaveChain& w, uint64_t lim,
                                            uint64_t gw)
{
  wave_lds_sync();
  const bool listed = (uint32_t)lane < dn;
  const uint64_t craw = listed ? dl[lane] : 0;
  bool valid = listed;
  uint64_t c = craw;
  if constexpr (LB) c = lb_batch(P, craw, listed, lane, dn, w);
  const uint64_t a = c & ~uint64_t(15);
  if constexpr (W != kWalkCtx || UGPU_SP_CTX_WIN) {
    const uint64_t last16 = (P.rend - 1) & ~uint64_t(15);
    const uint4 v0 = load16(P.g, a, last16), v1 = load16(P.g, a + 16, last16);
    wave_lds_sync();  // every lane has read its list entry before the windows overwrite it
    *reinterpret_cast<uint4*>(scr + 32 * lane) = v0;
    *reinterpret_cast<uint4*>(scr + 32 * lane + 16) = v1;
  }
  wave_lds_sync();
  if constexpr (W != kWalkPlain) {
    uint64_t len = 0;
    uint32_t le = 0;
    if (valid && ABL != 3) {
      // option W: the walk checks at_wb/at_we (device_common.hpp); context
      // accepts: the walk bits at c, the position bits at each accepting
      // state (ctx_accept).  Either way the candidates stay a superset (W and
      // the contexts only remove matches, the first bytes are the table's),
      // so the prefilter is unchanged.
      // (the walk reads its lane's 32-byte LDS window [a, a + 32) where it
      // can, global memory around it -- option W: -w '[a-z]+ing' 54.6 -> 45.1
      // ms per 16 GiB, profiles/r05_sparse_walks_ab.json; the context walks:
      // UGPU_SP_CTX_WIN above)
      Win win = win_of(P);
      if constexpr (W == kWalkCtx) {
        if (P.acap_lds) {  // (C.caps: the LDS copy of acap, amap after it)
          win.acap = C.caps;
          win.amap = C.caps + P.acap_n;
        }
      }
      if constexpr (W == kWalkWord || UGPU_SP_CTX_WIN) {
        win.wl = scr + 32 * lane;
        win.wa = a;
        win.wn = 32;
      }
      len = walk<0, W>(T, win, c, le, w.ovf);
    }
    resolve<WRITE, STAGE>(valid, c, len, le, lane, C, P, w);
    wave_lds_sync();  // the aux region is reused
    return;
  }
  BatchLane L{c, T.start, 0u, 0u, 0u, 0u, valid};
  if (valid && ABL != 3) {
    const uint64_t wl = a + 32 < lim ? a + 32 : lim;
    const uint32_t wr = (uint32_t)(wl - c);
    for (;;) {
      if (L.qr >= wr) {
        if (c + L.qr >= P.rend) {
          if (!P.at_eof) w.ovf = 1;  // a live walk ran into the end of this shard's readable bytes
        } else {
          L.st = c + L.qr >= lim ? 2u : 1u;
        }
        break;
      }
      const uint32_t e = T.step(L.s, scr[32 * lane + (uint32_t)(c - a) + L.qr]);
      if (e == 0) break;
      L.s = e;
      ++L.qr;
      if (e >= T.accb) {
        L.lr = L.qr;
        L.le = e;
      }
    }
  }
  if (!__ballot(L.st != 0)) {  // (the common case: every walk ended in its window)
    resolve<WRITE, STAGE>(valid, c, L.lr, L.le, lane, C, P, w);
    wave_lds_sync();  // the aux region is reused
    return;
  }
  wave_lds_sync();  // (the windows are dead from here)
  if constexpr (RESUME) {
    batch_finish<WRITE, STAGE>(L, lane, scr, T, C, P, w, lim, gw);
  } else {
    PendSlot ps;
    ps.c = L.c;
    ps.s = L.s;
    ps.le = L.le;
    ps.packed = L.qr | L.lr << 8 | L.st << 16 | (uint32_t)L.todo << 24;
    ps.pad = 0;
    P.srec[gw].lanes[lane] = ps;
    w.pend = 1;
    w.rs = readlane64(LB ? craw & ~kLbStart : craw, (int)dn - 1) + 1;  // the batch's candidates are consumed (list positions)
  }
}

// Prefilter one 4 KiB wave-tile held in registers (v_k = chunk k: bytes
// [ts + 1024k + 16*lane, +16)) and append its candidates, in position order
// (chunk, then lane, then byte), to the deferred list; a full list (64, one
// per lane) is walked and resolved by flush_deferred.  edge: the tile is cut
// by the wave's range [wlo, whi).
// ABL (benchmarking only; results are not matches): 1 loads alone, 2 loads +
// prefilter, 3 everything but the walks.
template <bool WRITE, int ABL, int W = kWalkPlain, bool STAGE = false, bool RESUME = false, bool LB = false>
__device__ __forceinline__ void tile_pass(const uint4& v0, const uint4& v1, const uint4& v2, const uint4& v3,
                                          uint64_t ts, bool edge, uint64_t wlo, uint64_t whi, int lane,
                                          const FTab& F, const Tab<0>& T, const Ctx& C, const ScanParams& P,
                                          uint64_t* dl, uint8_t* scr, WaveChain& w, uint64_t lim, uint64_t gw)
{
  if constexpr (ABL == 1) {
    w.acc.cnt += (v0.x ^ v1.y ^ v2.z ^ v3.w) & 1;
    return;
  }
  if (!RESUME && w.pend) return;  // suspended: the rest of the range is the resume launch's
  // the 4 bytes after chunk k of a lane are the next lane's first dword
  // (DPP wave_shl:1), or lane 0's of chunk k+1 for lane 63; past the tile
  // they are unknown and pass
  const uint32_t h0 = bucket_bits(v0.x, F), h1 = bucket_bits(v1.x, F), h2 = bucket_bits(v2.x, F),
                 h3 = bucket_bits(v3.x, F);
  // (the DPP moves must run with every lane enabled -- a disabled source lane
  // reads as 0 -- so they are computed unconditionally, then selected)
  const uint32_t n0 = __builtin_amdgcn_update_dpp(0, h0, 0x130, 0xf, 0xf, false);
  const uint32_t n1 = __builtin_amdgcn_update_dpp(0, h1, 0x130, 0xf, 0xf, false);
  const uint32_t n2 = __builtin_amdgcn_update_dpp(0, h2, 0x130, 0xf, 0xf, false);
  const uint32_t n3 = __builtin_amdgcn_update_dpp(0, h3, 0x130, 0xf, 0xf, false);
  const uint32_t s1 = __builtin_amdgcn_readlane(h1, 0), s2 = __builtin_amdgcn_readlane(h2, 0),
                 s3 = __builtin_amdgcn_readlane(h3, 0);
  const bool l63 = lane == 63;
  const uint32_t e0 = l63 ? s1 : n0, e1 = l63 ? s2 : n1, e2 = l63 ? s3 : n2, e3 = l63 ? 0x3f3f3f3fu : n3;
  uint32_t X[4][4];
  {
    const uint32_t y = bucket_bits(v0.y, F), z = bucket_bits(v0.z, F), u = bucket_bits(v0.w, F);
    X[0][0] = cand_flags(h0, y);
    X[0][1] = cand_flags(y, z);
    X[0][2] = cand_flags(z, u);
    X[0][3] = cand_flags(u, e0);
  }
  {
    const uint32_t y = bucket_bits(v1.y, F), z = bucket_bits(v1.z, F), u = bucket_bits(v1.w, F);
    X[1][0] = cand_flags(h1, y);
    X[1][1] = cand_flags(y, z);
    X[1][2] = cand_flags(z, u);
    X[1][3] = cand_flags(u, e1);
  }
  {
    const uint32_t y = bucket_bits(v2.y, F), z = bucket_bits(v2.z, F), u = bucket_bits(v2.w, F);
    X[2][0] = cand_flags(h2, y);
    X[2][1] = cand_flags(y, z);
    X[2][2] = cand_flags(z, u);
    X[2][3] = cand_flags(u, e2);
  }
  {
    const uint32_t y = bucket_bits(v3.y, F), z = bucket_bits(v3.z, F), u = bucket_bits(v3.w, F);
    X[3][0] = cand_flags(h3, y);
    X[3][1] = cand_flags(y, z);
    X[3][2] = cand_flags(z, u);
    X[3][3] = cand_flags(u, e3);
  }
  // no match starts right after a word character (P.wstart): the candidates
  // that follow an ASCII letter in the lane's 16 bytes are dropped below (the
  // first byte's predecessor is another lane's: it stays; a digit, '_' or a
  // non-ASCII byte before a candidate keeps it too -- a superset).  The
  // letter masks are taken here, so that the tile's bytes die early.
  uint32_t lt01 = 0, lt23 = 0;
  if (P.wstart) {
    lt01 = letters16(v0) | (letters16(v1) << 16);
    lt23 = letters16(v2) | (letters16(v3) << 16);
  }
  const uint32_t any0 = X[0][0] | X[0][1] | X[0][2] | X[0][3], any1 = X[1][0] | X[1][1] | X[1][2] | X[1][3];
  const uint32_t any2 = X[2][0] | X[2][1] | X[2][2] | X[2][3], any3 = X[3][0] | X[3][1] | X[3][2] | X[3][3];
  // (tail: the tile holds the last two readable positions of a non-final range)
  const bool tail = !P.at_eof && ts + kWaveTile + 2 > P.rend && ts < P.rend;
  if (!tail && !__ballot((any0 | any1 | any2 | any3) != 0)) return;  // the common case: no candidate in the tile
  const uint32_t anyk[4] = {any0, any1, any2, any3};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (!tail && !__ballot(anyk[k] != 0)) continue;
    uint32_t mk = flags4(X[k][0]) | (flags4(X[k][1]) << 4) | (flags4(X[k][2]) << 8) | (flags4(X[k][3]) << 12);
    if (P.wstart) mk &= ~(((k < 2 ? lt01 : lt23) >> (16 * (k & 1))) << 1) & 0xffffu;
    const uint64_t p0 = ts + 1024u * k + 16u * lane;
    if (!P.at_eof && p0 + 18 > P.rend && p0 < P.rend) {
      // the last two readable positions of a non-final range: their prefilter
      // window reaches bytes not read yet (past rend the granule holds stale
      // bytes), so they stay candidates and their walks report HALO
      const uint64_t lo2 = P.rend >= 2 ? P.rend - 2 : 0;
      const uint64_t a = lo2 > p0 ? lo2 - p0 : 0, z = P.rend - p0 > 16 ? 16 : P.rend - p0;
      mk |= (uint32_t)((lowbits(z) & ~lowbits(a)) & 0xffffu);
    }
    if (edge) {
      const uint64_t a = wlo > p0 ? (wlo - p0 > 16 ? 16 : wlo - p0) : 0;
      const uint64_t z = whi > p0 ? (whi - p0 > 16 ? 16 : whi - p0) : 0;
      mk &= (uint32_t)((lowbits(z) & ~lowbits(a)) & 0xffffu);
    }
    const uint64_t xr = w.x > w.rs ? w.x : w.rs;
    if (xr > p0) {
      // positions below the end of the last kept match are never kept (the
      // chain resumes there): drop them before they are walked -- in a long
      // run of candidates only the batch holding its start is walked.  (w.x
      // comes from the batches flushed so far, so it can lag behind the
      // queued candidates: resolve drops those.)  Below w.rs: candidates a
      // pending batch already consumed, when the tile is processed again.
      const uint64_t a = xr - p0;
      mk &= (uint32_t)(~lowbits(a < 16 ? a : 16) & 0xffffu);
    }
    if constexpr (ABL == 2) {
      w.acc.cnt += __popc(mk);
      continue;
    }
    // rank this chunk's candidates by a DPP scan of the per-lane counts
    const uint32_t cnt = __popc(mk);
    const uint32_t incl = dpp_scan_add(cnt);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
    const uint32_t rank = incl - cnt;
    for (uint32_t done = 0; done < tot;) {
      if (w.dn == (uint32_t)kDefer) {
        flush_deferred<WRITE, ABL, W, STAGE, RESUME, LB>(dl, scr, w.dn, lane, T, C, P, w, lim, gw);
        w.dn = 0;
        if (!RESUME && w.pend) {  // the wave suspends (the resume launch repeats this tile)
          w.ptile = ts;
          return;
        }
      }
      const uint32_t take = tot - done < kDefer - w.dn ? tot - done : kDefer - w.dn;
      uint32_t m = mk, r = rank;
      while (m) {
        const uint32_t bit = __builtin_ctz(m);
        m &= m - 1;
        if (r - done < take) dl[w.dn + r - done] = p0 + bit;
        ++r;
      }
      w.dn += take;
      done += take;
    }
  }
}

// Buffer resource of tile i of a wave (base = the wave's first tile, rel =
// readable bytes from there rounded up to 16, < 2^32).
__device__ __forceinline__ TileLoad wave_tile(const uint8_t* wbase, uint32_t i, uint32_t rel)
{
  const uint32_t off = i * (uint32_t)kWaveTile;
  const uint32_t n = rel > off ? rel - off : 0u;
  // readfirstlane: the value is uniform, but without it hipcc computes it on
  // the VALU and wraps every load in a waterfall loop
  const int nr = __builtin_amdgcn_readfirstlane((int)(n < (uint32_t)kWaveTile ? n : (uint32_t)kWaveTile));
  return TileLoad{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wbase + off), (short)0, nr, 0x00020000)};
}

}  // namespace

template <bool WRITE, int ABL, int W = kWalkPlain, bool STAGE = false, bool RESUME = false, bool LB = false>
__global__ __launch_bounds__(kSpWaves * 64, RESUME ? 1 : (W == kWalkCtx ? UGPU_SP_CTX_OCC : 6)) void sparse_kernel(ScanParams P)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar control flow
  const uint64_t gw = (uint64_t)blockIdx.x * kSpWaves + wid;
  // RESUME: only the waves the main launch suspended (the others return)
  bool mine = true;
  if constexpr (RESUME) {
    mine = P.susp[gw] != 0;
    if (!__syncthreads_or(mine)) return;
  }
  // per-wave aux region, time-multiplexed: the deferred candidate list (u64)
  // and, while it is walked, the walk windows (32 B per lane) / coop_walk's
  // staging
  uint8_t* aux = smem + wid * kAux;
  uint64_t* dl = reinterpret_cast<uint64_t*>(aux);
  uint8_t* scr = aux;
  uint16_t* ltrans = reinterpret_cast<uint16_t*>(smem + kSpWaves * kAux);
  uint32_t* lcaps = reinterpret_cast<uint32_t*>(ltrans + P.ntrans_pad);
  {
    const uint4* src = reinterpret_cast<const uint4*>(P.trans);
    uint4* dst = reinterpret_cast<uint4*>(ltrans);
    for (uint32_t i = tid; i < P.ntrans_pad / 8; i += kSpWaves * 64) dst[i] = src[i];
    for (uint32_t i = tid; i < P.nstates; i += kSpWaves * 64) lcaps[i] = P.caps[i];
    if constexpr (W == kWalkCtx) {
      // (small context tables: acap, then amap, after the accept indices)
      if (P.acap_lds) {
        uint32_t* la = lcaps + P.nstates;
        for (uint32_t i = tid; i < P.acap_n; i += kSpWaves * 64) la[i] = P.acap[i];
        if (P.ctx_word)
          for (uint32_t i = tid; i < P.nstates; i += kSpWaves * 64) la[P.acap_n + i] = P.amap[i];
      }
    }
  }
  __syncthreads();  // the only workgroup barrier: tables staged
  if (!mine) return;
  const Tab<0> T{ltrans, nullptr, P.start, P.accb};
  // (context accepts: a walk's `le` is the acap index, whose entry is the accept index)
  const Ctx C = W == kWalkCtx ? Ctx{P.acap_lds ? lcaps + P.nstates : P.acap, 0u, P.delta}
                              : Ctx{lcaps, P.log_row, P.delta};
  const FTab F{P.ft[0], P.ft[1], P.ft[2], P.ft[3], P.ft[4]};

  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kWaveTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kWaveTile, P.lo, P.hi);
  WaveChain w;
  w.x = WRITE ? P.entries[gw] : wlo;
  w.dn = 0;
  w.widx = WRITE ? P.out_base[gw] : 0;
  w.wover = 0;
  w.ovf = 0;
  w.first = w.open = 0;
  w.c1 = w.e1 = 0;
  w.le1 = 0;
  w.pend = 0;
  w.rs = w.ptile = 0;
  w.wlo = wlo;
  w.whi = whi;
  w.lbr = w.lbs = wlo;
  // walk limit: with truncation (P.open) a walk still alive at the range end
  // of any wave but the last becomes the wave's open walk (fix_kernel); the
  // last wave's walks run to the readable end, as the range's exit needs
  const uint64_t lim = (W == kWalkPlain && P.open && whi < P.hi) ? whi : P.rend;
  if constexpr (WRITE && !RESUME) {  // single-pass OFFSETS: this wave's records were staged and copied already
    if (P.st_n && P.st_n[gw] == kStageDone) {
      if (P.susp && lane == 0) P.susp[gw] = 0;
      return;
    }
  }
  if constexpr (STAGE) {
    w.sg.start = P.st_start + gw * P.st_per;
    w.sg.len = P.st_len + gw * P.st_per;
    w.sg.cap = P.st_cap + gw * P.st_per;
  }

  // Tiles arrive by coalesced 16 B/lane loads into two register sets used in
  // turn (a* = tile i, b* = tile i+1): the load of the next tile is in flight
  // while the current one is filtered, with no register copies between
  // iterations.  All loop control is 32-bit scalar (tile index i < n, the
  // engine keeps n * 4 KiB < 4 GiB); past n the resource is empty (no access).
  const uint32_t n = (uint32_t)(te - tb);
  const uint8_t* wbase = P.g + tb * kWaveTile;
  const uint64_t rend16 = (P.rend + 15) & ~uint64_t(15), wb = tb * kWaveTile;
  const uint64_t relw = rend16 > wb ? rend16 - wb : 0;
  const uint32_t rel = (uint32_t)(relw < (uint64_t)n * kWaveTile ? relw : (uint64_t)n * kWaveTile);
  const bool clip_lo = wlo != wb, clip_hi = whi != te * kWaveTile;
  const uint32_t lo16 = 16u * lane;
  uint32_t i = 0;
  if constexpr (RESUME) {
    // the suspended state: the chain so far, then the pending batch
    const SuspRec& sr = P.srec[gw];
    w.x = sr.x;
    w.widx = sr.widx;
    w.wover = sr.wover;
    w.ovf = sr.ovf;
    w.acc.cnt = lane == 0 ? sr.cnt : 0;
    w.acc.dg = lane == 0 ? sr.dg : 0;
    w.acc.dc = lane == 0 ? sr.dc : 0;
    w.sg.n = sr.sgn;
    w.sg.over = sr.sgover;
    w.first = sr.first;
    w.open = sr.open;
    w.c1 = sr.c1;
    w.e1 = sr.e1;
    w.le1 = sr.le1;
    w.rs = sr.rs;
    w.lbr = sr.lbr;  // (the lookback carry: lane 0's walk-back stays bounded by the previous entry)
    w.lbs = sr.lbs;
    i = sr.tile;
    const PendSlot ps = sr.lanes[lane];
    BatchLane L{ps.c, ps.s, ps.packed & 0xffu, (ps.packed >> 8) & 0xffu, ps.le, (ps.packed >> 16) & 0xffu,
                (ps.packed >> 24) != 0};
    batch_finish<WRITE, STAGE>(L, lane, scr, T, C, P, w, lim, gw);
  }
  if constexpr (!RESUME && W != kWalkCtx) {
    // loop-needle tables: the range start inside a C-run is a candidate of its
    // own (the chain from there may match; no needle before it says so)
    if (LB && whi > wlo && lb_in(P, P.g[wlo])) {
      if (lane == 0) dl[0] = wlo | kLbStart;
      wave_lds_sync();
      w.dn = 1;
    }
  }
  uint4 a0, a1, a2, a3, b0, b1, b2, b3;
  {
    const TileLoad La = wave_tile(wbase, i, rel);
    a0 = stream16(La, lo16);
    a1 = stream16(La, lo16 + 1024);
    a2 = stream16(La, lo16 + 2048);
    a3 = stream16(La, lo16 + 3072);
    const TileLoad Lb = wave_tile(wbase, i + 1, rel);
    b0 = stream16(Lb, lo16);
    b1 = stream16(Lb, lo16 + 1024);
    b2 = stream16(Lb, lo16 + 2048);
    b3 = stream16(Lb, lo16 + 3072);
  }
  // one exit at the bottom (a mid-loop break let hipcc rotate the loop so that
  // its header waited on the loads just issued; a suspended wave streams the
  // rest of its range without processing it); an odd last tile follows
  if (n >= i + 2) {
    do {
      tile_pass<WRITE, ABL, W, STAGE, RESUME, LB>(a0, a1, a2, a3, wb + (uint64_t)i * kWaveTile, i == 0 && clip_lo, wlo, whi,
                                              lane, F, T, C, P, dl, scr, w, lim, gw);
      {
        const TileLoad L = wave_tile(wbase, i + 2, rel);
        a0 = stream16(L, lo16);
        a1 = stream16(L, lo16 + 1024);
        a2 = stream16(L, lo16 + 2048);
        a3 = stream16(L, lo16 + 3072);
      }
      tile_pass<WRITE, ABL, W, STAGE, RESUME, LB>(b0, b1, b2, b3, wb + (uint64_t)(i + 1) * kWaveTile, i + 2 == n && clip_hi,
                                              wlo, whi, lane, F, T, C, P, dl, scr, w, lim, gw);
      {
        const TileLoad L = wave_tile(wbase, i + 3, rel);
        b0 = stream16(L, lo16);
        b1 = stream16(L, lo16 + 1024);
        b2 = stream16(L, lo16 + 2048);
        b3 = stream16(L, lo16 + 3072);
      }
      i += 2;
    } while (i + 1 < n);
  }
  if (i < n)  // a* holds tile i = n - 1
    tile_pass<WRITE, ABL, W, STAGE, RESUME, LB>(a0, a1, a2, a3, wb + (uint64_t)i * kWaveTile,
                                            (i == 0 && clip_lo) || clip_hi, wlo, whi, lane, F, T, C, P, dl, scr, w,
                                            lim, gw);
  if constexpr (LB) {
    // loop-needle tables: the C-run that reaches the range end is this wave's
    // candidate (its needles may all lie in the next waves' ranges)
    if (!w.pend && whi > wlo && lb_in(P, P.g[whi - 1])) {
      const uint64_t r = lb_back_wave(P, whi, wlo, lane);
      {
        if (w.dn == (uint32_t)kDefer) {
          // (a suspension in this flush resumes straight into this block: no
          // tile is left to repeat)
          w.ptile = te * kWaveTile;
          flush_deferred<WRITE, ABL, W, STAGE, RESUME, LB>(dl, scr, w.dn, lane, T, C, P, w, lim, gw);
          w.dn = 0;
        }
        if (!w.pend) {
          wave_lds_sync();
          if (lane == 0) dl[w.dn] = r | kLbStart;
          wave_lds_sync();
          ++w.dn;
        }
      }
    }
  }
  if (!w.pend && w.dn) {
    flush_deferred<WRITE, ABL, W, STAGE, RESUME, LB>(dl, scr, w.dn, lane, T, C, P, w, lim, gw);
    w.ptile = te * kWaveTile;  // (no tile left to repeat)
  }
  if constexpr (!RESUME) {
    if (P.susp) {
      if (w.pend) {  // suspend: the resume launch continues from here
        const uint64_t c = wave_sum(w.acc.cnt), d = wave_sum(w.acc.dg), dc = wave_sum(w.acc.dc);
        if (lane == 0) {
          SuspRec* sr = P.srec + gw;
          sr->x = w.x;
          sr->widx = w.widx;
          sr->cnt = c;
          sr->dg = d;
          sr->dc = dc;
          sr->c1 = w.c1;
          sr->e1 = w.e1;
          sr->rs = w.rs;
          sr->lbr = w.lbr;
          sr->lbs = w.lbs;
          sr->sgn = w.sg.n;
          sr->wover = w.wover;
          sr->ovf = w.ovf;
          sr->first = w.first;
          sr->open = w.open;
          sr->le1 = w.le1;
          sr->sgover = w.sg.over;
          sr->tile = (uint32_t)((w.ptile - wb) / kWaveTile);
          sr->dn = 0;
          P.susp[gw] = 1;
        }
        return;
      }
      if (lane == 0) P.susp[gw] = 0;
    }
  }
  uint64_t x = w.x > whi ? w.x : whi;  // chain exit: the last kept match end or the range end
  if (tb == te) x = wlo;
  if (w.open) x = lim;  // (placeholder: fix_kernel resolves the open walk)

  if (w.ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (!WRITE && w.open && lane == 0) atomicOr(P.flags, UGPU_FLAG_OPEN);
  if (w.wover) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  if constexpr (!WRITE) {
    const uint64_t c = wave_sum(w.acc.cnt), d = wave_sum(w.acc.dg), dc = wave_sum(w.acc.dc);
    if (STAGE && lane == 0) P.st_n[gw] = w.sg.over ? kStageOver : (uint32_t)w.sg.n;
    if (lane == 0) {
      BlockRec rec;
      rec.entry = wlo;
      rec.exit = x;
      rec.cnt = c;
      rec.dg = d;
      rec.dc = dc;
      rec.pad0 = rec.pad1 = rec.pad2 = 0;
      if (W == kWalkPlain) {  // the first kept match (fix_kernel shortcuts), the open walk
        rec.pad0 = w.c1;
        rec.pad1 = w.first ? w.e1 : 0;
        rec.pad2 = (uint64_t)w.le1 | (w.open ? kRecOpen : 0) | kRecFirst;
      }
      P.recs[gw] = rec;
    }
  }
}

// ---------------------------------------------------------------- launchers
size_t sparse_smem_bytes(uint32_t ntrans_pad, uint32_t nstates, uint32_t nlds_acap)
{
  size_t b = (size_t)kSpWaves * kAux + 2 * (size_t)ntrans_pad + 4 * (size_t)nstates + 4 * (size_t)nlds_acap;
  return (b + 15) & ~size_t(15);
}

namespace {

template <bool WRITE, int ABL, int W = kWalkPlain, bool STAGE = false, bool RESUME = false, bool LB = false>
hipError_t sparse_launch(const ScanParams& P, size_t smem, hipStream_t stream)
{
  static size_t attr_smem = 65536;
  if (smem > attr_smem) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sparse_kernel<WRITE, ABL, W, STAGE, RESUME, LB>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_smem = smem;
  }
  hipLaunchKernelGGL((sparse_kernel<WRITE, ABL, W, STAGE, RESUME, LB>), dim3(P.grid), dim3(kSpWaves * 64), smem, stream,
                     P);
  return hipGetLastError();
}

// The main launch, then (plain walks) the resume launch for the waves it
// suspended at long walks.
template <bool WRITE, int ABL, int W = kWalkPlain, bool STAGE = false, bool LB = false>
hipError_t sparse_one(const ScanParams& P, size_t smem, hipStream_t stream)
{
  hipError_t e = sparse_launch<WRITE, ABL, W, STAGE, false, LB>(P, smem, stream);
  if constexpr (W == kWalkPlain && ABL == 0) {
    if (e == hipSuccess && P.susp) e = sparse_launch<WRITE, 0, kWalkPlain, STAGE, true, LB>(P, smem, stream);
  }
  return e;
}

// Single-pass OFFSETS, second half: one workgroup per staged wave record
// copies its records to their final slots (fix_kernel's output bases) when
// the wave's speculative chain was the true one (its exact entry equals its
// own) and its slice held them all; other waves are left to a WRITE pass
// (UGPU_FLAG_NEEDWRITE), which skips the copied ones.
__global__ __launch_bounds__(256) void stage_copy_kernel(ScanParams P)
{
  const uint32_t b = blockIdx.x;
  if (b >= P.nrec) return;
  const uint32_t n = P.st_n[b];
  const uint64_t base = P.out_base[b];
  const uint64_t next = b + 1 < P.nrec ? P.out_base[b + 1] : P.totals->count;
  const bool ok = n != kStageOver && P.entries[b] == P.recs[b].entry && next - base == n;
  __syncthreads();
  if (!ok) {
    if (threadIdx.x == 0) atomicOr(P.flags, UGPU_FLAG_NEEDWRITE);
    return;
  }
  if (base + n > P.out_capacity) {
    if (threadIdx.x == 0) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
    return;
  }
  const uint64_t s0 = (uint64_t)b * P.st_per;
  for (uint32_t i = threadIdx.x; i < n; i += 256) {
    P.out_start[base + i] = P.st_start[s0 + i];
    P.out_len[base + i] = P.st_len[s0 + i];
    if (P.out_cap) P.out_cap[base + i] = P.st_cap[s0 + i];
  }
  __syncthreads();
  if (threadIdx.x == 0) P.st_n[b] = kStageDone;
}

}  // namespace

hipError_t launch_stage_copy(const ScanParams& P, hipStream_t stream)
{
  hipLaunchKernelGGL(stage_copy_kernel, dim3(P.nrec), dim3(256), 0, stream, P);
  return hipGetLastError();
}

hipError_t launch_sparse(const ScanParams& P, bool write, size_t smem, hipStream_t stream)
{
  if (P.acap) {  // (word boundaries, line anchors: context accepts)
    if (write) return sparse_one<true, 0, kWalkCtx>(P, smem, stream);
    return P.st_n ? sparse_one<false, 0, kWalkCtx, true>(P, smem, stream)
                  : sparse_one<false, 0, kWalkCtx>(P, smem, stream);
  }
  if (P.lb_cls) {  // (loop-needle tables: lb_batch)
    if (P.wtab) {
      if (write) return sparse_one<true, 0, kWalkWord, false, true>(P, smem, stream);
      return P.st_n ? sparse_one<false, 0, kWalkWord, true, true>(P, smem, stream)
                    : sparse_one<false, 0, kWalkWord, false, true>(P, smem, stream);
    }
    if (write) return sparse_one<true, 0, kWalkPlain, false, true>(P, smem, stream);
    return P.st_n ? sparse_one<false, 0, kWalkPlain, true, true>(P, smem, stream)
                  : sparse_one<false, 0, kWalkPlain, false, true>(P, smem, stream);
  }
  if (P.wtab) {
    if (write) return sparse_one<true, 0, kWalkWord>(P, smem, stream);
    return P.st_n ? sparse_one<false, 0, kWalkWord, true>(P, smem, stream)
                  : sparse_one<false, 0, kWalkWord>(P, smem, stream);
  }
  if (write) return sparse_one<true, 0>(P, smem, stream);
  if (P.st_n) return sparse_one<false, 0, false, true>(P, smem, stream);
  switch (P.ablate) {  // benchmarking knob (UGPU_ABLATE): count pass only
    case 1: return sparse_one<false, 1>(P, smem, stream);
    case 2: return sparse_one<false, 2>(P, smem, stream);
    case 3: return sparse_one<false, 3>(P, smem, stream);
    default: return sparse_one<false, 0>(P, smem, stream);
  }
}

hipError_t sparse_occupancy(const ScanParams& P, size_t smem, int* n)
{
  (void)P;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, sparse_kernel<false, 0>, kSpWaves * 64, smem);
}

}  // namespace ugpu
