// xc_kernel.hip -- FIND over two-state tables by carry propagation: token
// patterns whose DFA is  start --G--> A,  A --X--> A  (A accepting, G a subset
// of X, every other edge dead), over ASCII byte sets: identifiers
// [A-Za-z_][A-Za-z0-9_]*, digit runs [0-9]+, ASCII words.  No table walk at all.
//
// What it replaces: the reference's per-match FIND loop (lib/matcher.cpp:
// 42-750) with its DFA opcode walk (:125-546) for such patterns; results are
// the same (count, digest = sum(31 start + len), dcap = sum((start + 1) cap)).
//
// The chain as an addition.  For such a table the FIND chain is inside a match
// at byte i (In_i) iff  In_i = G_i | (X_i & In_{i-1}):  a G byte starts or
// continues a match, a byte of X \ G (P) only continues one, any other byte
// (K) ends it.  That is the carry recurrence of a binary adder (G = generate,
// P = propagate), so In for a whole run of bytes is one integer addition: with
// every byte encoded as X' = 0x7F | X << 7 and G' = G << 7, the carry out of
// byte i of  S = X' + G' + carry_in  is In_i, and the byte (S ^ X' ^ G') is
// 0xFF exactly where the carry INTO byte i (In_{i-1}) is set.  Then
//   a match starts at i   <=>  G_i & !In_{i-1}
//   sum len = #In bytes = sum over bytes of In_{i-1}, corrected at the ends.
// Byte classes come from SWAR range tests on 4 bytes per dword (a host-built
// program of at most 6 ranges, tables.cpp), the adds are v_add_co/v_addc
// chains, the counts v_bcnt and v_dot4: about 5 VALU per byte, no LDS.
//
// Layout.  Fully coalesced: a wave reads 1 KiB chunks, 16 bytes per lane
// (lane l holds bytes [16 l, 16 l + 16)), four chunks in flight.  Lane
// carries are resolved per chunk by a carry-lookahead over the 64 lanes in
// scalar registers: lane l's carry-out with carry-in 0 (generate) and whether
// a carry-in would pass through it (propagate) are two ballots, and
// T = (gen | prop) + gen + c gives every lane's carry-in (T ^ (gen|prop) ^ gen).
// The wave's carry runs from chunk to chunk in an SGPR.
//
// Records.  A wave owns tiles [tb, te); its carry-in (is the chain inside a
// match at its first byte?) comes from a look-back over the chunk before it,
// which decides it unless that chunk is all P bytes (then further back; past
// 8 KiB of P bytes the scan sets UGPU_FLAG_BUDGET and the host resolves the
// range with the forest FIND).  With exact carries every wave counts exactly
// the starts and In bytes of its own byte range, so its record is
// (entry = its first byte, exit = its end) and fix_kernel merges nothing.  The
// wave holding the range end hi finds the chain exit: past hi no match starts
// (G = 0), the match crossing hi runs on through X bytes, and the exit is the
// first position >= hi whose carry-in is clear (capped at the readable end;
// a match reaching a non-EOF readable end raises UGPU_FLAG_HALO).
#include "device_common.hpp"
#include "tables.hpp"

namespace ugpu {

namespace {

constexpr int kCWaves = 4;             // waves per workgroup
constexpr uint32_t kCChunk = 1024;     // one wave-load: 16 bytes per lane
#ifndef UGPU_XC_ITER
#define UGPU_XC_ITER 4
#endif
#ifndef UGPU_XC_MINW
#define UGPU_XC_MINW 1  // waves per SIMD the register budget must allow
#endif
constexpr int kCIter = UGPU_XC_ITER;   // chunks per iteration (loads in flight per wave)
constexpr uint32_t kCTile = kCChunk * kCIter;
constexpr int kCLook = 8;              // look-back chunks before giving up

__device__ __forceinline__ uint4 cload(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2 /* nt */);
  return uint4{v.x, v.y, v.z, v.w};
}

// buffer resource over [base, base + readable) (zero fill past it; readable
// rounded up to the 16-byte granule by the caller)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t crsrc(const uint8_t* base, uint64_t readable)
{
  const uint32_t n = readable < 0x7fffff00ull ? (uint32_t)readable : 0x7fffff00u;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)n), 0x00020000);
}

// The class program (tables.hpp XcProg): NF range tests on the case-folded
// byte (b | 0x20) and NG on the byte itself give G, NP tests give X \ G.  A
// test of [lo, hi] on 7-bit v is bit 7 of (v + (0x80 - lo)) & ~(v + (0x7f - hi));
// bytes >= 0x80 are K.
template <int NF, int NG, int NP>
struct CProg {
  uint32_t k[14];
  __device__ __forceinline__ void operator()(uint32_t x, uint32_t& G, uint32_t& X) const
  {
    const uint32_t x7 = x & 0x7f7f7f7fu;
    uint32_t g = 0;
    if constexpr (NF > 0) {
      const uint32_t h = x7 | 0x20202020u;
#pragma unroll
      for (int i = 0; i < NF; ++i) g |= (h + k[2 * i]) & ~(h + k[2 * i + 1]);
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) g |= (x7 + k[4 + 2 * i]) & ~(x7 + k[5 + 2 * i]);
    G = g & ~x & 0x80808080u;
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < NP; ++i) p |= (x7 + k[10 + 2 * i]) & ~(x7 + k[11 + 2 * i]);
    X = (p & ~x) | G | 0x7f7f7f7fu;
  }
};

// The byte classes by lookup (the default): xc_cls[byte] = G << 7 | X << 6 in
// LDS, four independent ds_read_u8 per dword (any byte sets, ASCII or not).
// Text bytes < 0x80 sit in 32 dwords, one per bank: lanes never conflict.
struct CLds {
  const uint8_t* t;
  __device__ __forceinline__ void operator()(uint32_t x, uint32_t& G, uint32_t& X) const
  {
    const uint32_t r0 = t[x & 0xffu] | ((uint32_t)t[(x >> 16) & 0xffu] << 16);
    const uint32_t r1 = t[(x >> 8) & 0xffu] | ((uint32_t)t[x >> 24] << 16);
    const uint32_t e = r0 | (r1 << 8);
    G = e & 0x80808080u;
    X = (e << 1) | 0x7f7f7f7fu;  // (bit 7 of a byte shifts into the next byte's bit 0, which is set anyway)
  }
};

template <int NF, int NG, int NP>
struct CSel {
  typedef CProg<NF, NG, NP> type;
};
template <>
struct CSel<-1, 0, 0> {
  typedef CLds type;
};

// bytes of the dword at q that lie below lim (0xff per byte)
__device__ __forceinline__ uint32_t below(uint64_t q, uint64_t lim)
{
  const uint64_t n = lim > q ? lim - q : 0;
  return n >= 4 ? 0xffffffffu : (uint32_t)((1ull << (8 * n)) - 1);
}

// Byte limits of a masked chunk: positions < qlo and >= qr are K, positions
// >= qg start nothing.
struct CLim {
  uint64_t qlo, qg, qr;
};

// Classes of one lane's 16 bytes and its adder inputs.
struct CLane {
  uint32_t G[4], X[4], S[4];
};

// Option W (ugrep -w) for tables whose X is exactly the ASCII word bytes
// [0-9A-Za-z_] (tables.cpp xc_w): a match must start where at_wb holds, i.e.
// after a non-word byte, so a G byte starts a match only where the byte before
// it is not in X (an X-run beginning with a P byte, "9abc", yields nothing),
// and every match ends before a non-X byte, which is a non-word byte when it
// is ASCII (at_we holds).  Runs next to bytes >= 0x80 need the reference's
// UTF-8 decode (include/reflex/matcher.h:1194-1237): the wave flags any such
// byte and the host redoes the range with wfind_kernel.
struct CW {
  uint32_t cx = 0;   // bit 31: the byte before the chunk is in X (uniform)
  uint32_t hi = 0;   // lane: OR of the bytes seen (bit 7s: a byte >= 0x80)
  uint64_t bob = 0;  // buffer start (base coordinates): at_wb holds there
};

template <bool MASK, bool W, class PROG>
__device__ __forceinline__ void cclass(const PROG& pr, const uint4& v, CLane& L, uint64_t q, const CLim& lim, CW& wc)
{
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) pr(w[d], L.G[d], L.X[d]);
  if constexpr (W) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t m = 0xffffffffu;
      if constexpr (MASK) {  // bytes before the buffer are neither word bytes nor seen
        m = ~below(q + 4 * d, wc.bob);
        L.X[d] &= m | 0x7f7f7f7fu;
      }
      wc.hi |= w[d] & m;
    }
    // X of the byte before each byte: the previous dword, lane, or chunk
    const uint32_t lane = threadIdx.x & 63;
    uint32_t prev = __shfl_up(L.X[3], 1, 64);
    if (lane == 0) prev = wc.cx;
    wc.cx = __shfl(L.X[3], 63, 64);
    uint32_t xp[4];
    xp[0] = __builtin_amdgcn_alignbyte(L.X[0], prev, 3);
#pragma unroll
    for (int d = 1; d < 4; ++d) xp[d] = __builtin_amdgcn_alignbyte(L.X[d], L.X[d - 1], 3);
#pragma unroll
    for (int d = 0; d < 4; ++d) L.G[d] &= ~xp[d];
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if constexpr (MASK) {
      const uint64_t qd = q + 4 * d;
      const uint32_t live = ~below(qd, lim.qlo) & below(qd, lim.qr);
      L.G[d] &= live & below(qd, lim.qg);
      L.X[d] &= live | 0x7f7f7f7fu;
    }
  }
}

// Lane adders with carry-in 0: returns the lane's generate bit, sets prop.
__device__ __forceinline__ bool cadd(CLane& L, bool& prop)
{
  uint32_t k;
  L.S[0] = __builtin_addc(L.X[0], L.G[0], 0u, &k);
  L.S[1] = __builtin_addc(L.X[1], L.G[1], k, &k);
  L.S[2] = __builtin_addc(L.X[2], L.G[2], k, &k);
  L.S[3] = __builtin_addc(L.X[3], L.G[3], k, &k);
  prop = (L.S[0] & L.S[1] & L.S[2] & L.S[3]) == 0xffffffffu;
  return k != 0;
}

// Carry-lookahead over the lanes: the carry into each lane (bit l) given the
// carry c into lane 0; co = the carry out of lane 63.
__device__ __forceinline__ uint64_t clook(uint64_t gen, uint64_t prop, uint32_t c, uint32_t& co)
{
  const uint64_t xm = gen | prop;
  const uint64_t cin = (xm + gen + (uint64_t)c) ^ xm ^ gen;
  co = (uint32_t)((gen >> 63) | ((prop >> 63) & (cin >> 63)));
  return cin;
}

// Per-iteration lane sums: starts per chunk, 128 x start offsets in the lane
// (v_dot4 weights), carry-in bits (8 per In byte).
struct CIt {
  uint32_t cs[kCIter] = {};
  uint32_t ws = 0, ls = 0;
};

// Finish one chunk: final adds with the lane carry-in, then the events.
// Returns the lane's carry-in bytes (0xff where In_{i-1}) in cb.
__device__ __forceinline__ void cfinish(CLane& L, uint32_t ci, uint32_t& cs, uint32_t& ws, uint32_t& ls, uint32_t cb[4])
{
  uint32_t k;
  L.S[0] = __builtin_addc(L.S[0], ci, 0u, &k);
  L.S[1] = __builtin_addc(L.S[1], 0u, k, &k);
  L.S[2] = __builtin_addc(L.S[2], 0u, k, &k);
  L.S[3] = __builtin_addc(L.S[3], 0u, k, &k);
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t c = L.S[d] ^ L.X[d] ^ L.G[d];
    const uint32_t st = L.G[d] & ~c;
    cs = __builtin_popcount(st) + cs;
    ls = __builtin_popcount(c) + ls;
    const uint32_t wd = (4u * d) | ((4u * d + 1) << 8) | ((4u * d + 2) << 16) | ((4u * d + 3) << 24);
    ws = __builtin_amdgcn_udot4(st, wd, ws, false);
    cb[d] = c;
  }
}

// One chunk (16 bytes per lane at q = chunk base + 16 lane); cw = the wave's
// carry, updated.  Returns the lane's carry-in bytes.
template <bool MASK, bool W, class PROG>
__device__ __forceinline__ void cchunk(const PROG& pr, const uint4& v, uint64_t q, const CLim& lim, uint32_t& cw,
                                       uint32_t& cs, uint32_t& ws, uint32_t& ls, uint32_t cb[4], CW& wc)
{
#if defined(UGPU_XC_ABL) && UGPU_XC_ABL == 1  // loads only (benchmarking; wrong counts)
  if (!MASK) {
    cs += v.x ^ v.y ^ v.z ^ v.w;
    return;
  }
#endif
  CLane L;
#if defined(UGPU_XC_ABL) && UGPU_XC_ABL == 4  // trivial classes (benchmarking; wrong counts)
  if (!MASK) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      L.G[d] = w[d] & 0x80808080u;
      L.X[d] = w[d] | 0x7f7f7f7fu;
    }
  } else
#endif
  cclass<MASK, W>(pr, v, L, q, lim, wc);
  bool prop;
  const bool gen = cadd(L, prop);
#if defined(UGPU_XC_ABL) && UGPU_XC_ABL == 3  // no events (benchmarking; wrong counts)
  if (!MASK) {
    cs += L.S[0] ^ L.S[1] ^ L.S[2] ^ L.S[3] ^ (gen ? 1u : 0u) ^ (prop ? 2u : 0u);
    return;
  }
#endif
#if defined(UGPU_XC_ABL) && UGPU_XC_ABL == 2  // no lane carry-lookahead (benchmarking; wrong counts)
  if (!MASK) {
    cfinish(L, gen ^ prop ? 1u : 0u, cs, ws, ls, cb);
    return;
  }
#endif
  const uint64_t cin = clook(__ballot(gen), __ballot(prop), cw, cw);
  cfinish(L, __builtin_amdgcn_inverse_ballot_w64(cin) ? 1u : 0u, cs, ws, ls, cb);
}

// Exit search after a masked chunk of the wave holding hi: the exit is the
// first q >= hi with In_q clear (no match starts past hi, so q is the end of
// the match crossing hi, or hi), i.e. the first p = q + 1 > hi whose carry-in
// byte is clear; ~0 when there is none in this chunk.  Also flags a match that
// reaches the readable end rend (when not at EOF).
__device__ __forceinline__ uint64_t cexit(const uint32_t cb[4], uint64_t q, uint64_t hi, uint64_t rend, bool at_eof,
                                          uint32_t& ovf)
{
  uint32_t first = 64;  // byte index in the lane's 16 bytes
#pragma unroll
  for (int d = 3; d >= 0; --d) {
    const uint64_t qd = q + 4 * d;
    const uint32_t z = ~cb[d] & ~below(qd, hi + 1) & 0x80808080u;  // clear carry-in at a position > hi
    if (z) first = 4 * d + (__builtin_ctz(z) >> 3);
    if (!at_eof && rend >= qd && rend < qd + 4 && ((cb[d] >> (8 * (rend - qd))) & 0x80u)) ovf = 1;
  }
  const uint64_t m = __ballot(first < 64);
  if (!m) return ~0ull;
  const int l = __builtin_ctzll(m);
  const uint32_t f = (uint32_t)__shfl((int)first, l, 64);
  const uint64_t x = q - 16ull * (threadIdx.x & 63) + 16ull * l + f - 1;
  return x < rend ? x : rend;
}

}  // namespace

template <int NF, int NG, int NP, bool W>
__global__ __launch_bounds__(kCWaves * 64, UGPU_XC_MINW) void xc_kernel(ScanParams P)
{
  typename CSel<NF, NG, NP>::type pr;
  __shared__ uint32_t ctab[NF < 0 ? 64 : 1];
  if constexpr (NF < 0) {
    if (threadIdx.x < 64) ctab[threadIdx.x] = reinterpret_cast<const uint32_t*>(P.xc_cls)[threadIdx.x];
    __syncthreads();
    pr.t = reinterpret_cast<const uint8_t*>(ctab);
  } else {
#pragma unroll
    for (int i = 0; i < 14; ++i) pr.k[i] = P.xc[i];
  }
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kCWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kCTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kCTile, P.lo, P.hi);
  const uint32_t n = (uint32_t)(te - tb);
  const bool last_wave = n && whi == P.hi;
  const uint64_t rend16 = (P.rend + 15) & ~uint64_t(15);
  const uint32_t lo16 = 16u * (uint32_t)lane;
  CW wc;
  wc.bob = P.bob;
  // option W: bit 31 = the byte before position p is in X (at_wb fails there)
  auto xprev = [&](uint64_t p) -> uint32_t {
    if constexpr (W) {
      if (p <= P.bob) return 0u;
      return (uint32_t)(pr.t[P.g[p - 1]] & 0x40u) << 25;
    }
    return 0u;
  };

  // ---- the wave's carry-in: the chain enters P.lo fresh; other waves look back
  uint32_t cw = 0;
  if (n && wlo > P.lo) {
    bool known = false;
    for (int b = 1; b <= kCLook && !known; ++b) {
      const uint64_t cb0 = wlo - (uint64_t)b * kCChunk;  // wlo is tile aligned here
      const CLim lim{P.lo, wlo, wlo};
      CLane L;
      const uint4 v = cload(crsrc(P.g + cb0, rend16 > cb0 ? rend16 - cb0 : 0), lo16);
      wc.cx = xprev(cb0);
      cclass<true, W>(pr, v, L, cb0 + lo16, lim, wc);
      bool prop;
      const bool gen = cadd(L, prop);
      const uint64_t g = __ballot(gen), p = __ballot(prop);
      uint32_t c0, c1;
      (void)clook(g, p, 0u, c0);
      (void)clook(g, p, 1u, c1);
      if (c0 == c1 || cb0 <= P.lo) {  // decided by this chunk, or the chain enters at lo inside it
        cw = c0;
        known = true;
      }
    }
    if (!known) {
      // more than kCLook chunks of bytes that only continue matches: the carry
      // is unknown here; the host resolves the range with the forest FIND
      if (lane == 0) atomicOr(P.flags, UGPU_FLAG_BUDGET);
      cw = 0;
    }
  }
  const uint32_t cin0 = cw;

  uint64_t cnt = 0, pos = 0, lbits = 0;  // lane sums (absolute start positions)
  uint64_t exit = whi;
  uint32_t ovf = 0;
  bool found = false;
  const CLim lim{wlo, P.hi, P.rend};

  // Full tiles [ftb, fte) run the unmasked main loop; the chunks before them
  // (the first wave, lo not tile aligned) and after them (the wave holding hi,
  // then on past hi until the exit) run one masked chunk at a time, outside
  // the main loop's register budget.
  uint64_t ftb = (wlo + kCTile - 1) / kCTile, fte = whi / kCTile;
  if (!n || ftb >= fte) ftb = fte = 0;
  // one masked chunk at q0 (exit search on chunks reaching past hi)
  auto masked = [&](uint64_t q0) {
    const uint4 v = cload(crsrc(P.g + q0, rend16 > q0 ? rend16 - q0 : 0), lo16);
    uint32_t cs = 0, ws = 0, ls = 0, cb[4];
    cchunk<true, W>(pr, v, q0 + lo16, lim, cw, cs, ws, ls, cb, wc);
    cnt += cs;
    pos += (uint64_t)cs * (q0 + lo16) + (ws >> 7);
    lbits += ls;
    if (last_wave && !found && q0 + kCChunk > P.hi + 1) {
      const uint64_t x = cexit(cb, q0 + lo16, P.hi, P.rend, P.at_eof != 0, ovf);
      if (x != ~0ull) {
        exit = x;
        found = true;
      }
    }
  };
  uint64_t q0 = wlo & ~uint64_t(kCChunk - 1);
  wc.cx = xprev(fte > ftb && q0 >= ftb * kCTile ? ftb * kCTile : q0);
  wc.hi = 0;
#ifndef UGPU_XC_NOEDGE
  if (fte > ftb)
    for (; q0 < ftb * kCTile; q0 += kCChunk) masked(q0);
#endif

  uint4 cur[kCIter], nxt[kCIter];
  if (fte > ftb) {
    const uint64_t ts = ftb * kCTile;
    const __amdgpu_buffer_rsrc_t rs = crsrc(P.g + ts, rend16 > ts ? rend16 - ts : 0);
#pragma unroll
    for (int j = 0; j < kCIter; ++j) cur[j] = cload(rs, j * kCChunk + lo16);
  }
  for (uint64_t t = ftb; t < fte; ++t) {
    const uint64_t ts = t * kCTile;
    {
      const uint64_t tn = t + 1 < fte ? ts + kCTile : ts;
      const __amdgpu_buffer_rsrc_t rn = crsrc(P.g + tn, rend16 > tn ? rend16 - tn : 0);
#pragma unroll
      for (int j = 0; j < kCIter; ++j) nxt[j] = cload(rn, j * kCChunk + lo16);
    }
    CIt a;
    uint32_t cb[4];
#pragma unroll
    for (int j = 0; j < kCIter; ++j) cchunk<false, W>(pr, cur[j], 0, lim, cw, a.cs[j], a.ws, a.ls, cb, wc);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kCIter; ++j) c += a.cs[j];
    cnt += c;
    uint32_t cj = 0;
#pragma unroll
    for (int j = 1; j < kCIter; ++j) cj += j * a.cs[j];
    pos += (uint64_t)c * (ts + lo16) + (a.ws >> 7) + kCChunk * cj;
    lbits += a.ls;
#pragma unroll
    for (int j = 0; j < kCIter; ++j) cur[j] = nxt[j];
  }
  if (fte > ftb) q0 = fte * kCTile;
  // the rest of the wave's range; the wave holding hi goes on until the exit
  // (the match crossing hi runs on through X bytes, no starts past hi).  Bytes
  // past the readable end are K, so the search ends at the latest in the chunk
  // after the one holding rend (its loads read nothing: the resource is empty).
#ifndef UGPU_XC_NOEDGE
  if (n)
    for (; q0 < whi || (last_wave && !found); q0 += kCChunk) masked(q0);
#endif
  if (found) cw = 0;  // past the exit every carry is clear
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if constexpr (W) {
    if (__ballot((wc.hi & 0x80808080u) != 0) && lane == 0) atomicOr(P.flags, UGPU_FLAG_WSLOW);
  }
  const uint64_t c = wave_sum(cnt), s = wave_sum(pos), lb = wave_sum(lbits);
  if (lane == 0) {
    // In bytes = carry-in bits / 8, minus the carry into the first byte, plus
    // the carry out of the last processed byte
    const uint64_t len = n ? lb / 8 - cin0 + cw : 0;
    const uint64_t s_rep = s + c * (uint64_t)P.delta;  // reported starts
    BlockRec rec;
    rec.entry = wlo;
    rec.exit = n ? exit : wlo;
    rec.cnt = c;
    rec.dg = 31 * s_rep + len;
    rec.dc = (uint64_t)P.cap1 * (s_rep + c);
    rec.pad0 = rec.pad1 = rec.pad2 = 0;
    P.recs[gw] = rec;
  }
}

namespace {
template <int NF, int NG, int NP>
hipError_t launch_shape(const ScanParams& P, hipStream_t stream)
{
  if (P.xc_w)
    hipLaunchKernelGGL((xc_kernel<-1, 0, 0, true>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  else
    hipLaunchKernelGGL((xc_kernel<NF, NG, NP, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  return hipGetLastError();
}
#ifdef UGPU_XC_SWAR
template <int NF, int NG>
hipError_t launch_np(const ScanParams& P, uint32_t np, hipStream_t stream)
{
  switch (np) {
    case 0: return launch_shape<NF, NG, 0>(P, stream);
    case 1: return launch_shape<NF, NG, 1>(P, stream);
    default: return launch_shape<NF, NG, 2>(P, stream);
  }
}
template <int NF>
hipError_t launch_ng(const ScanParams& P, uint32_t ng, uint32_t np, hipStream_t stream)
{
  switch (ng) {
    case 0: return launch_np<NF, 0>(P, np, stream);
    case 1: return launch_np<NF, 1>(P, np, stream);
    case 2: return launch_np<NF, 2>(P, np, stream);
    default: return launch_np<NF, 3>(P, np, stream);
  }
}
#endif
}  // namespace

// The SWAR classifier (range tests instead of the LDS lookup) is a build
// option, UGPU_XC_SWAR (measured slower on C3: docs in DESIGN.md).
hipError_t launch_xc(const ScanParams& P, hipStream_t stream)
{
#ifdef UGPU_XC_SWAR
  const uint32_t nf = P.xc_shape & 15, ng = (P.xc_shape >> 4) & 15, np = (P.xc_shape >> 8) & 15;
  if (nf <= 1 && ng <= 3 && np <= 2 && nf + ng > 0)
    return nf ? launch_ng<1>(P, ng, np, stream) : launch_ng<0>(P, ng, np, stream);
#endif
  return launch_shape<-1, 0, 0>(P, stream);
}

hipError_t xc_occupancy(int* n)
{
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xc_kernel<-1, 0, 0, true>, kCWaves * 64, 0);
}
uint32_t xc_unit() { return kCTile; }
uint32_t xc_waves() { return kCWaves; }

}  // namespace ugpu
