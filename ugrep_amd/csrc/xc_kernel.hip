// xc_kernel.hip -- FIND over two-state tables by carry propagation: token
// patterns whose DFA is  start --G--> A,  A --X--> A  (A accepting, G a subset
// of X, every other edge dead): identifiers [A-Za-z_][A-Za-z0-9_]*, digit runs
// [0-9]+, byte-class words.  No table walk at all.
//
// What it replaces: the reference's per-match FIND loop (lib/matcher.cpp:
// 42-750) with its DFA opcode walk (:125-546) for such patterns; results are
// the same (count, digest = sum(31 start + len), dcap = sum((start + 1) cap)).
//
// The chain as an addition.  For such a table the FIND chain is inside a match
// at byte i (In_i) iff  In_i = G_i | (X_i & In_{i-1}):  a G byte starts or
// continues a match, a byte of X \ G (P) only continues one, any other byte
// (K) ends it.  That is the carry recurrence of a binary adder (G = generate,
// P = propagate), so In for a whole run of bytes is one integer addition.
// Every byte is coded  e = 0xFF (G), 0xFE (P), 0x00 (K)  and added to 0x01:
// 0xFF + 1 always carries out of the byte, 0xFE + 1 carries exactly when a
// carry comes in, 0x00 + 1 never does.  So with  S = e + 0x01010101 + c_in
// the carry out of byte i is In_i, and bit 0 of (S ^ e ^ 0x01010101) is the
// carry INTO byte i, In_{i-1}.  Then
//   a match starts at i   <=>  G_i & !In_{i-1}   (bit 0 of e & ~(S ^ e ^ 1))
//   sum len = #In bytes   = sum over bytes of In_{i-1}, corrected at the ends.
// The byte codes of two bytes at once come from one LDS lookup (a 64 Ki-entry
// u16 pair table built from the 256 byte classes in the prologue), the adds
// are v_add_co/v_addc chains, the counts v_bcnt and v_dot4.
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
// (G becomes P), the match crossing hi runs on through X bytes, and the exit is
// the first position >= hi outside a match (capped at the readable end; a
// match reaching a non-EOF readable end raises UGPU_FLAG_HALO).
#include "device_common.hpp"
#include "tables.hpp"

#include <type_traits>

namespace ugpu {

namespace {

#ifndef UGPU_XC_ITER
#define UGPU_XC_ITER 4
#endif
#ifdef UGPU_XC_BYTE
constexpr bool kCPair = false;  // byte-code lookups (4 per dword), measured against the pair table
#else
constexpr bool kCPair = true;   // pair-code lookups (2 per dword)
#endif
constexpr int kCWaves = kCPair ? 16 : 4;  // waves per workgroup (the pair table takes 128 KiB of LDS per CU)
constexpr uint32_t kCChunk = 1024;        // one wave-load: 16 bytes per lane
constexpr int kCIter = UGPU_XC_ITER;      // chunks per iteration (loads in flight per wave)
constexpr uint32_t kCTile = kCChunk * kCIter;
#ifndef UGPU_XU_ITER
#define UGPU_XU_ITER 2
#endif
// the COUNT pass's In-bit stores non-temporal: C3 OFFSETS 8.54 against 8.70 ms
// (xc_bm_kernel 3.57 against 3.72), C4 even; non-temporal loads of the bits in
// the expansion were slower (profiles/r05_offsets_ab.json)
#ifndef UGPU_XBM_NT
#define UGPU_XBM_NT 1
#endif
// U mode pair-table layout: 2 (default since round 6) = entry (x, y) at
// x << 8 | (y ^ x), one full-rate XOR per dword; 1 = at x << 8 | (y ^ (x << 2
// & 0xfc)) (a half-rate shift and a masked XOR); both spread ASCII lanes over
// the LDS banks.  0 = at x << 8 | y, so a lookup address is one v_perm of the
// lane's bytes -- 2.53 against 2.07 ms: without a swizzle ASCII text piles onto
// a few banks
#ifndef UGPU_XU_SWZ
#define UGPU_XU_SWZ 2
#endif
__device__ __forceinline__ uint32_t xu_swz(uint32_t x)
{
  return UGPU_XU_SWZ == 2 ? x : UGPU_XU_SWZ ? ((x << 2) & 0xfcu) : 0u;
}
// (round 6, on: C4 1.93-1.97 against 2.01-2.04 ms with the swizzle y ^ x and
// the one-shift fill, C3 -0.3 %; profiles/r06_c4_valu_ab.txt)
#ifndef UGPU_XC_ACC32
#define UGPU_XC_ACC32 1
#endif
#ifndef UGPU_XU_FIX7
#define UGPU_XU_FIX7 1
#endif
#ifndef UGPU_XU_PACK
#define UGPU_XU_PACK 1
#endif
constexpr int kUIter = UGPU_XU_ITER;  // U mode: fewer chunks in flight per wave, twice the waves
// U mode: the byte masks of the code arithmetic held in VGPRs (CU::k*,
// UGPU_XU_VK=1) instead of SGPRs / literals.  In isolation a v_bitop3 or v_add
// with an SGPR operand issued at half rate and the same instruction with three
// VGPR operands at full rate (tools/probe/valu_rate3.hip,
// profiles/r06_valu_rate3.txt); in this kernel the VGPR form measured even or
// slower (2.078-2.111 against 2.062-2.079 ms on C4, 13 against 6 spilled
// VGPRs; profiles/r06_c4_vk_ab.json), so it stays off
#ifndef UGPU_XU_VK
#define UGPU_XU_VK 0
#endif
static_assert(kCIter <= 4 && kUIter <= 4, "CIt");
constexpr int kCLook = 8;                 // look-back chunks before giving up
constexpr uint32_t kOnes = 0x01010101u;

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

// Byte codes of a dword (0xFF G, 0xFE P, 0x00 K per byte) from the LDS tables:
// the pair table (u16 codes of every byte pair) or the byte table.
struct CCodes {
  const uint16_t* pair;
  const uint8_t* byte;
  __device__ __forceinline__ uint32_t operator()(uint32_t x) const
  {
    if constexpr (kCPair) {
      return (uint32_t)pair[x & 0xffffu] | ((uint32_t)pair[x >> 16] << 16);
    } else {
      const uint32_t r0 = byte[x & 0xffu] | ((uint32_t)byte[(x >> 16) & 0xffu] << 16);
      const uint32_t r1 = byte[(x >> 8) & 0xffu] | ((uint32_t)byte[x >> 24] << 16);
      return r0 | (r1 << 8);
    }
  }
};

// bytes of the dword at q that lie below lim (0xff per byte)
__device__ __forceinline__ uint32_t below(uint64_t q, uint64_t lim)
{
  const uint64_t n = lim > q ? lim - q : 0;
  return n >= 4 ? 0xffffffffu : (uint32_t)((1ull << (8 * n)) - 1);
}

// Byte limits of a masked chunk: positions < qlo and >= qr are K, positions
// >= qg start nothing (G becomes P).
struct CLim {
  uint64_t qlo, qg, qr;
};

// Option W (ugrep -w) for tables whose X is exactly the ASCII word bytes
// [0-9A-Za-z_] (tables.cpp xc_w): a match must start where at_wb holds, i.e.
// after a non-word byte, so a G byte starts a match only where the byte before
// it is not in X (an X-run beginning with a P byte, "9abc", yields nothing),
// and every match ends before a non-X byte, which is a non-word byte when it
// is ASCII (at_we holds).  Runs next to bytes >= 0x80 need the reference's
// UTF-8 decode (include/reflex/matcher.h:1194-1237): the wave flags any such
// byte and the host redoes the range with wfind_kernel.
//
// Subset mode (ScanParams::xc_w == 2, tables.cpp xc_wsub: X a proper subset of
// the ASCII word bytes, [A-Za-z]+): the word bytes outside X get the code 0x02
// -- K for the adder (0x02 + 0x01 + carry never carries, and bit 0 is clear: no
// start), but bit 1 set, so the G -> P rule above sees them as word bytes.  A
// match then still starts only after a non-word byte; it must also END before
// one (at_we), which the forward chain cannot see at the start: a run of X
// followed by a word byte outside X ("abc1") is no match.  The wave flags any
// such end (an In byte followed by a 0x02 byte, wc.inv) and the host redoes the
// range with wfind_kernel, as for bytes >= 0x80; letter-only text never flags.
struct CW {
  uint32_t cx = 0;   // byte 3: the code of the byte before the chunk (uniform)
  uint32_t hi = 0;   // lane: OR of the bytes seen (bit 7s: a byte >= 0x80)
  uint64_t bob = 0;  // buffer start (base coordinates): at_wb holds there
  uint32_t sub = 0;  // (uniform) subset mode
  uint32_t inv = 0;  // lane: bit 0 of a byte: a match followed by a word byte outside X (subset mode)
};

// Codes and adder sums of one lane's 16 bytes.
struct CLane {
  uint32_t E[4], S[4];
};

template <bool MASK, bool W>
__device__ __forceinline__ void ccodes(const CCodes& cc, const uint4& v, CLane& L, uint64_t q, const CLim& lim,
                                       CW& wc)
{
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) L.E[d] = cc(w[d]);
  if constexpr (W) {
    if constexpr (MASK) {  // bytes before the buffer are K and not seen
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t m = ~below(q + 4 * d, wc.bob);
        L.E[d] &= m;
        wc.hi |= w[d] & m;
      }
    } else {
      wc.hi |= w[0] | w[1] | w[2] | w[3];
    }
    // a G byte whose previous byte is in X (code bit 1) becomes P: bit 1 of the
    // previous byte lands on bit 0 by one funnel shift (v_alignbit by 25)
    // (DPP wave_shr:1: lane l gets lane l-1's last dword, lane 0 keeps the
    // previous chunk's, held in wc.cx)
    const uint32_t prev = __builtin_amdgcn_update_dpp(wc.cx, L.E[3], 0x138, 0xf, 0xf, false);
    wc.cx = __builtin_amdgcn_readlane(L.E[3], 63);
    uint32_t xp[4];
    xp[0] = __builtin_amdgcn_alignbit(L.E[0], prev, 25);
#pragma unroll
    for (int d = 1; d < 4; ++d) xp[d] = __builtin_amdgcn_alignbit(L.E[d], L.E[d - 1], 25);
#pragma unroll
    for (int d = 0; d < 4; ++d) L.E[d] &= ~(xp[d] & kOnes);
  }
  if constexpr (MASK) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint64_t qd = q + 4 * d;
      const uint32_t live = ~below(qd, lim.qlo) & below(qd, lim.qr);
      L.E[d] &= live & (below(qd, lim.qg) | ~kOnes);
    }
  }
}

// ---- U mode: code-point runs (tables.hpp xu_*) ----------------------------
// The language is S+ for single-code-point tokens, so the FIND matches are the
// maximal runs of bytes inside a token (M bytes).  Each byte gets the code of
// the token starting at it (a thermometer of the bytes it covers, from one
// LDS byte lookup: ASCII bytes by themselves, continuation bytes all to one
// entry, lead bytes by (lead, next byte)); M_i = OR_k bit k of code_{i-k} by
// three funnel shifts; then e = 0xFF * M feeds the same adder as the two-state
// tables (past hi the M bytes become P: they only continue the match crossing
// hi).  Context: byte i's code reads bytes i+1, i+2 (the next lane's first
// dword by DPP wave_shl:1, lane 63 the next chunk's), M_i reads codes i-3..i-1
// (the previous lane's last code dword by DPP wave_shr:1, lane 0 the previous
// chunk's).  Bytes outside [lo, readable end) read as the table's fill byte.
struct CU {
  const uint8_t* tab = nullptr;   // LDS: kXuTab token codes
  const uint32_t* bm3 = nullptr;  // LDS: 3-byte completion bits
  uint32_t null4 = 0;             // the fill byte, in every byte
  uint64_t lo = 0, rend = 0;      // the bytes read as themselves
  uint32_t nx0 = 0;               // (uniform) the dword after the chunk, filled
  uint32_t cprev = 0;             // (uniform) codes of the 4 bytes before the chunk
  uint32_t slow = 0;              // lane: OR of the codes (bit 3: XU_SLOW, a 4-byte token)
  // option W (UW: tables equivalent to \w+): the lane's stray continuation
  // bytes right after a token byte (bit 0 of a byte; see umask)
  uint32_t risk = 0;
  uint32_t x8 = 0;  // lane (FAST main loop): OR of the codes, bit 3 = an XU_MIX or XU_SLOW lead
  // the masks 0x70707070, 0x80808080, 0x01010101, 0xfcfcfcfc (UGPU_XU_VK: in VGPRs)
  uint32_t k70 = 0x70707070u, k80 = 0x80808080u, k01 = 0x01010101u, kfc = 0xfcfcfcfcu;
  __device__ __forceinline__ void vk()
  {
#if UGPU_XU_VK
    // (an empty asm that "changes" them: the compiler can no longer fold them
    // into literals or SGPRs, so they stay VGPR operands)
    asm volatile("" : "+v"(k70), "+v"(k80), "+v"(k01), "+v"(kfc));
#endif
  }
};

// bytes of the dword at q inside [lo, rend) (0xff per byte)
__device__ __forceinline__ uint32_t uinside(const CU& u, uint64_t q) { return ~below(q, u.lo) & below(q, u.rend); }

// token codes of the 4 bytes of x (the next 4 bytes in nx); c7 = bit 7 of
// each continuation byte of x
__device__ __forceinline__ uint32_t ucode_dw(const CU& u, uint32_t x, uint32_t nx)
{
  // a 64 KiB table of every byte pair (built in the prologue from the host's
  // tables), entry (x, y) at x << 8 | (y ^ (x << 2 & 0xfc)): the swizzle
  // spreads the lanes of ASCII text over the banks.  (Addressing the host
  // tables directly, ASCII and continuation lanes on few dwords, had fewer
  // bank conflicts but 26 instead of 11 VALU per dword: 3.57 vs 3.17 ms on C4.)
#if UGPU_XU_SWZ
  const uint32_t y = __builtin_amdgcn_alignbit(nx, x, 8);
  const uint32_t sw = UGPU_XU_SWZ == 2 ? y ^ x : y ^ ((x << 2) & 0xfcfcfcfcu);
#endif
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#if UGPU_XU_SWZ
    const uint32_t a = __builtin_amdgcn_perm(x, sw, 0x0c0c0000u | (uint32_t)(4 + k) << 8 | (uint32_t)k);
#else
    const uint32_t a = __builtin_amdgcn_perm(nx, x, 0x0c0c0000u | (uint32_t)k << 8 | (uint32_t)(k + 1));
#endif
#if defined(UGPU_XU_ABL) && UGPU_XU_ABL == 1  // broadcast lookups: no bank conflicts (benchmarking; wrong counts)
    r |= (uint32_t)u.tab[a & 3u] << (8 * k);
#elif defined(UGPU_XU_ABL) && UGPU_XU_ABL == 2  // no LDS lookups (benchmarking; wrong counts)
    r |= ((a >> 13) & 1u) << (8 * k);
#else
    r |= (uint32_t)u.tab[a] << (8 * k);
#endif
  }
  return r;
}

// token codes of a lane's 16 bytes w (nx: the 4 bytes after them): all 16
// LDS addresses first, then the 16 lookups two to a VGPR (bytes k and k + 2
// of a dword in its 16-bit halves: ds_read_u8_d16 / ds_read_u8_d16_hi), so a
// wave waits on its lookups once instead of once per dword
__device__ __forceinline__ void ucode_lane(const CU& u, const uint32_t w[4], uint32_t nx, uint32_t c[4])
{
  typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
  uint32_t a[16];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t x = w[d];
#if UGPU_XU_SWZ
    const uint32_t y = __builtin_amdgcn_alignbit(d < 3 ? w[d + 1] : nx, x, 8);
    const uint32_t sw = UGPU_XU_SWZ == 2 ? y ^ x : y ^ ((x << 2) & u.kfc);
#pragma unroll
    for (int k = 0; k < 4; ++k) a[4 * d + k] = __builtin_amdgcn_perm(x, sw, 0x0c0c0000u | (uint32_t)(4 + k) << 8 | (uint32_t)k);
#else
    // (bytes k + 1 and k of the lane's stream, k + 1 = 4 being the next dword's first)
    const uint32_t xn = d < 3 ? w[d + 1] : nx;
#pragma unroll
    for (int k = 0; k < 4; ++k) a[4 * d + k] = __builtin_amdgcn_perm(xn, x, 0x0c0c0000u | (uint32_t)k << 8 | (uint32_t)(k + 1));
#endif
  }
#if UGPU_XU_PACK
  // (the four bytes of a dword packed by three v_lshl_or_b32 -- full-rate
  // VALU -- instead of two v_perm_b32, which issue at half rate on gfx950:
  // tools/probe/valu_rate.hip)
  uint32_t b[16];
#pragma unroll
#if defined(UGPU_XU_ABL) && UGPU_XU_ABL == 1  // broadcast lookups: no bank conflicts (benchmarking; wrong counts)
  for (int k = 0; k < 16; ++k) b[k] = u.tab[a[k] & 3u];
#elif defined(UGPU_XU_ABL) && UGPU_XU_ABL == 2  // no LDS lookups (benchmarking; wrong counts)
  for (int k = 0; k < 16; ++k) b[k] = (a[k] >> 13) & 1u;
#else
  for (int k = 0; k < 16; ++k) b[k] = u.tab[a[k]];
#endif
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t lo, hi;
    asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(lo) : "v"(b[4 * d + 1]), "v"(b[4 * d]));
    asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(hi) : "v"(b[4 * d + 3]), "v"(b[4 * d + 2]));
    asm("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(c[d]) : "v"(hi), "v"(lo));
  }
#else
  v2u16 r[8];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    r[2 * d].x = u.tab[a[4 * d]];
    r[2 * d].y = u.tab[a[4 * d + 2]];
    r[2 * d + 1].x = u.tab[a[4 * d + 1]];
    r[2 * d + 1].y = u.tab[a[4 * d + 3]];
  }
#pragma unroll
  for (int d = 0; d < 4; ++d)
    c[d] = __builtin_bit_cast(uint32_t, r[2 * d]) | (__builtin_bit_cast(uint32_t, r[2 * d + 1]) << 8);
#endif
}

// the code of byte 0 of x (byte 1 of x follows it)
__device__ __forceinline__ uint32_t ucode_b0(const CU& u, uint32_t x)
{
  const uint32_t a = ((x & 0xffu) << 8) | (((x >> 8) & 0xffu) ^ xu_swz(x & 0xffu));
  return u.tab[a];
}

// resolve the 3-byte tokens of code dword c (bytes x, next bytes nx; cn =
// the codes of the next 4 bytes): a 3-byte lead (XU_L3) shares a class bit
// with the code of the byte after it (which carries the class of the third
// byte) -- one AND for all 4 bytes.  EXACT: leads whose third bytes are no
// union of classes (XU_MIX, kernel code kUMix) ask the bitmap (the divergent
// loop); otherwise the caller knows that the dword has none.
constexpr uint32_t kUMix = 0xF8u;  // XU_MIX in the LDS table: bit 3 without bit 0 (XU_SLOW = 0x0F)
template <bool EXACT = true>
__device__ __forceinline__ uint32_t ucode_fix(const CU& u, uint32_t c, uint32_t x, uint32_t nx, uint32_t cn)
{
  const uint32_t cy = __builtin_amdgcn_alignbit(cn, c, 8);  // code of byte k + 1, in byte k
  uint32_t v7 = c & ((c & cy & u.k70) + u.k70) & u.k80;
  if constexpr (!EXACT) {
#if UGPU_XU_FIX7
    // (0x7f: bits 0-6; only bits 0-2 are read after the fix -- M, below -- so
    // one shift less than 0x07)
    c |= v7 - (v7 >> 7);
#else
    c |= (v7 >> 4) - (v7 >> 7);  // 0x07: the token covers x .. x + 2
#endif
    return c;
  }
  uint32_t mm = c & ~(c << 3) & 0x08080808u;  // XU_MIX leads
  v7 &= ~(mm << 4);
  c |= (v7 >> 4) - (v7 >> 7);
  while (mm) {
    const uint32_t j = (uint32_t)__builtin_ctz(mm) >> 3;
    const uint32_t b = __builtin_amdgcn_alignbit(nx, x, 8 * j);  // bytes x+j .. x+j+3
    const uint32_t i = (b & 15u) << 12 | ((b >> 8) & 63u) << 6 | ((b >> 16) & 63u);
    if (((u.bm3[i >> 5] >> (i & 31)) & 1u) && ((b >> 16) & 0xc0u) == 0x80u) c |= 7u << (8 * j);
    mm &= ~(0xffu << (8 * j));
  }
  return c;
}

// codes of the dword at q - 4 (for the chunk at q): every lane the same
__device__ __forceinline__ uint32_t ucode_before(const CU& u, const uint8_t* g, uint64_t q)
{
  if (q < 4) return 0;  // (the fill byte starts no token)
  const uint32_t* p = reinterpret_cast<const uint32_t*>(g + q - 4);
  const uint32_t x = (p[0] & uinside(u, q - 4)) | (u.null4 & ~uinside(u, q - 4));
  const uint32_t nx = q < u.rend ? (p[1] & uinside(u, q)) | (u.null4 & ~uinside(u, q)) : u.null4;
  return ucode_fix(u, ucode_dw(u, x, nx), x, nx, ucode_dw(u, nx, u.null4));
}

// the filled dword at q (uniform)
__device__ __forceinline__ uint32_t uload_dw(const CU& u, const uint8_t* g, uint64_t q)
{
  if (q >= u.rend) return u.null4;
  const uint32_t x = *reinterpret_cast<const uint32_t*>(g + q);
  return (x & uinside(u, q)) | (u.null4 & ~uinside(u, q));
}

// UW: continuation bytes of w in no token right after a token byte (bit 0 of a
// byte; m = M of the bytes, mp = M of the bytes before them)
__device__ __forceinline__ uint32_t ustray(uint32_t w, uint32_t m, uint32_t mp)
{
  return (w >> 7) & ~(w >> 6) & ~m & mp;
}

// One lane's 16 bytes at q: M (bit 0 of each byte: the byte lies inside a
// token).  FAST (the unmasked COUNT main loop of xu_kernel<.., false>): the
// 3-byte test runs without the XU_MIX bitmap and without the XU_SLOW check;
// the codes' bit 3 (an XU_MIX or XU_SLOW lead) is collected in u.x8, and the
// host redoes a range that met one with the exact kernel.  (Deciding that per
// chunk, by a ballot and a branch, cost 3.19 vs 2.22 ms on C4: the branch
// splits the chunk bodies, so the loads and LDS lookups of one chunk no longer
// overlap the VALU of the other.)
//
// UW (option W on tables equivalent to \w+): the matches are the
// runs, and at_wb / at_we (include/reflex/matcher.h:1194-1237) hold at their
// edges unless at_wb, after a continuation byte, decodes backwards to a word
// character: the first non-continuation byte j before the run start lies in a
// token.  The continuation bytes between j and the start are then not all in
// that token, so one of them is a stray continuation byte (in no token) right
// after a token byte -- which never occurs in valid UTF-8.  (at_we after a
// run: the byte is ASCII non-word, a continuation byte (true), or a lead whose
// restricted decode is a word character only when it starts a token, which
// would extend the run.)  u.risk collects such bytes; the host redoes a range
// with any with wfind_kernel.
// (F: 0 = the exact 3-byte test; 1 = FAST; 2 = the exact test in chunks where
// some lane of the wave met a code with bit 3, by a ballot: the exact kernel's
// main loop)
template <bool MASK, int F = 0, bool UW = false>
__device__ __forceinline__ void umask(CU& u, const uint4& v, uint64_t q, uint32_t m[4])
{
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (MASK) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t in = uinside(u, q + 4 * d);
      w[d] = (w[d] & in) | (u.null4 & ~in);
    }
  }
  const uint32_t nx = __builtin_amdgcn_update_dpp(u.nx0, w[0], 0x130, 0xf, 0xf, false);  // wave_shl:1
  uint32_t c[4];
#ifdef UGPU_XU_PERDW
#pragma unroll
  for (int d = 0; d < 4; ++d) c[d] = ucode_dw(u, w[d], d < 3 ? w[d + 1] : nx);
#else
  ucode_lane(u, w, nx, c);
#endif
  // the code of the byte after the lane (only its first byte is used)
  const uint32_t cn = __builtin_amdgcn_update_dpp(ucode_b0(u, u.nx0), c[0], 0x130, 0xf, 0xf, false);
  if constexpr (F == 1) u.x8 |= c[0] | c[1] | c[2] | c[3];
  bool exact = F == 0;
  if constexpr (F == 2) exact = __ballot(((c[0] | c[1] | c[2] | c[3]) & 0x08080808u) != 0) != 0;
  if (exact) {
#pragma unroll
    for (int d = 0; d < 4; ++d) u.slow |= c[d] & (c[d] << 3);  // bit 3: XU_SLOW
#pragma unroll
    for (int d = 0; d < 4; ++d) c[d] = ucode_fix<true>(u, c[d], w[d], d < 3 ? w[d + 1] : nx, d < 3 ? c[d + 1] : cn);
  } else {
#pragma unroll
    for (int d = 0; d < 4; ++d) c[d] = ucode_fix<false>(u, c[d], w[d], d < 3 ? w[d + 1] : nx, d < 3 ? c[d + 1] : cn);
  }
  const uint32_t cp = __builtin_amdgcn_update_dpp(u.cprev, c[3], 0x138, 0xf, 0xf, false);  // wave_shr:1
  u.cprev = __builtin_amdgcn_readlane(c[3], 63);
  // (bit 3, a 4-byte token's fourth byte, is not needed: XU_SLOW hands the
  // whole range to another kernel)
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t pv = d ? c[d - 1] : cp;
    m[d] = (c[d] | __builtin_amdgcn_alignbit(c[d], pv, 25) | __builtin_amdgcn_alignbit(c[d], pv, 18)) & u.k01;
  }
  if constexpr (UW) {
    // M of the byte before the lane's 16 bytes, from the previous lane's codes
    // (bit k of the code k + 1 bytes back); the fill byte is no continuation
    const uint32_t m0 = ((cp >> 24) | (cp >> 17) | (cp >> 10)) & 1u;
#pragma unroll
    for (int d = 0; d < 4; ++d) u.risk |= ustray(w[d], m[d], __builtin_amdgcn_alignbit(m[d], d ? m[d - 1] : m0 << 24, 24));
  }
}

// ... as the adder codes e = 0xFF * M (limits as ccodes)
template <bool MASK, bool UW = false>
__device__ __forceinline__ void ucodes(CU& u, const uint4& v, CLane& L, uint64_t q, const CLim& lim)
{
  uint32_t m[4];
  umask<MASK, 0, UW>(u, v, q, m);
#pragma unroll
  for (int d = 0; d < 4; ++d) L.E[d] = (m[d] << 8) - m[d];  // 0xff per M byte
  if constexpr (MASK) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint64_t qd = q + 4 * d;
      const uint32_t live = ~below(qd, lim.qlo) & below(qd, lim.qr);
      L.E[d] &= live & (below(qd, lim.qg) | ~kOnes);
    }
  }
}

// Lane adders with carry-in 0: returns the lane's generate bit, sets prop.
__device__ __forceinline__ bool cadd(CLane& L, bool& prop)
{
  uint32_t k;
  L.S[0] = __builtin_addc(L.E[0], kOnes, 0u, &k);
  L.S[1] = __builtin_addc(L.E[1], kOnes, k, &k);
  L.S[2] = __builtin_addc(L.E[2], kOnes, k, &k);
  L.S[3] = __builtin_addc(L.E[3], kOnes, k, &k);
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

// Per-iteration lane sums: starts per chunk, start offsets in the lane (v_dot4
// weights), carry-in bits (one per In byte).
struct CIt {
  uint32_t cs[4] = {};
  uint32_t ws = 0, ls = 0;
  // U mode COUNT (kXuCnt): byte-wise sums of the tile's start bits per dword
  // (sacc) and of its M bits (macc), folded into ws / ls once per tile
  uint32_t sacc[4] = {}, macc = 0;
};

// U mode COUNT: sums per byte instead of v_bcnt / v_dot4 per dword.  Those
// two issue at half rate on gfx950 (4 cycles per wave-instruction at 8 waves
// per SIMD, against 2 for v_add / v_bitop3: tools/probe/valu_rate.hip), so
// the start bits and M bits of a chunk are added byte-wise (a byte counts at
// most 4 per chunk) and folded by one v_dot4 each per chunk (starts: the
// chunk's count) or per tile (positions, In bytes).
#ifndef UGPU_XU_CNT
#define UGPU_XU_CNT 1
#endif
constexpr bool kXuCnt = UGPU_XU_CNT != 0;

// Finish one chunk: final adds with the lane carry-in, then the events.
// cb = the lane's carry-in bits (bit 0 of each byte: In_{i-1}).
__device__ __forceinline__ void cfinish(CLane& L, uint32_t ci, uint32_t& cs, uint32_t& ws, uint32_t& ls, uint32_t cb[4],
                                        uint32_t sb[4])
{
  uint32_t k;
  L.S[0] = __builtin_addc(L.S[0], ci, 0u, &k);
  L.S[1] = __builtin_addc(L.S[1], 0u, k, &k);
  L.S[2] = __builtin_addc(L.S[2], 0u, k, &k);
  L.S[3] = __builtin_addc(L.S[3], 0u, k, &k);
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t x = L.S[d] ^ L.E[d] ^ kOnes;
    const uint32_t c = x & kOnes;
    const uint32_t st = L.E[d] & ~x & kOnes;
    cs = __builtin_popcount(st) + cs;
    ls = __builtin_popcount(c) + ls;
    const uint32_t wd = (4u * d) | ((4u * d + 1) << 8) | ((4u * d + 2) << 16) | ((4u * d + 3) << 24);
    ws = __builtin_amdgcn_udot4(st, wd, ws, false);
    cb[d] = c;
    sb[d] = st;
  }
}

// OFFSETS pass (WRITE): the wave's output cursor (index of its next match
// start; fix_kernel's output base at the wave start) and the output arrays.
struct COut {
  uint64_t cur = 0;
  uint64_t* start = nullptr;
  uint32_t* len = nullptr;
  uint32_t* cap = nullptr;
  uint64_t capacity = 0;
  int64_t delta = 0;
  uint32_t cap1 = 0;
  uint32_t over = 0;
  // the match open at the chunk start (uniform): open = 1 when one is, its
  // reported start (~0: started by an earlier wave -- its len slot gets the end
  // position and fix, the index, for xc_fix_kernel)
  uint32_t open = 0;
  uint64_t open_start = ~0ull;
  uint64_t fix = ~0ull;
  uint16_t* stage = nullptr;  // the wave's LDS staging, two slots: kStage start offsets, then kStage end offsets
};

// lanes' 16-byte masks: bit 8j of dword d -> bit 4d + j
__device__ __forceinline__ uint32_t nib16(const uint32_t m[4])
{
  uint32_t r = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) r |= ((m[d] * 0x10204080u) >> 28) << (4 * d);
  return r;
}

__device__ __forceinline__ uint32_t cscan_add(uint32_t v)
{
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

__device__ __forceinline__ void cwave_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the staging capacity per wave, slot and kind (starts, ends): two slots of
// 960 B per wave for the pair classifier (30 KiB beside its 128 KiB table);
// U mode (UGPU_XC_STAGE_U) 2 KiB per wave beside its 72 KiB
constexpr uint32_t kStage = 240;
#ifndef UGPU_XC_STAGE_U
#define UGPU_XC_STAGE_U 256
#endif
constexpr uint32_t kStageU = UGPU_XC_STAGE_U;

// A chunk's staged records whose stores wait for the end of the tile (see
// cflush); all uniform.
struct CPend {
  uint64_t q0 = 0, cur = 0, open_start = ~0ull;
  uint32_t R = 0, E = 0, open = 0;
};

// Write the chunk's match records.  An end at position e (In_{e-1} set, In_e
// clear or a new start at e) closes the latest match started before it;
// starts get consecutive indices in chain order.  The chunk's start and end
// offsets are staged in LDS slot `slot` of the wave (ordered by a wave scan of
// the lanes' counts); cflush then writes them by consecutive lanes: start[],
// cap[] and the lengths (end - start: the start is staged too, or the open
// match's) leave as coalesced stores.  A match opened by an earlier wave gets
// its raw end position and is fixed by xc_fix_kernel.  Chunks with more than
// kStage starts or ends take the per-lane path (stores at once).
//
// The main loop stages a tile's chunks, waits for the next tile's loads (and
// with them the previous tile's stores: gfx950 counts loads and stores in one
// in-order vmcnt) and only then issues the tile's stores (cflush), so that no
// store of a tile is waited for before a whole tile of work.  Measured: the
// same time as storing right after each chunk (C4 OFFSETS 8.4 ms per step
// either way); the pass is bound by its own work -- taking the stores out
// (with their LDS reads) saves 1.9 ms, the staging another 2.0 ms, against
// 2.1 ms for the scan itself.
template <uint32_t kStage>
__device__ __forceinline__ void cwrite(const CLane& L, const uint32_t cb[4], const uint32_t sb[4], uint64_t q, COut& o,
                                       CPend& pd, uint16_t* slot)
{
  uint32_t enm[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t c = cb[d], st = sb[d];
    const uint32_t in = (L.E[d] | ((L.E[d] >> 1) & c)) & kOnes;  // In_i = G_i | X_i & In_{i-1}
    enm[d] = c & (~in | st);
  }
  const uint32_t s16 = nib16(sb), e16 = nib16(enm);
  const uint32_t ns = __builtin_popcount(s16), ne = __builtin_popcount(e16);
  const uint32_t is = cscan_add(ns), ie = cscan_add(ne);
  const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)is, 63), E = (uint32_t)__builtin_amdgcn_readlane((int)ie, 63);
  const int lane = threadIdx.x & 63;
  const uint64_t q0 = q - 16ull * (uint32_t)lane + (uint64_t)o.delta;  // the chunk's reported base
  pd.R = pd.E = 0;
  if (R == 0 && E == 0) return;
  if (R <= kStage && E <= kStage) {
    uint16_t* S = slot;
    uint16_t* En = slot + kStage;
    const uint32_t lb = 16u * (uint32_t)lane;
    uint32_t m = s16, k = is - ns;
    while (m) {
      S[k++] = (uint16_t)(lb + __builtin_ctz(m));
      m &= m - 1;
    }
    m = e16;
    k = ie - ne;
    while (m) {
      En[k++] = (uint16_t)(lb + __builtin_ctz(m));
      m &= m - 1;
    }
    pd.q0 = q0;
    pd.cur = o.cur;
    pd.open = o.open;
    pd.open_start = o.open_start;
    pd.R = R;
    pd.E = E;
    // the match open after the chunk: the last start, when it has no end
    const uint32_t open = o.open + R - E;
    if (open && R) {
      const int lh = 63 - __builtin_clzll(__ballot(s16 != 0));
      const uint32_t last = lb + 31u - (uint32_t)__builtin_clz(s16 | 1u);  // (read in lane lh)
      o.open_start = q0 + (uint32_t)__builtin_amdgcn_readlane((int)last, lh);
    }
    o.open = open;
    o.cur += R;
    return;
  }
  // the per-lane path: each lane writes its own records; an end closes the
  // latest start before it -- in the lane, in an earlier lane (a wave max-scan
  // of the lanes' last start offsets), or the match open at the chunk start
  const uint32_t top = s16 ? 31u - __builtin_clz(s16) : 0u;
  uint32_t v = ns ? 16u * (uint32_t)lane + top + 1u : 0u;  // (offset + 1 of the lane's last start)
#pragma unroll
  for (int sft = 1; sft < 64; sft <<= 1) {
    const uint32_t y = __shfl_up(v, sft, 64);
    if (lane >= sft && y > v) v = y;
  }
  uint32_t before = __shfl_up(v, 1, 64);
  if (lane == 0) before = 0;
  uint64_t cur = o.cur + (is - ns);
  uint64_t last = before ? q0 + (before - 1) : o.open_start;  // start of the match open at the lane start
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t en = enm[d], st = sb[d];
    uint32_t mm = en | st;
    while (mm) {
      const uint32_t j = (uint32_t)__builtin_ctz(mm) >> 3, bit = 1u << (8 * j);
      const uint64_t pos = q + 4 * d + j + (uint64_t)o.delta;
      if (en & bit) {
        if (cur - 1 < o.capacity) {
          if (last == ~0ull) {
            o.len[cur - 1] = (uint32_t)pos;  // (raw: xc_fix_kernel subtracts the start)
            o.fix = cur - 1;
          } else {
            o.len[cur - 1] = (uint32_t)(pos - last);
          }
        } else {
          o.over = 1;
        }
      }
      if (st & bit) {
        if (cur < o.capacity) {
          o.start[cur] = pos;
          if (o.cap) o.cap[cur] = o.cap1;
        } else {
          o.over = 1;
        }
        last = pos;
        ++cur;
      }
      mm &= ~bit;
    }
  }
  // (at most one match per wave has an unknown start: the lane that closed it
  // holds its index)
  const uint64_t fl = __ballot(o.fix != ~0ull);
  if (fl) {
    const int l = __builtin_ctzll(fl);
    o.fix = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(o.fix >> 32), l) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)o.fix, l);
  }
  const uint32_t open = o.open + R - E;
  if (open && R) {
    const uint32_t vv = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);  // the chunk's last start offset + 1
    o.open_start = q0 + (vv - 1);
  }
  o.open = open;
  o.cur += R;
}

// The stores of a staged chunk (cwrite); the caller has synchronised the
// wave after staging and does again before the slot is staged anew.
template <uint32_t kStage>
__device__ __forceinline__ void cflush(const CPend& p, const uint16_t* slot, COut& o)
{
  if (p.R == 0 && p.E == 0) return;
  const uint16_t* S = slot;
  const uint16_t* En = slot + kStage;
  const uint32_t lane = threadIdx.x & 63;
  if (p.cur + p.R <= o.capacity && p.E <= p.cur + p.R) {
    // (all in range: wave-uniform bases, 32-bit lane offsets, no checks)
    uint64_t* const st = o.start + p.cur;
    uint32_t* const ln = o.len + (p.cur - p.open);
    for (uint32_t t = lane; t < p.R; t += 64) st[t] = p.q0 + S[t];
    if (o.cap)  // (NULL: 12-byte records)
      for (uint32_t t = lane; t < p.R; t += 64) o.cap[p.cur + t] = o.cap1;
    uint32_t t = lane;
    if (p.open && t == 0 && t < p.E) {  // the end of the match open at the chunk start
      const uint64_t e = p.q0 + En[0];
      if (p.open_start == ~0ull) {
        ln[0] = (uint32_t)e;  // (raw: xc_fix_kernel subtracts the start)
        o.fix = p.cur - 1;
      } else {
        ln[0] = (uint32_t)(e - p.open_start);
      }
      t += 64;
    }
    for (; t < p.E; t += 64) ln[t] = (uint32_t)En[t] - (uint32_t)S[t - p.open];
  } else {
    for (uint32_t t = lane; t < p.R; t += 64) {
      const uint64_t i = p.cur + t;
      if (i < o.capacity) {
        o.start[i] = p.q0 + S[t];
        if (o.cap) o.cap[i] = o.cap1;
      } else {
        o.over = 1;
      }
    }
    for (uint32_t t = lane; t < p.E; t += 64) {
      const uint64_t i = p.cur + t - p.open;  // the match this end closes
      const uint64_t e = p.q0 + En[t];
      if (i < o.capacity) {
        if (t < p.open) {
          if (p.open_start == ~0ull) {
            o.len[i] = (uint32_t)e;  // (raw: xc_fix_kernel subtracts the start)
            o.fix = i;
          } else {
            o.len[i] = (uint32_t)(e - p.open_start);
          }
        } else {
          o.len[i] = (uint32_t)(e - (p.q0 + S[t - p.open]));
        }
      } else {
        o.over = 1;
      }
    }
  }
  if (p.open && p.E) {
    const uint64_t fl = __ballot(o.fix != ~0ull);  // (only lane 0 can close the open match, t = 0)
    if (fl) {
      const int l = __builtin_ctzll(fl);
      o.fix = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(o.fix >> 32), l) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)o.fix, l);
    }
  }
}

// cwrite with its stores at once (the masked chunks), in slot 0
template <uint32_t kStage>
__device__ __forceinline__ void cwrite_now(const CLane& L, const uint32_t cb[4], const uint32_t sb[4], uint64_t q,
                                           COut& o)
{
  CPend p;
  cwrite<kStage>(L, cb, sb, q, o, p, o.stage);
  if (p.R == 0 && p.E == 0) return;
  cwave_sync();
  cflush<kStage>(p, o.stage, o);
  cwave_sync();
}

// One chunk (16 bytes per lane at q = chunk base + 16 lane); cw = the wave's
// carry, updated.  Returns the lane's carry-in bits.
template <bool MASK, bool W, bool WR = false, bool U = false, bool BM = false>
__device__ __forceinline__ void cchunk(const CCodes& cc, const uint4& v, uint64_t q, const CLim& lim, uint32_t& cw,
                                       uint32_t& cs, uint32_t& ws, uint32_t& ls, uint32_t cb[4], CW& wc, COut& o,
                                       CU& u, CPend* pd = nullptr, uint16_t* slot = nullptr, uint16_t* ib = nullptr,
                                       uint16_t* ibl = nullptr)
{
#if defined(UGPU_XC_ABL) && UGPU_XC_ABL == 1  // loads only (benchmarking; wrong counts)
  if (!MASK) {
    cs += v.x ^ v.y ^ v.z ^ v.w;
    return;
  }
#endif
  CLane L;
  if constexpr (U)
    ucodes<MASK, W>(u, v, L, q, lim);  // (U mode: W is the UW edge check)
  else
    ccodes<MASK, W>(cc, v, L, q, lim, wc);
  bool prop;
  const bool gen = cadd(L, prop);
  const uint64_t cin = clook(__ballot(gen), __ballot(prop), cw, cw);
  uint32_t sb[4];
  cfinish(L, __builtin_amdgcn_inverse_ballot_w64(cin) ? 1u : 0u, cs, ws, ls, cb, sb);
  if constexpr (W && !U) {
    if (wc.sub) {
#pragma unroll
      for (int d = 0; d < 4; ++d) wc.inv |= cb[d] & (L.E[d] >> 1) & ~(L.E[d] >> 7);  // In_{i-1} and code 0x02
    }
  }
  if constexpr (BM) {
    if constexpr (U) {
      uint32_t in[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) in[d] = (L.E[d] | ((L.E[d] >> 1) & cb[d])) & kOnes;  // In_i = G_i | X_i & In_{i-1}
      if (ibl)
        ibl[(q >> 4) & 63] = (uint16_t)nib16(in);
      else
        ib[q >> 4] = (uint16_t)nib16(in);
    } else {
      // the carry-in bits C_i = In_{i-1}, which cfinish has anyway (the adder
      // codes die here: fewer live registers than In_i); xc_expand_kernel
      // shifts them
#if defined(UGPU_XBM_ABL) && UGPU_XBM_ABL == 1  // bits stored into 32 KiB (benchmarking; wrong records)
      ib[(q >> 4) & 0x3fff] = (uint16_t)nib16(cb);
#elif defined(UGPU_XBM_ABL) && UGPU_XBM_ABL == 2  // bits not stored (benchmarking; wrong records)
      cs += nib16(cb) == 0x12345u;
#else
      if (ibl)
        ibl[(q >> 4) & 63] = (uint16_t)nib16(cb);  // (the tile's bits leave by wide stores)
      else
        ib[q >> 4] = (uint16_t)nib16(cb);
#endif
    }
  }
  if constexpr (WR) {
    if (pd)
      cwrite<U ? kStageU : kStage>(L, cb, sb, q, o, *pd, slot);  // (stores by the caller's cflush)
    else
      cwrite_now<U ? kStageU : kStage>(L, cb, sb, q, o);
  }
}

// U mode, COUNT, a chunk wholly inside [wlo, hi): no byte only continues a
// match, so In = M and no carry chain is needed: starts M & !M_prev, In bytes
// counted directly (ls counts In_i here, not In_{i-1}; the caller corrects the
// difference at the main loop's ends).  mprev (uniform): M of the 4 bytes
// before the chunk (bit 24: the byte just before).
template <bool UW, bool FAST, bool BM = false>
__device__ __forceinline__ void uchunk_direct(CU& u, const uint4& v, uint64_t q, uint32_t& mprev, uint32_t& cs,
                                              uint32_t& ws, uint32_t& ls, uint16_t* ib = nullptr,
                                              uint16_t* ibl = nullptr, CIt* acc = nullptr)
{
#if defined(UGPU_XU_ABL) && UGPU_XU_ABL == 3  // loads only (benchmarking; wrong counts)
  cs += v.x ^ v.y ^ v.z ^ v.w;
  return;
#endif
  uint32_t m[4];
  umask<false, FAST ? 1 : 2>(u, v, q, m);
  const uint32_t mp = __builtin_amdgcn_update_dpp(mprev, m[3], 0x138, 0xf, 0xf, false);  // wave_shr:1
  mprev = __builtin_amdgcn_readlane(m[3], 63);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if (kXuCnt && acc) {
    uint32_t st[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t pm = __builtin_amdgcn_alignbit(m[d], d ? m[d - 1] : mp, 24);  // M of the byte before
      st[d] = m[d] & ~pm;
      if constexpr (UW) u.risk |= ustray(w[d], m[d], pm);
      acc->sacc[d] += st[d];
    }
    cs = __builtin_amdgcn_udot4((st[0] + st[1]) + (st[2] + st[3]), kOnes, cs, false);
    acc->macc += (m[0] + m[1]) + (m[2] + m[3]);
    if constexpr (BM) {
      if (ibl)
        ibl[(q >> 4) & 63] = (uint16_t)nib16(m);
      else
        ib[q >> 4] = (uint16_t)nib16(m);
    }
    return;
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t pm = __builtin_amdgcn_alignbit(m[d], d ? m[d - 1] : mp, 24);  // M of the byte before
    const uint32_t st = m[d] & ~pm;
    if constexpr (UW) u.risk |= ustray(w[d], m[d], pm);
    cs = __builtin_popcount(st) + cs;
    ls = __builtin_popcount(m[d]) + ls;
    const uint32_t wd = (4u * d) | ((4u * d + 1) << 8) | ((4u * d + 2) << 16) | ((4u * d + 3) << 24);
    ws = __builtin_amdgcn_udot4(st, wd, ws, false);
  }
  if constexpr (BM) {
    if (ibl)
      ibl[(q >> 4) & 63] = (uint16_t)nib16(m);  // (In = M here; the tile's bits leave by wide stores)
    else
      ib[q >> 4] = (uint16_t)nib16(m);
  }
}

// U mode, OFFSETS (WRITE), a chunk wholly inside [wlo, hi): In = M here too,
// so the chunk's records come straight from M -- starts M & !M_prev, ends
// M_prev & !M -- with no carry chain, in cwrite's form (the adder codes
// e = 0xFF * M, the carry-in bits M_prev).  FAST as uchunk_direct: the COUNT
// pass of the same range ran the same test and met no XU_MIX / XU_SLOW lead.
template <bool FAST>
__device__ __forceinline__ void uchunk_write(CU& u, const uint4& v, uint64_t q, uint32_t& mprev, COut& o, CPend& pd,
                                             uint16_t* slot)
{
  uint32_t m[4];
  umask<false, FAST ? 1 : 2>(u, v, q, m);
  const uint32_t mp = __builtin_amdgcn_update_dpp(mprev, m[3], 0x138, 0xf, 0xf, false);  // wave_shr:1
  mprev = __builtin_amdgcn_readlane(m[3], 63);
  CLane L;
  uint32_t cb[4], sb[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t pm = __builtin_amdgcn_alignbit(m[d], d ? m[d - 1] : mp, 24);  // M of the byte before
    cb[d] = pm;
    sb[d] = m[d] & ~pm;
    L.E[d] = (m[d] << 8) - m[d];
  }
  cwrite<kStageU>(L, cb, sb, q, o, pd, slot);
}

// Exit search after a masked chunk of the wave holding hi: the exit is the
// first q >= hi with In_q clear (no match starts past hi, so q is the end of
// the match crossing hi, or hi), i.e. the first p = q + 1 > hi whose carry-in
// bit is clear; ~0 when there is none in this chunk.  Also flags a match that
// reaches the readable end rend (when not at EOF).
__device__ __forceinline__ uint64_t cexit(const uint32_t cb[4], uint64_t q, uint64_t hi, uint64_t rend, bool at_eof,
                                          uint32_t& ovf)
{
  uint32_t first = 64;  // byte index in the lane's 16 bytes
#pragma unroll
  for (int d = 3; d >= 0; --d) {
    const uint64_t qd = q + 4 * d;
    const uint32_t z = ~cb[d] & ~below(qd, hi + 1) & kOnes;  // clear carry-in at a position > hi
    if (z) first = 4 * d + (__builtin_ctz(z) >> 3);
    if (!at_eof && rend >= qd && rend < qd + 4 && ((cb[d] >> (8 * (rend - qd))) & 1u)) ovf = 1;
  }
  const uint64_t m = __ballot(first < 64);
  if (!m) return ~0ull;
  const int l = __builtin_ctzll(m);
  const uint32_t f = (uint32_t)__shfl((int)first, l, 64);
  const uint64_t x = q - 16ull * (threadIdx.x & 63) + 16ull * l + f - 1;
  return x < rend ? x : rend;
}

// f(integral_constant<J>) for J = I .. N-1 (compile-time chunk indices)
template <int I, int N, class F>
__device__ __forceinline__ void cunroll(F& f)
{
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    cunroll<I + 1, N>(f);
  }
}

// code of a byte class (xc_cls: G << 7 | X << 6)
__device__ __forceinline__ uint32_t ccode(uint32_t cls) { return cls & 0x80u ? 0xffu : (cls & 0x40u ? 0xfeu : 0u); }

}  // namespace

// (the body of the kernels below)
template <bool W, bool WR, bool U, bool FAST = false, bool BM = false>
__device__ __forceinline__ void xc_body(const ScanParams& P)
{
  constexpr int kIt = U ? kUIter : kCIter;  // chunks per iteration
  constexpr uint32_t kTile = kCChunk * kIt;
  // LDS: byte codes, and (pair classifier) the codes of every byte pair; U
  // mode: the token codes and 3-byte completion bits
  __shared__ __attribute__((aligned(16))) uint8_t bcode[256];
  __shared__ __attribute__((aligned(16))) uint16_t pcode[(kCPair && !U) ? 65536 : 8];
  __shared__ __attribute__((aligned(16))) uint32_t utab[U ? 65536 / 4 : 1];
  __shared__ __attribute__((aligned(16))) uint32_t ubm3[U ? kXuBm3 : 1];
  constexpr uint32_t kStg = U ? kStageU : kStage;
  __shared__ __attribute__((aligned(16))) uint16_t wstage[WR ? kCWaves * 2 * 2 * kStg : 2];
  // BM: a tile's In bits (64 lanes x 16 bits per chunk), gathered so that they
  // leave as one store of kIt * 2 bytes per lane instead of a 2-byte store per
  // lane and chunk (those ran at a fraction of the HBM write rate)
  __shared__ __attribute__((aligned(16))) uint16_t bmst[BM ? kCWaves * 64 * kIt : 1];
  CU u;
  if constexpr (U) {
    // the pair table: entry (x, y) at x << 8 | (y ^ xu_swz(x))
    for (uint32_t i = threadIdx.x; i < 65536 / 4; i += kCWaves * 64) {
      uint32_t w = 0;
      for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t a = 4 * i + b, x = a >> 8, y = (a & 0xffu) ^ xu_swz(x);
        uint32_t e = x < 0x80   ? P.xu_tab[x]
                     : x < 0xc0 ? P.xu_tab[kXuCls + y]
                                : P.xu_tab[256 + (x & 63) * 256 + y];
        if (e == XU_MIX) e = kUMix;
        w |= e << (8 * b);
      }
      utab[i] = w;
    }
    for (uint32_t i = threadIdx.x; i < kXuBm3; i += kCWaves * 64) ubm3[i] = P.xu_bm3[i];
    __syncthreads();
    u.tab = reinterpret_cast<const uint8_t*>(utab);
    u.bm3 = ubm3;
    u.null4 = P.xu_null * 0x01010101u;
    u.vk();
    u.lo = P.lo;
    u.rend = P.rend;
  } else {
    for (uint32_t i = threadIdx.x; i < 256; i += kCWaves * 64) {
      const uint32_t cls = P.xc_cls[i];
      // (subset mode: the ASCII word bytes outside X, code 0x02; see CW)
      bcode[i] = (uint8_t)(ccode(cls) | (P.xc_w == 2 && !(cls & 0xc0u) && (cls & 0x20u) ? 0x02u : 0u));
    }
    __syncthreads();
  }
  if constexpr (kCPair && !U) {
    // pcode[b1 << 8 | b0] = code(b0) | code(b1) << 8, two entries (b0, b0 + 1) per store
    for (uint32_t i = threadIdx.x; i < 65536u / 2; i += kCWaves * 64) {
      const uint32_t b1 = i >> 7, b0 = (2 * i) & 0xffu;
      const uint32_t hi = (uint32_t)bcode[b1] << 8;
      reinterpret_cast<uint32_t*>(pcode)[i] = (hi | bcode[b0]) | ((hi | bcode[b0 + 1]) << 16);
    }
    __syncthreads();
  }
  const CCodes cc{pcode, bcode};
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kCWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kTile, P.lo, P.hi);
  const uint32_t n = (uint32_t)(te - tb);
  const bool last_wave = n && whi == P.hi;
  const uint64_t rend16 = (P.rend + 15) & ~uint64_t(15);
  const uint32_t lo16 = 16u * (uint32_t)lane;
  CW wc;
  wc.bob = P.bob;
  wc.sub = P.xc_w == 2 ? 1u : 0u;
  COut out;
  if constexpr (WR) {
    out.cur = n ? P.out_base[gw] : 0;
    out.start = P.out_start;
    out.len = P.out_len;
    out.cap = P.out_cap;
    out.capacity = P.out_capacity;
    out.delta = P.delta;
    out.cap1 = P.cap1;
    out.stage = wstage + (uint32_t)wid * 4u * kStg;
  }
  // option W: the code of the byte before position p (byte 3), 0 at the buffer start
  auto xprev = [&](uint64_t p) -> uint32_t { return W && !U && p > P.bob ? (uint32_t)bcode[P.g[p - 1]] << 24 : 0u; };

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
      if constexpr (U) {
        u.nx0 = uload_dw(u, P.g, cb0 + kCChunk);
        u.cprev = ucode_before(u, P.g, cb0);
        ucodes<true>(u, v, L, cb0 + lo16, lim);
      } else {
        ccodes<true, W>(cc, v, L, cb0 + lo16, lim, wc);
      }
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
  if constexpr (WR) out.open = cw;  // a match opened by the previous wave (its start is unknown here)

  uint64_t cnt = 0, pos = 0, lbits = 0;  // lane sums (absolute start positions)
  uint64_t exit = whi;
  uint32_t ovf = 0;
  bool found = false;
  const CLim lim{wlo, P.hi, P.rend};

  // Full tiles [ftb, fte) run the unmasked main loop; the chunks before them
  // (the first wave, lo not tile aligned) and after them (the wave holding hi,
  // then on past hi until the exit) run one masked chunk at a time, outside
  // the main loop's register budget.
  uint64_t ftb = (wlo + kTile - 1) / kTile, fte = whi / kTile;
  if (!n || ftb >= fte) ftb = fte = 0;
  // one masked chunk at q0 (exit search on chunks reaching past hi)
  auto masked = [&](uint64_t q0) __attribute__((always_inline)) {
    const uint4 v = cload(crsrc(P.g + q0, rend16 > q0 ? rend16 - q0 : 0), lo16);
    uint32_t cs = 0, ws = 0, ls = 0, cb[4];
    if constexpr (U) u.nx0 = uload_dw(u, P.g, q0 + kCChunk);
    cchunk<true, W, WR, U, BM>(cc, v, q0 + lo16, lim, cw, cs, ws, ls, cb, wc, out, u, nullptr, nullptr, P.inbits);
    cnt += cs;
    pos += (uint64_t)cs * (q0 + lo16) + ws;
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
  wc.cx = xprev(q0);
  if constexpr (U) u.cprev = ucode_before(u, P.g, q0);
  wc.hi = 0;
  // option W: at_wb at the range start decodes the character before it; when
  // lo is chunk aligned no chunk holds that byte, so it is seen here (>= 0x80:
  // the host redoes the range with wfind_kernel)
  if constexpr (W && !U) {
    if (n && wlo == P.lo && P.lo > P.bob) wc.hi |= (uint32_t)P.g[P.lo - 1];
  }
  if (fte > ftb)
    for (; q0 < ftb * kTile; q0 += kCChunk) masked(q0);

  // U mode: M of the byte before the chunk (uniform)
  uint32_t mprev = 0;
  const uint32_t cw_main = cw;
  {
    uint4 cur[kIt], nxt[kIt];
    // U mode: the first dword of the tile after the current one (the last
    // chunk's context), loaded one tile ahead
    uint32_t nfc = 0, nfn = 0;
    if (fte > ftb) {
      const uint64_t ts = ftb * kTile;
      const __amdgpu_buffer_rsrc_t rs = crsrc(P.g + ts, rend16 > ts ? rend16 - ts : 0);
#pragma unroll
      for (int j = 0; j < kIt; ++j) cur[j] = cload(rs, j * kCChunk + lo16);
      if constexpr (U) nfc = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)kTile, 0, 0);
      mprev = cw << 24;
    }
    CPend pend[2];  // (WR: the staged chunks of the tile)
    // one tile of the main loop; c = its starts, cj = their chunk-weighted
    // count, ws = in-chunk start offsets, ls = In bits (lane sums)
    auto tile_step = [&](uint64_t t, uint32_t& c, uint32_t& cj, uint32_t& tws, uint32_t& tls)
                         __attribute__((always_inline)) {
      const uint64_t ts = t * kTile;
      {
        // (U mode reads the next tile also after the last: its first dword is
        // the last chunk's context)
        const uint64_t tn = (U || t + 1 < fte) ? ts + kTile : ts;
        const __amdgpu_buffer_rsrc_t rn = crsrc(P.g + tn, rend16 > tn ? rend16 - tn : 0);
#pragma unroll
        for (int j = 0; j < kIt; ++j) {
#if defined(UGPU_XU_ABL) && UGPU_XU_ABL == 4  // compute only: no HBM reads in the main loop (benchmarking; wrong counts)
          nxt[j] = uint4{cur[j].y, cur[j].z, cur[j].w, cur[j].x ^ (uint32_t)t};
#else
          nxt[j] = cload(rn, j * kCChunk + lo16);
#endif
        }
        if constexpr (U) nfn = __builtin_amdgcn_raw_buffer_load_b32(rn, (int)kTile, 0, 0);
      }
      CIt a;
      uint32_t cb[4];
      // (chunk indices are compile-time constants, so cur[] and nxt[] stay in
      // registers also when the body is too large for the loop unroller)
      auto chunk = [&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        if constexpr (U) {
          // the dword after the chunk (its last lane's context)
          if constexpr (j + 1 < kIt) {
            u.nx0 = __builtin_amdgcn_readlane(cur[j + 1].x, 0);
          } else {
            const uint32_t in = uinside(u, ts + kTile);
            u.nx0 = (__builtin_amdgcn_readfirstlane(nfc) & in) | (u.null4 & ~in);
          }
        }
        uint16_t* const slot = out.stage + (uint32_t)(j & 1) * 2u * kStg;
        uint16_t* const ibl = BM ? bmst + ((uint32_t)wid * kIt + j) * 64u : nullptr;
        if constexpr (U && !WR)
          uchunk_direct<W, FAST, BM>(u, cur[j], ts + j * kCChunk + lo16, mprev, a.cs[j], a.ws, a.ls, P.inbits, ibl,
                                     &a);
        else if constexpr (U && WR)
          uchunk_write<FAST>(u, cur[j], ts + j * kCChunk + lo16, mprev, out, pend[j & 1], slot);
        else if constexpr (WR)
          cchunk<false, W, WR, U>(cc, cur[j], ts + j * kCChunk + lo16, lim, cw, a.cs[j], a.ws, a.ls, cb, wc, out, u,
                                  &pend[j & 1], slot);
        else
          cchunk<false, W, WR, U, BM>(cc, cur[j], ts + j * kCChunk + lo16, lim, cw, a.cs[j], a.ws, a.ls, cb, wc, out,
                                      u, nullptr, nullptr, P.inbits, ibl);
        if constexpr (WR) {
          // the stores of the staged slots: at the tile end after the next
          // tile's loads (cwrite: they then overlap the next tile's work),
          // mid-tile when both slots are full
          if constexpr ((j & 1) == 1 || j + 1 == kIt) {
            if constexpr (j + 1 == kIt) __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
            cwave_sync();
            cflush<kStg>(pend[0], out.stage, out);
            if constexpr ((j & 1) == 1) cflush<kStg>(pend[1], out.stage + 2u * kStg, out);
            cwave_sync();
          }
        }
      };
      cunroll<0, kIt>(chunk);
      if constexpr (BM) {
        // the tile's bits: kIt * 128 contiguous bytes at bit offset ts
        using BmWord = typename std::conditional<kIt == 8, uint4, typename std::conditional<kIt == 4, uint2, uint32_t>::type>::type;
        static_assert(sizeof(BmWord) == 2 * kIt, "one word per lane");
        cwave_sync();
        const BmWord v = reinterpret_cast<const BmWord*>(bmst + (uint32_t)wid * kIt * 64u)[lane];
#if UGPU_XBM_NT
        if constexpr (kIt == 4) {
          __builtin_nontemporal_store(__builtin_bit_cast(uint64_t, v), reinterpret_cast<uint64_t*>(P.inbits + (ts >> 4)) + lane);
        } else if constexpr (kIt == 2) {
          __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(P.inbits + (ts >> 4)) + lane);
        } else {
          reinterpret_cast<BmWord*>(P.inbits + (ts >> 4))[lane] = v;
        }
#else
        reinterpret_cast<BmWord*>(P.inbits + (ts >> 4))[lane] = v;
#endif
        cwave_sync();  // (the next tile's chunks write the slots anew)
      }
      if constexpr (U && !WR && kXuCnt) {
        // (the byte sums of the tile: kIt <= 4 chunks, at most 4 per byte each)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t wd = (4u * d) | ((4u * d + 1) << 8) | ((4u * d + 2) << 16) | ((4u * d + 3) << 24);
          a.ws = __builtin_amdgcn_udot4(a.sacc[d], wd, a.ws, false);
        }
        a.ls = __builtin_amdgcn_udot4(a.macc, kOnes, a.ls, false);
      }
      c = 0;
      cj = 0;
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        c += a.cs[j];
        cj += j * a.cs[j];
      }
      tws = a.ws;
      tls = a.ls;
#pragma unroll
      for (int j = 0; j < kIt; ++j) cur[j] = nxt[j];
      nfc = nfn;
    };
#if UGPU_XC_ACC32
    // the main loop's lane sums in 32 bits, folded into cnt / pos / lbits once
    // after the loop (the 64-bit multiply-adds per tile were ~12 VALU of the
    // loop): c32 = starts, s32 = the running start count summed over the tiles
    // (so sum_k k c_k = nt c32 - s32), l32 = in-tile offsets, b32 = In bits.
    // Per lane and tile at most 16 starts at offsets < kTile, so up to kFold
    // tiles per wave keep s32 < 2^30 and l32 < 2^29; longer wave ranges take
    // the 64-bit loop.
    constexpr uint64_t kFold = 8192;
    if (fte - ftb <= kFold) {
      uint32_t c32 = 0, s32 = 0, l32 = 0, b32 = 0;
      for (uint64_t t = ftb; t < fte; ++t) {
        uint32_t c, cj, tws, tls;
        tile_step(t, c, cj, tws, tls);
        c32 += c;
        s32 += c32;
        l32 += tws + kCChunk * cj;
        b32 += tls;
      }
      cnt += c32;
      pos += (uint64_t)c32 * (ftb * kTile + lo16) + (uint64_t)kTile * ((fte - ftb) * c32 - s32) + l32;
      lbits += b32;
    } else
#endif
    for (uint64_t t = ftb; t < fte; ++t) {
      uint32_t c, cj, tws, tls;
      tile_step(t, c, cj, tws, tls);
      cnt += c;
      pos += (uint64_t)c * (t * kTile + lo16) + tws + kCChunk * cj;
      lbits += tls;
    }
  }
  if (fte > ftb) q0 = fte * kTile;
  if constexpr (U && WR) {
    if (fte > ftb) cw = (mprev >> 24) & 1u;  // (the match open after the main loop)
  }
  if constexpr (U && !WR) {
    if (fte > ftb) {
      // the wave carry after the main loop, and ls's In_i -> In_{i-1} form:
      // sum In_{i-1} over [a, b) = sum In_i + In_{a-1} - In_{b-1}
      cw = (mprev >> 24) & 1u;
      if (lane == 0) lbits += (uint64_t)cw_main - (uint64_t)cw;
    }
  }
  // the rest of the wave's range; the wave holding hi goes on until the exit
  // (the match crossing hi runs on through X bytes, no starts past hi).  Bytes
  // past the readable end are K, so the search ends at the latest in the chunk
  // after the one holding rend (its loads read nothing: the resource is empty).
  if (n)
    for (; q0 < whi || (last_wave && !found); q0 += kCChunk) masked(q0);
  if (found) cw = 0;  // past the exit every carry is clear
  // U mode: the codes of the last 3 bytes before a non-EOF readable end
  // depend on bytes not read yet -- except at an ASCII byte, which lies in no
  // token that starts before it, so an exit there is decided
  if (U && last_wave && !P.at_eof && exit + 3 >= P.rend && !(exit < P.rend && P.g[exit] < 0x80)) ovf = 1;
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if constexpr (U) {
    if (__ballot((u.slow & 0x08080808u) != 0) && lane == 0) atomicOr(P.flags, UGPU_FLAG_USLOW);
  }
  if constexpr (WR) {
    if (__ballot(out.over) && lane == 0) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
    if (lane == 0) P.out_fix[gw] = out.fix;  // (~0: none)
    return;  // (the records are the COUNT pass's)
  }
  if constexpr (W && !U) {
    if (__ballot((wc.hi & 0x80808080u) != 0 || (wc.inv & kOnes) != 0) && lane == 0) atomicOr(P.flags, UGPU_FLAG_WSLOW);
  }
  if constexpr (W && U) {
    if (__ballot((u.risk & kOnes) != 0) && lane == 0) atomicOr(P.flags, UGPU_FLAG_WSLOW);
  }
  if constexpr (U && FAST) {
    if (__ballot((u.x8 & 0x08080808u) != 0) && lane == 0) atomicOr(P.flags, UGPU_FLAG_UMIX);
  }
  const uint64_t c = wave_sum(cnt), s = wave_sum(pos), lb = wave_sum(lbits);
  if (lane == 0) {
    // In bytes = carry-in bits, minus the carry into the first byte, plus the
    // carry out of the last processed byte
    const uint64_t len = n ? lb - cin0 + cw : 0;
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

template <bool W, bool WR, bool U>
__global__ __launch_bounds__(kCWaves * 64) void xc_kernel(ScanParams P)
{
  xc_body<W, WR, U>(P);
}

// U mode OFFSETS: FAST unless the COUNT pass needed the exact kernel
template <bool FAST>
__global__ __launch_bounds__(kCWaves * 64) void xu_write_kernel(ScanParams P)
{
  xc_body<false, true, true, FAST>(P);
}

// U mode COUNT: LDS-latency bound (its byte lookups), so two workgroups per CU
// (8 waves per SIMD, at most 64 VGPRs; the tables take 72 KiB per workgroup)
#ifndef UGPU_XU_WAVES_PER_EU
#define UGPU_XU_WAVES_PER_EU 8
#endif
// (option W: its checks keep more state live; UGPU_XU_W_WAVES_PER_EU)
#ifndef UGPU_XU_W_WAVES_PER_EU
#define UGPU_XU_W_WAVES_PER_EU UGPU_XU_WAVES_PER_EU
#endif
template <bool UW, bool FAST>
__global__ __launch_bounds__(kCWaves * 64) __attribute__((amdgpu_waves_per_eu(UW ? UGPU_XU_W_WAVES_PER_EU
                                                                                  : UGPU_XU_WAVES_PER_EU)))
void xu_kernel(ScanParams P)
{
  xc_body<UW, false, true, FAST>(P);
}

// COUNT passes that also write the In bits (P.inbits; no option W)
template <bool FAST>
__global__ __launch_bounds__(kCWaves * 64) __attribute__((amdgpu_waves_per_eu(UGPU_XU_WAVES_PER_EU)))
void xu_bm_kernel(ScanParams P)
{
  xc_body<false, false, true, FAST, true>(P);
}
__global__ __launch_bounds__(kCWaves * 64) void xc_bm_kernel(ScanParams P)
{
  xc_body<false, false, false, false, true>(P);
}

// OFFSETS from the In bits of the COUNT pass.  In is the FIND chain's
// "inside a match" bit per byte, so the matches are its runs: a start where
// In rises, an end where it falls, and the k-th end of the chain closes the
// k-th start.  Block b writes the records of COUNT wave b: the starts in its
// range [wlo, whi) (the last wave's ends run on to the chain exit) at indices
// from that wave's output base, and the ends in the range, which close the
// match open at wlo first (index base - 1; its start was written by an
// earlier block: the raw end goes into len and out_fix names the index for
// xc_fix_kernel, as in the WRITE pass).  64-bit words of In bits, 64 a
// wave-round; the round's starts and ends are ordered by DPP scans and staged
// in LDS (u16 offsets from the round's first position), then stored by
// consecutive lanes -- starts, caps (none for 12-byte records) and lengths
// (the k-th end of the round closes the k-th start, or the match open at
// the round start) all leave as coalesced stores.  No table, no walk: the pass
// reads 1/8 of the input's bytes and writes the records.
#ifndef UGPU_XE_CAP
#define UGPU_XE_CAP 1024
#endif
// non-temporal record stores: 1 starts, 2 lengths, 3 both.  Starts only is
// the default: C4 OFFSETS 5.03 / 5.82 against 5.49 / 6.11 ms per step, C3
// 9.05 against 9.33 (two runs on one box); lengths too was slower on C3
// (profiles/r05_offsets_ab.json)
#ifndef UGPU_XE_NT
#define UGPU_XE_NT 1
#endif

// a word load the compiler does not track (no s_waitcnt of its own); the
// caller waits with xe_wait, whose count N must be at most the number of
// vector-memory instructions issued after the load
__device__ __forceinline__ uint64_t xe_load(const uint64_t* p)
{
  uint64_t v;
#if UGPU_XE_LNT
  asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
#else
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
#endif
  return v;
}
template <int N>
__device__ __forceinline__ void xe_wait(uint64_t& a, uint64_t& b)
{
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
// a lane's events (bits of m, positions lb + bit) staged at k0 .. k1 - 1 of
// o in position order
__device__ __forceinline__ void xe_stage(uint16_t* o, uint32_t k0, uint32_t k1, uint32_t lb, uint64_t m)
{
  // (32-bit halves side by side, each from both ends: a step writes up to 4
  // events, with 32-bit bit scans)
  uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
  uint32_t a0 = k0, a1 = k0 + (uint32_t)__builtin_popcount(lo), b0 = a1, b1 = k1;
  while (lo | hi) {
    if (lo) {
      const uint32_t f = (uint32_t)__builtin_ctz(lo), g = 31u - (uint32_t)__builtin_clz(lo);
      o[a0++] = (uint16_t)(lb + f);
      o[--a1] = (uint16_t)(lb + g);  // (f == g: the same slot, the same value)
      lo &= lo - 1;
      lo &= ~(1u << g);
    }
    if (hi) {
      const uint32_t f = (uint32_t)__builtin_ctz(hi), g = 31u - (uint32_t)__builtin_clz(hi);
      o[b0++] = (uint16_t)(lb + 32u + f);
      o[--b1] = (uint16_t)(lb + 32u + g);
      hi &= hi - 1;
      hi &= ~(1u << g);
    }
  }
}
// the same with N the largest of 48, 32, 24, 16, 12, 8, 4, 0 not above k (uniform): one
// asm statement, so that a and b are never read (copied) before the wait
__device__ __forceinline__ void xe_wait_k(uint64_t& a, uint64_t& b, uint32_t k)
{
  asm volatile(
      "s_cmp_lt_u32 %2, 48\n\t"
      "s_cbranch_scc1 1f\n\t"
      "s_waitcnt vmcnt(48)\n\t"
      "s_branch 9f\n"
      "1:\n\t"
      "s_cmp_lt_u32 %2, 32\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_waitcnt vmcnt(32)\n\t"
      "s_branch 9f\n"
      "2:\n\t"
      "s_cmp_lt_u32 %2, 24\n\t"
      "s_cbranch_scc1 3f\n\t"
      "s_waitcnt vmcnt(24)\n\t"
      "s_branch 9f\n"
      "3:\n\t"
      "s_cmp_lt_u32 %2, 16\n\t"
      "s_cbranch_scc1 4f\n\t"
      "s_waitcnt vmcnt(16)\n\t"
      "s_branch 9f\n"
      "4:\n\t"
      "s_cmp_lt_u32 %2, 12\n\t"
      "s_cbranch_scc1 5f\n\t"
      "s_waitcnt vmcnt(12)\n\t"
      "s_branch 9f\n"
      "5:\n\t"
      "s_cmp_lt_u32 %2, 8\n\t"
      "s_cbranch_scc1 6f\n\t"
      "s_waitcnt vmcnt(8)\n\t"
      "s_branch 9f\n"
      "6:\n\t"
      "s_cmp_lt_u32 %2, 4\n\t"
      "s_cbranch_scc1 7f\n\t"
      "s_waitcnt vmcnt(4)\n\t"
      "s_branch 9f\n"
      "7:\n\t"
      "s_waitcnt vmcnt(0)\n"
      "9:"
      : "+v"(a), "+v"(b)
      : "s"(__builtin_amdgcn_readfirstlane(k))
      : "memory", "scc");
}

// NW = 4: the range is cut into 4 quarters of whole words, one per wave.  A
// first pass counts each quarter's starts and ends and finds its last start;
// after one block barrier every wave knows its output bases and writes its
// quarter alone.  NW = 1: one wave takes the COUNT wave's whole range, its
// output base is the COUNT pass's, and there is no first pass (the bitmap is
// read once, and no block barrier separates the passes) -- with one block per
// COUNT wave (8192) the chip still holds 32 of these waves per CU.
constexpr uint32_t kXeWaveCap = UGPU_XE_CAP;  // starts (and ends) a wave-round stages at once (2 KiB each)

template <bool U, int NW>
#ifndef UGPU_XE_WAVES_PER_EU
#define UGPU_XE_WAVES_PER_EU 7
#endif
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(UGPU_XE_WAVES_PER_EU))) void xc_expand_kernel(ScanParams P)
{
  __shared__ uint16_t st_off[NW][kXeWaveCap];  // a round's start positions, from the round's first position
  __shared__ uint16_t en_off[NW][kXeWaveCap];  // its end positions
  __shared__ uint32_t qs[NW], qe[NW];
  __shared__ int64_t ql[NW];
  __shared__ uint64_t fix_s;
  constexpr uint64_t kTile = (uint64_t)kCChunk * (U ? kUIter : kCIter);
  const uint64_t gw = blockIdx.x;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t tb = P.t0 + gw * P.tpb;
  const uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  if (threadIdx.x == 0) fix_s = ~0ull;
  const uint64_t wlo = clampu(tb * kTile, P.lo, P.hi), whi = clampu(te * kTile, P.lo, P.hi);
  const bool any = te > tb;
  const bool last = any && whi == P.hi;
  const uint64_t end = !any ? wlo : last ? P.totals->exit + 1 : whi;  // event positions [wlo, end)
  const uint64_t* words = reinterpret_cast<const uint64_t*>(P.inbits);
  // the events of word wi (positions [wlo, end) only).  U: the bits are In_i;
  // two-state tables: C_i = In_{i-1} (cchunk), so In_i is bit i + 1
  // (loads and arithmetic apart: the passes issue the loads of several words,
  // or of the next round, before they use any -- the pass is latency-bound)
  struct Raw {
    uint64_t a = 0, b = 0;  // word wi, and its neighbour (U: wi - 1, else wi + 1)
  };
  auto load_raw = [&](uint64_t wi) __attribute__((always_inline)) {
    Raw r;
    const uint64_t pos = wi * 64;
    if (pos >= end || pos + 64 <= wlo) return r;
    r.a = words[wi];
    if constexpr (U) {
      if (pos > P.lo) r.b = words[wi - 1];
    } else {
      // (C_{pos + 64}: the next wave's first bit at whi; for the wave holding
      // hi, In is 0 from position end - 1 -- the exit -- on)
      if (last ? pos + 64 < end : pos + 64 <= end) r.b = words[wi + 1];
    }
    return r;
  };
  auto events = [&](uint64_t wi, const Raw& r, uint64_t& st, uint64_t& en) __attribute__((always_inline)) {
    const uint64_t pos = wi * 64;
    st = en = 0;
    if (pos >= end || pos + 64 <= wlo) return;
    uint64_t w, prev;
    if constexpr (U) {
      w = r.a;
      prev = (w << 1) | (r.b >> 63);
    } else {
      prev = r.a;
      w = (prev >> 1) | (r.b << 63);
      if (last) {
        const uint64_t zi = end - 1 - pos;
        if (zi < 64) w &= (1ull << zi) - 1ull;
      }
    }
    const uint64_t a = wlo > pos ? wlo - pos : 0, z = end - pos;
    const uint64_t lim = (~0ull << a) & (z >= 64 ? ~0ull : ((1ull << z) - 1ull));
    st = w & ~prev & lim;
    en = prev & ~w & lim;
  };
  const uint64_t wb = wlo >> 6, we = end > wlo ? (end + 63) >> 6 : wb;  // words [wb, we)
  const uint64_t nq = (we - wb + NW - 1) / NW;
  const uint64_t qb = wb + wv * nq, qend = qb + nq < we ? qb + nq : we;  // this wave's words
  // pass 1: the quarter's counts and last start
  if constexpr (NW > 1) {
    uint32_t ns = 0, ne = 0;
    int64_t ls = -1;
    for (uint64_t wi0 = qb + lane; wi0 < qend; wi0 += 256) {
      Raw r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (wi0 + 64 * k < qend) r[k] = load_raw(wi0 + 64 * k);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t wi = wi0 + 64 * k;
        if (wi >= qend) break;
        uint64_t st, en;
        events(wi, r[k], st, en);
        ns += (uint32_t)__builtin_popcountll(st);
        ne += (uint32_t)__builtin_popcountll(en);
        if (st) ls = (int64_t)(wi * 64 + 63 - __builtin_clzll(st));
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      ns += __shfl_xor(ns, d, 64);
      ne += __shfl_xor(ne, d, 64);
      const int64_t o = __shfl_xor(ls, d, 64);
      ls = o > ls ? o : ls;
    }
    if (lane == 0) {
      qs[wv] = ns;
      qe[wv] = ne;
      ql[wv] = ls;
    }
  }
  __syncthreads();
  if (any) {
    const uint64_t base = P.out_base[gw];
    // In_{wlo - 1}: U bit wlo - 1; two-state tables C_wlo
    const uint32_t open0 = wlo <= P.lo ? 0u
                           : U        ? (uint32_t)((words[(wlo - 1) >> 6] >> ((wlo - 1) & 63)) & 1ull)
                                      : (uint32_t)((words[wlo >> 6] >> (wlo & 63)) & 1ull);
    uint64_t s_before = 0, e_before = 0;
    int64_t last_start = -1;  // the last start so far (-1: none since wlo)
    for (uint32_t w = 0; w < wv; ++w) {
      s_before += qs[w];
      e_before += qe[w];
      if (ql[w] >= 0) last_start = ql[w];
    }
    uint16_t* so = st_off[wv];
    uint16_t* eo = en_off[wv];
    const uint64_t cap_n = P.out_capacity;
    // the words of a round (a) and their neighbours (b) come in by loads the
    // compiler does not track (xe_load): its own wait for them would be a
    // vmcnt(0) -- the round's record stores lie between a prefetch and its use
    // -- so every round would wait for its stores and its prefetch.  Here the
    // next round's loads go out before this round's stores and the round ends
    // with a wait that lets up to K of those stores stay in flight (xe_wait).
    const uint64_t wlo6 = P.lo >> 6;
    auto ia = [&](uint64_t wi) __attribute__((always_inline)) { return wi < qend ? wi : qend - 1; };
    auto ib = [&](uint64_t wi) __attribute__((always_inline)) {
      if constexpr (U) {
        const uint64_t v = wi > 0 ? wi - 1 : 0;
        return v > wlo6 ? v : wlo6;
      } else {
        return wi + 1 < (end >> 6) ? wi + 1 : (end >> 6);  // (every word read where b counts; inside the bitmap)
      }
    };
    auto raw = [&](uint64_t wi, uint64_t a, uint64_t b) __attribute__((always_inline)) {
      Raw r;
      const uint64_t pos = wi * 64;
      if (pos >= end || pos + 64 <= wlo) return r;
      r.a = a;
      if constexpr (U)
        r.b = pos > P.lo ? b : 0;
      else
        r.b = (last ? pos + 64 < end : pos + 64 <= end) ? b : 0;
      return r;
    };
    uint64_t A = 0, B = 0;
    if (qb < qend) {
      A = xe_load(words + ia(qb + lane));
      B = xe_load(words + ib(qb + lane));
      xe_wait<0>(A, B);
    }
    for (uint64_t w0 = qb; w0 < qend; w0 += 64) {
      const uint64_t wi = w0 + lane, pos = wi * 64;
      // (U: the neighbour words of the next round are this round's, one lane
      // up -- no second load)
      uint64_t An = xe_load(words + ia(wi + 64)), Bn = 0;
      if constexpr (!U) Bn = xe_load(words + ib(wi + 64));
      uint64_t st = 0, en = 0;
      if (wi < qend) events(wi, raw(wi, A, B), st, en);
      const uint64_t pb = w0 * 64;
      const uint32_t lb = (uint32_t)(pos - pb);
      // a round stages all its starts and ends at once unless one of them
      // exceeds kXeWaveCap; then lanes 0-31 and 32-63 go as two rounds
      // (at most 32 starts per word); K counts the store iterations
      uint32_t K = 0;
      auto part = [&](uint64_t pst, uint64_t pen) __attribute__((always_inline)) {
        const uint32_t ns = (uint32_t)__builtin_popcountll(pst), ne = (uint32_t)__builtin_popcountll(pen);
        const uint32_t is = cscan_add(ns), ie = cscan_add(ne);
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)is, 63);
        const uint32_t E = (uint32_t)__builtin_amdgcn_readlane((int)ie, 63);
        const uint64_t hs = __ballot(pst != 0);
        const int64_t myls = pst ? (int64_t)(pos + 63 - __builtin_clzll(pst)) : -1;
        // (two events per step: the lowest from the front, the highest from the back)
        xe_stage(so, is - ns, is, lb, pst);
        xe_stage(eo, ie - ne, ie, lb, pen);
        cwave_sync();
        // (uniform) a match is open at the round start: its end is the round's first
        const uint32_t open_r = (uint32_t)(open0 + s_before - e_before);
        const uint64_t sb0 = base + s_before, eb0 = base - open0 + e_before;
#if defined(UGPU_XE_ABL) && (UGPU_XE_ABL == 1 || UGPU_XE_ABL == 3)  // no start stores (benchmarking; wrong records)
        if (R == ~0u)
#endif
        if (sb0 + R <= cap_n && !P.out_cap) {
          // (the usual case: 4 staged starts read, then 4 stores)
          const uint64_t sbase = pb + (uint64_t)P.delta;
#if defined(UGPU_XE_ABL) && UGPU_XE_ABL == 4  // records into 3 MiB (L2-resident; benchmarking; wrong records)
          uint64_t* const os = P.out_start + (sb0 & 0x3ffffu);
#else
          uint64_t* const os = P.out_start + sb0;
#endif
          for (uint32_t t0 = 0; t0 < R; t0 += 256) {
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t t = t0 + 64 * j + lane;
              v[j] = t < R ? so[t] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t t = t0 + 64 * j + lane;
#if UGPU_XE_NT & 1
              if (t < R) __builtin_nontemporal_store(sbase + v[j], &os[t]);
#else
              if (t < R) os[t] = sbase + v[j];
#endif
            }
          }
        } else {
          for (uint32_t t = lane; t < R; t += 64) {
            const uint64_t i = sb0 + t;
            if (i < cap_n) {
              P.out_start[i] = pb + so[t] + (uint64_t)P.delta;
              if (P.out_cap) P.out_cap[i] = P.cap1;
            } else {
              atomicOr(P.flags, UGPU_FLAG_CAPACITY);
            }
          }
        }
#if defined(UGPU_XE_ABL) && (UGPU_XE_ABL == 1 || UGPU_XE_ABL == 2)  // no length stores (benchmarking; wrong records)
        if (E == ~0u)
#endif
        uint32_t t1 = 0;  // the ends from t1 on close starts of this round
        if (open_r && E) {
          // (the one end that closes the match open at the round start)
          if (lane == 0) {
            const uint64_t i = eb0;
            if (i >= cap_n) {
              atomicOr(P.flags, UGPU_FLAG_CAPACITY);
            } else if (last_start >= 0) {
              P.out_len[i] = (uint32_t)(pb + eo[0] - (uint64_t)last_start);
            } else {
              P.out_len[i] = (uint32_t)(pb + eo[0] + (uint64_t)P.delta);  // raw (reported): the match open at wlo
              fix_s = i;
            }
          }
          t1 = 1;
        }
        if (eb0 + E <= cap_n) {
#if defined(UGPU_XE_ABL) && UGPU_XE_ABL == 4
          uint32_t* const ol = P.out_len + (eb0 & 0x3ffffu);
#else
          uint32_t* const ol = P.out_len + eb0;
#endif
          for (uint32_t t0 = t1; t0 < E; t0 += 256) {
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t t = t0 + 64 * j + lane;
              v[j] = t < E ? (uint32_t)eo[t] - (uint32_t)so[t - open_r] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t t = t0 + 64 * j + lane;
#if UGPU_XE_NT & 2
              if (t < E) __builtin_nontemporal_store(v[j], &ol[t]);
#else
              if (t < E) ol[t] = v[j];
#endif
            }
          }
        } else {
          for (uint32_t t = t1 + lane; t < E; t += 64) {
            const uint64_t i = eb0 + t;
            if (i >= cap_n)
              atomicOr(P.flags, UGPU_FLAG_CAPACITY);
            else
              P.out_len[i] = (uint32_t)eo[t] - (uint32_t)so[t - open_r];
          }
        }
        s_before += R;
        e_before += E;
        const int64_t rl = __shfl(myls, hs ? 63 - __builtin_clzll(hs) : 0, 64);
        if (hs) last_start = rl;
#if !defined(UGPU_XE_ABL) || UGPU_XE_ABL == 4  // (ablations 1-3 skip stores: K stays 0)
        // (a store instruction goes out for every 64 records: lane 0 takes part
        // in each; the one store of the match open at the round start aside)
        K += (R + 63) / 64 + (E > t1 ? (E - t1 + 63) / 64 : 0);
#endif
      };
      const uint32_t cs = (uint32_t)__builtin_popcountll(st), ce = (uint32_t)__builtin_popcountll(en);
      // (no lane above 16 events of a kind: the round fits; else count exactly)
      bool fits = __ballot(cs > kXeWaveCap / 64 || ce > kXeWaveCap / 64) == 0;
      if (!fits) {
        const uint32_t rs = (uint32_t)__builtin_amdgcn_readlane((int)cscan_add(cs), 63);
        const uint32_t re = (uint32_t)__builtin_amdgcn_readlane((int)cscan_add(ce), 63);
        fits = rs <= kXeWaveCap && re <= kXeWaveCap;
      }
      if (fits) {
        part(st, en);
      } else {
        part(lane < 32 ? st : 0, lane < 32 ? en : 0);
        cwave_sync();  // (the second half stages anew)
        part(lane < 32 ? 0 : st, lane < 32 ? 0 : en);
      }
      xe_wait_k(An, Bn, K);
      if constexpr (U) {
        // b of lane l is word wi - 1: lane l - 1's, and for lane 0 this
        // round's last word
        const uint64_t a63 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(A >> 32), 63) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)A, 63);
        const uint32_t blo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)a63, (int)(uint32_t)An, 0x138, 0xf, 0xf,
                                                                   false);  // wave_shr:1
        const uint32_t bhi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(a63 >> 32), (int)(uint32_t)(An >> 32),
                                                                   0x138, 0xf, 0xf, false);
        B = ((uint64_t)bhi << 32) | blo;
      } else {
        B = Bn;
      }
      A = An;
      cwave_sync();  // (the next round stages anew)
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) P.out_fix[gw] = fix_s;
}

// OFFSETS, second step: the one match per wave whose start an earlier wave
// wrote (fix[w] = its index, ~0 none) holds its end position (low 32 bits,
// reported coordinates) in len: subtract the start
__global__ __launch_bounds__(256) void xc_fix_kernel(const uint64_t* fix, uint32_t nrec, const uint64_t* start,
                                                     uint32_t* len, uint64_t n)
{
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  if (w >= nrec) return;
  const uint64_t k = fix[w];
  if (k < n) len[k] -= (uint32_t)start[k];
}

hipError_t launch_xc(const ScanParams& P, bool write, hipStream_t stream, uint64_t count)
{
  if (write) {
    if (P.xu_tab && !P.xu_exact)
      hipLaunchKernelGGL((xu_write_kernel<true>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    else if (P.xu_tab)
      hipLaunchKernelGGL((xu_write_kernel<false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    else if (P.xc_w)
      hipLaunchKernelGGL((xc_kernel<true, true, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    else
      hipLaunchKernelGGL((xc_kernel<false, true, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t n = count < P.out_capacity ? count : P.out_capacity;
    const uint32_t nrec = P.grid * (uint32_t)kCWaves;
    if (n)
      hipLaunchKernelGGL(xc_fix_kernel, dim3((nrec + 255) / 256), dim3(256), 0, stream, P.out_fix, nrec, P.out_start,
                         P.out_len, n);
    return hipGetLastError();
  }
  if (P.inbits && !P.xc_w && !P.xu_w) {
    if (P.xu_tab && !P.xu_exact)
      hipLaunchKernelGGL((xu_bm_kernel<true>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    else if (P.xu_tab)
      hipLaunchKernelGGL((xu_bm_kernel<false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    else
      hipLaunchKernelGGL(xc_bm_kernel, dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
    return hipGetLastError();
  }
  // (U mode: the FAST kernel unless the host redoes a range that met an XU_MIX
  // or XU_SLOW lead, UGPU_FLAG_UMIX)
  if (P.xu_tab && P.xu_w && !P.xu_exact)
    hipLaunchKernelGGL((xu_kernel<true, true>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  else if (P.xu_tab && P.xu_w)
    hipLaunchKernelGGL((xu_kernel<true, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  else if (P.xu_tab && !P.xu_exact)
    hipLaunchKernelGGL((xu_kernel<false, true>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  else if (P.xu_tab)
    hipLaunchKernelGGL((xu_kernel<false, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  else if (P.xc_w)
    hipLaunchKernelGGL((xc_kernel<true, false, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  else
    hipLaunchKernelGGL((xc_kernel<false, false, false>), dim3(P.grid), dim3(kCWaves * 64), 0, stream, P);
  return hipGetLastError();
}

hipError_t xc_occupancy(bool u, int* n)
{
  if (u) return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xu_kernel<false, true>, kCWaves * 64, 0);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, xc_kernel<true, true, false>, kCWaves * 64, 0);
}
uint32_t xc_unit(bool u) { return u ? kCChunk * kUIter : kCTile; }
uint32_t xc_waves() { return kCWaves; }

hipError_t launch_xc_expand(const ScanParams& P, hipStream_t stream, uint64_t count)
{
  const uint32_t nrec = P.grid * (uint32_t)kCWaves;
  // (UGPU_XE_WAVES: 1 = one wave per COUNT wave, no counting pass; 4 = quarters)
  static const int nw = [] {
    const char* e = std::getenv("UGPU_XE_WAVES");
    return e && *e == '1' ? 1 : 4;
  }();
  if (nw == 4) {
    if (P.xu_tab)
      hipLaunchKernelGGL((xc_expand_kernel<true, 4>), dim3(nrec), dim3(256), 0, stream, P);
    else
      hipLaunchKernelGGL((xc_expand_kernel<false, 4>), dim3(nrec), dim3(256), 0, stream, P);
  } else {
    if (P.xu_tab)
      hipLaunchKernelGGL((xc_expand_kernel<true, 1>), dim3(nrec), dim3(64), 0, stream, P);
    else
      hipLaunchKernelGGL((xc_expand_kernel<false, 1>), dim3(nrec), dim3(64), 0, stream, P);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t n = count < P.out_capacity ? count : P.out_capacity;
  if (n)
    hipLaunchKernelGGL(xc_fix_kernel, dim3((nrec + 255) / 256), dim3(256), 0, stream, P.out_fix, nrec, P.out_start,
                       P.out_len, n);
  return hipGetLastError();
}

}  // namespace ugpu
