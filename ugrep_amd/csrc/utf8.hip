// utf8.hip -- binary-file detection on the device.
//
// Replaces, for a fully buffered input:
//   * reflex::isutf8(s, e) (lib/simd.cpp:169-421; AVX2 body
//     lib/simd_avx2.cpp:82-150): true iff [s, e) is a sequence of
//     ASCII 0x01-0x7f | [c2-df] cont | [e0-ef] cont{2} | [f0-f4] cont{3}
//     (cont = 80-bf; NUL, c0, c1, f5-ff rejected; surrogates and 3/4-byte
//     overlongs pass, as in the reference);
//   * memchr(s, '\0', n), the NUL test ugrep uses with -a/-U
//     (src/ugrep.cpp:698-711).
//
// The reference's p/q/r recurrence (simd.cpp:201-216) makes the check local:
// byte i needs a continuation iff b[i-1] >= c0 or b[i-2] >= e0 or
// b[i-3] >= f0, and the buffer is valid iff every byte is a valid byte whose
// continuation-ness equals that need, and position n (the end) needs none.
// So one pass reports the first failing position; the reference's
// SIMD/scalar split, ASCII prescan and end backtrack (simd.cpp:174-183,
// :296-298) do not change the result.
//
// Layout: wave-persistent over ranges of whole 4 KiB tiles, the tile loaded
// as 4 coalesced non-temporal 16 B/lane buffer loads.  A tile that is pure
// ASCII without NUL (one OR and one zero-byte test per dword) costs one
// ballot; otherwise the exact per-byte test runs on the registers it already
// holds, with the lead flags of the previous 3 bytes passed from lane l-1 by
// DPP (wave_shr) and from lane 63 to the next 1 KiB chunk.  A wave stops at its
// first failing byte (atomicMin of the position) and when a lower position
// has already been found.
#include "device_common.hpp"

namespace ugpu {

namespace {

constexpr int kUTile = 4096;
constexpr int kUWaves = 4;

__device__ __forceinline__ uint4 uload16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2 /* nt */);
  return uint4{v.x, v.y, v.z, v.w};
}

// bytes [lo, hi) of the dword at relative offset o are inside the buffer; the
// others are replaced by 0x01 (valid ASCII that needs no continuation and
// leaves no lead behind)
__device__ __forceinline__ uint32_t clip(uint32_t c, uint64_t o, uint64_t lo, uint64_t hi)
{
  const uint32_t a = lo > o ? (uint32_t)(lo - o < 4 ? lo - o : 4) : 0u;  // bytes below lo
  const uint32_t b = hi > o ? (uint32_t)(hi - o < 4 ? hi - o : 4) : 0u;  // bytes below hi
  const uint32_t mb = b >= 4 ? 0xffffffffu : (1u << (8 * b)) - 1u;
  const uint32_t ma = a >= 4 ? 0xffffffffu : (1u << (8 * a)) - 1u;
  const uint32_t m = mb & ~ma;
  return (c & m) | (0x01010101u & ~m);
}

// Lead flags (bit 7 of each byte): l2 = byte >= c0, l3 = byte >= e0, l4 = byte >= f0.
struct Lead {
  uint32_t l2, l3, l4;
};

__device__ __forceinline__ Lead lead(uint32_t c)
{
  Lead f;
  f.l2 = c & (c << 1);
  f.l3 = f.l2 & (c << 2);
  f.l4 = f.l3 & (c << 3);
  return f;
}

// bit 7 of each byte: the byte fails (invalid byte, or continuation-ness differs
// from the need set by the 3 preceding bytes, whose lead flags are in p)
__device__ __forceinline__ uint32_t bad_bytes(uint32_t c, const Lead& f, const Lead& p)
{
  const uint32_t need = __builtin_amdgcn_alignbyte(f.l2, p.l2, 3) | __builtin_amdgcn_alignbyte(f.l3, p.l3, 2) |
                        __builtin_amdgcn_alignbyte(f.l4, p.l4, 1);
  const uint32_t cont = c & ~(c << 1);                                   // 10xxxxxx
  const uint32_t zero = ~(((c & 0x7f7f7f7fu) + 0x7f7f7f7fu) | c);        // 0x00
  const uint32_t y = c ^ 0xc0c0c0c0u;
  const uint32_t c01 = ~(((y & 0x7e7e7e7eu) + 0x7e7e7e7eu) | y);         // 0xc0, 0xc1
  const uint32_t f5 = f.l4 & (((c & 0x0f0f0f0fu) + 0x0b0b0b0bu) << 3);  // 0xf5-0xff
  return (zero | c01 | f5 | (need ^ cont)) & 0x80808080u;
}

__device__ __forceinline__ uint32_t zero_bytes(uint32_t c) { return ~(((c & 0x7f7f7f7fu) + 0x7f7f7f7fu) | c) & 0x80808080u; }

// value of lane l-1 (lane 0: `first`, wave-uniform)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t first)
{
  return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
}

}  // namespace

// mode NUL: first 0x00 byte (memchr); otherwise the first byte failing isutf8.
template <bool NUL>
__global__ __launch_bounds__(kUWaves * 64) void utf8_kernel(Utf8Params U)
{
  const int lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * kUWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw >= U.nwaves) return;
  // this wave's byte range [lo, hi) of the aligned span [0, span)
  const uint64_t lo = gw * U.per;
  if (lo >= U.span) return;
  const uint64_t hi = lo + U.per < U.span ? lo + U.per : U.span;
  const uint32_t rel = (uint32_t)(hi - lo);
  const uint32_t rel16 = (rel + 15u) & ~15u;
  const uint8_t* wbase = U.g + lo;
  const uint64_t dend = U.head + U.len;  // data bytes are [head, dend) of the span

  Lead carry{0u, 0u, 0u};  // lead flags of the dword before the current chunk (lane 63's last)
  if (!NUL && lo > 0) {
    const uint32_t c = clip(*reinterpret_cast<const uint32_t*>(wbase - 4), lo - 4, U.head, dend);
    carry = lead(c);
  }
  const uint32_t ntiles = (rel + kUTile - 1) / kUTile;
  uint64_t found = ~0ull;
  for (uint32_t i = 0; i < ntiles; ++i) {
    if ((i & 7u) == 7u && __hip_atomic_load(U.out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < lo) break;
    const uint32_t toff = i * (uint32_t)kUTile;
    const uint32_t n = rel16 - toff < (uint32_t)kUTile ? rel16 - toff : (uint32_t)kUTile;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(wbase + toff), (short)0, __builtin_amdgcn_readfirstlane((int)n), 0x00020000);
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = uload16(rs, 16u * lane + 1024u * k);
    const uint64_t tbase = lo + toff;
    // head/tail tiles: bytes outside the data become 0x01 (uniform branch)
    if (tbase < U.head || tbase + kUTile > dend) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t o = tbase + 16u * lane + 1024u * k;
        v[k].x = clip(v[k].x, o, U.head, dend);
        v[k].y = clip(v[k].y, o + 4, U.head, dend);
        v[k].z = clip(v[k].z, o + 8, U.head, dend);
        v[k].w = clip(v[k].w, o + 12, U.head, dend);
      }
    }
    // fast test: pure ASCII without NUL (bit 7 set by a high byte or a zero byte)
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (NUL) {
        acc |= zero_bytes(v[k].x) | zero_bytes(v[k].y) | zero_bytes(v[k].z) | zero_bytes(v[k].w);
      } else {
        const uint32_t c[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) acc |= c[j] | ((c[j] - 0x01010101u) & ~c[j]);
      }
    }
    const bool hit = __ballot((acc & 0x80808080u) != 0u) != 0ull || (carry.l2 | carry.l3 | carry.l4) != 0u;
    if (!hit) continue;  // (carry stays 0: the tile ended in ASCII)
    // exact test, chunk by chunk (1 KiB each, lane l holds bytes [16 l, 16 l + 16))
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t c[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      uint32_t bad[4];
      if (NUL) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bad[j] = zero_bytes(c[j]);
      } else {
        Lead f[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = lead(c[j]);
        Lead p;
        p.l2 = from_prev_lane(f[3].l2, carry.l2);
        p.l3 = from_prev_lane(f[3].l3, carry.l3);
        p.l4 = from_prev_lane(f[3].l4, carry.l4);
        bad[0] = bad_bytes(c[0], f[0], p);
#pragma unroll
        for (int j = 1; j < 4; ++j) bad[j] = bad_bytes(c[j], f[j], f[j - 1]);
        carry.l2 = (uint32_t)__builtin_amdgcn_readlane((int)f[3].l2, 63);
        carry.l3 = (uint32_t)__builtin_amdgcn_readlane((int)f[3].l3, 63);
        carry.l4 = (uint32_t)__builtin_amdgcn_readlane((int)f[3].l4, 63);
      }
      const uint32_t any = bad[0] | bad[1] | bad[2] | bad[3];
      const uint64_t lanes = __ballot(any != 0u);
      if (lanes) {
        const int l0 = __builtin_ctzll(lanes);  // first lane holding a failing byte
        uint32_t off = 0;
        if (lane == l0) {
          const int j = bad[0] ? 0 : bad[1] ? 1 : bad[2] ? 2 : 3;
          off = 16u * (uint32_t)lane + 4u * (uint32_t)j + (uint32_t)(__builtin_ctz(bad[j]) >> 3);
        }
        off = (uint32_t)__builtin_amdgcn_readlane((int)off, l0);
        found = tbase + 1024u * (uint32_t)k + off;
        break;
      }
    }
    if (found != ~0ull) break;
  }
  // the end of the data needs no continuation (isutf8 rejects a truncated
  // sequence; a ragged end was clipped to 0x01 bytes and tested above)
  if (!NUL && found == ~0ull && hi == U.span && dend == U.span) {
    const uint32_t need = (carry.l2 >> 24) | (carry.l3 >> 16) | (carry.l4 >> 8);
    if (need & 0x80u) found = dend;
  }
  if (found != ~0ull && lane == 0) atomicMin(reinterpret_cast<unsigned long long*>(U.out), found);
}

hipError_t launch_utf8(const Utf8Params& U, bool nul, hipStream_t stream)
{
  const uint32_t grid = (uint32_t)((U.nwaves + kUWaves - 1) / kUWaves);
  if (nul)
    hipLaunchKernelGGL(utf8_kernel<true>, dim3(grid), dim3(kUWaves * 64), 0, stream, U);
  else
    hipLaunchKernelGGL(utf8_kernel<false>, dim3(grid), dim3(kUWaves * 64), 0, stream, U);
  return hipGetLastError();
}

uint32_t utf8_tile() { return kUTile; }

}  // namespace ugpu
