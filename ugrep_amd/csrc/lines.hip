// lines.hip -- line-level consumers of the FIND results.
//
// Replaces, for a fully buffered input:
//   * newline counting for line numbers: AbstractMatcher::lineno()
//     (include/reflex/absmatcher.h:695-766) over simd nlcount
//     (lib/simd.cpp:62-166, lib/simd_avx2.cpp:48-79);
//   * ugrep -c's matching-line count: one count per line holding a match, the
//     search skipping to the next line after the first hit
//     (src/ugrep.cpp:10567-10586).  For patterns whose matches cannot contain
//     '\n' this is the number of distinct lines holding a match start.
//
// Two wave-persistent passes over 4 KiB tiles (the sparse kernel's load
// scheme: per-tile buffer resources, non-temporal 16 B/lane loads):
//   nl_count_kernel  newlines per wave range (sparse mode: also per 1 KiB
//                    quarter, u16, 1/512 of the input written);
//   (host)           exclusive scan of the per-wave counts (<= 8192 values);
//   nl_assign_kernel line = 1 + newlines before each match start, walking the
//                    sorted match list alongside the bytes, 64 matches per
//                    step; per-wave line transition counts for -c, stitched on
//                    the host.  Dense mode reloads every tile and keeps its
//                    16-byte granule masks and prefix in LDS; sparse mode
//                    (matches rarer than one per ~2 KiB, e.g. C2) loads only
//                    the quarters holding a match start, adds the quarter
//                    prefix from qcount and gathers granule masks across lanes
//                    with ds_bpermute, so the second pass reads ~1 KiB per
//                    match instead of the whole buffer.
#include "device_common.hpp"

namespace ugpu {

namespace {

constexpr int kLTile = 4096;
constexpr int kLWaves = 4;

__device__ __forceinline__ uint4 lload16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2 /* nt */);
  return uint4{v.x, v.y, v.z, v.w};
}

// bit 7 of each byte set iff the byte is '\n' (exact: no carries between bytes)
__device__ __forceinline__ uint32_t nl_bits(uint32_t x)
{
  const uint32_t t = x ^ 0x0a0a0a0au;
  const uint32_t nz = ((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t;
  return ~nz & 0x80808080u;
}

// 4-bit mask of newline bytes of a dword
__device__ __forceinline__ uint32_t nl4(uint32_t x) { return ((nl_bits(x) >> 7) * 0x01020408u) >> 24; }

__device__ __forceinline__ uint32_t nl16(const uint4& v)
{
  return nl4(v.x) | (nl4(v.y) << 4) | (nl4(v.z) << 8) | (nl4(v.w) << 12);
}

// Tile i of the range starting at wbase (rel = readable bytes from wbase).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ltile(const uint8_t* wbase, uint32_t i, uint32_t rel)
{
  const uint32_t off = i * (uint32_t)kLTile;
  const uint32_t n = rel > off ? rel - off : 0u;
  const int nr = __builtin_amdgcn_readfirstlane((int)(n < (uint32_t)kLTile ? n : (uint32_t)kLTile));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wbase + off), (short)0, nr, 0x00020000);
}

__device__ __forceinline__ uint32_t lscan_add(uint32_t v)
{
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

struct LRange {
  uint64_t lo, hi;  // byte range [lo, hi) of this wave
  uint32_t n;       // tiles
  uint32_t rel;     // bytes of the range (hi - lo)
  uint32_t rel16;   // rel rounded up to 16: the loads' bound (a buffer load
                    // past num_records zeroes the whole dword, so a ragged end
                    // is loaded whole, inside the aligned 16-byte granule, and
                    // masked with granule_valid)
};

// 16-bit mask of the bytes of granule [off, off+16) that lie below rel
__device__ __forceinline__ uint32_t granule_valid(uint32_t rel, uint32_t off)
{
  const uint32_t rem = rel > off ? rel - off : 0u;
  return rem >= 16u ? 0xffffu : (1u << rem) - 1u;
}

__device__ __forceinline__ LRange lrange(const LinesParams& L, uint64_t gw)
{
  LRange r;
  r.lo = gw * L.per;
  if (r.lo > L.len) r.lo = L.len;
  r.hi = r.lo + L.per < L.len ? r.lo + L.per : L.len;
  r.n = (uint32_t)((r.hi - r.lo + kLTile - 1) / kLTile);
  r.rel = (uint32_t)(r.hi - r.lo);
  r.rel16 = (r.rel + 15u) & ~15u;
  return r;
}

// First match with start >= lo: 64-ary search over the sorted starts.
__device__ __forceinline__ uint64_t first_match(const LinesParams& L, uint64_t lo, int lane)
{
  uint64_t a = 0, b = L.nmatch;  // answer in [a, b]
  while (b - a > 64) {
    const uint64_t step = (b - a + 63) / 64;
    const uint64_t idx = a + step * (uint64_t)lane;
    const bool below = idx < b && L.starts[idx] < lo;
    const int cntb = __popcll(__ballot(below));  // pivots below lo (a prefix of the lanes)
    const uint64_t na = cntb ? a + step * (uint64_t)(cntb - 1) + 1 : a;
    const uint64_t nb = a + step * (uint64_t)cntb;
    a = na;
    b = nb < b ? nb : b;
  }
  const uint64_t idx = a + (uint64_t)lane;
  const bool below = idx < b && L.starts[idx] < lo;
  return a + __popcll(__ballot(below));
}

// Per-wave -c bookkeeping over the wave's matches in order, 64 at a time
// (lanes holding a match form a prefix).
struct LineStats {
  uint64_t prev_line = 0, first_line = 0, trans = 0, nm = 0;

  __device__ __forceinline__ void add(uint64_t ln, bool in, uint64_t mb, int lane)
  {
    const uint64_t pl = __shfl_up(ln, 1, 64);
    const uint64_t before = lane == 0 ? prev_line : pl;
    const bool newl = in && (nm + (uint64_t)lane == 0 || ln != before);
    const uint32_t k = (uint32_t)__popcll(mb);
    trans += __popcll(__ballot(newl));
    if (nm == 0) first_line = __shfl(ln, 0, 64);
    prev_line = __shfl(ln, (int)k - 1, 64);
    nm += k;
  }

  __device__ __forceinline__ void store(LineRec* rec, int lane) const
  {
    if (lane == 0) {
      LineRec r;
      r.first_line = first_line;
      r.last_line = prev_line;
      r.trans = trans;
      r.nmatch = nm;
      *rec = r;
    }
  }
};

}  // namespace

template <bool SPARSE>
__global__ __launch_bounds__(kLWaves * 64) void nl_count_kernel(LinesParams L)
{
  const int lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * kLWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw >= L.nwaves) return;
  const LRange r = lrange(L, gw);
  uint32_t cnt = 0;
  for (uint32_t i = 0; i < r.n; ++i) {
    const __amdgpu_buffer_rsrc_t rs = ltile(L.g + r.lo, i, r.rel16);
    uint32_t c[4];
    if ((i + 1u) * (uint32_t)kLTile <= r.rel) {  // whole tile (uniform branch)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 v = lload16(rs, 16u * lane + 1024u * k);
        c[k] = __popc(nl_bits(v.x)) + __popc(nl_bits(v.y)) + __popc(nl_bits(v.z)) + __popc(nl_bits(v.w));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t o = 16u * lane + 1024u * k;
        c[k] = __popc(nl16(lload16(rs, o)) & granule_valid(r.rel, i * (uint32_t)kLTile + o));
      }
    }
    cnt += c[0] + c[1] + c[2] + c[3];
    if (SPARSE) {  // quarter counts (<= 1024 each) packed two per dword, one scan each
      const uint32_t p01 = (uint32_t)__builtin_amdgcn_readlane(lscan_add(c[0] | (c[1] << 16)), 63);
      const uint32_t p23 = (uint32_t)__builtin_amdgcn_readlane(lscan_add(c[2] | (c[3] << 16)), 63);
      if (lane == 0)
        reinterpret_cast<uint64_t*>(L.qcount)[(r.lo / kLTile) + i] = (uint64_t)p01 | ((uint64_t)p23 << 32);
    }
  }
  const uint64_t t = wave_sum(cnt);
  if (lane == 0) L.counts[gw] = t;
}

__global__ __launch_bounds__(kLWaves * 64) void nl_assign_kernel(LinesParams L)
{
  __shared__ uint16_t gmask[kLWaves][256], gpre[kLWaves][256];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kLWaves + wid;
  if (gw >= L.nwaves) return;
  const LRange r = lrange(L, gw);
  uint64_t j = first_match(L, r.lo, lane);  // next match to assign
  uint64_t line = 1 + L.prefix[gw];         // line of byte r.lo
  LineStats st;
  uint16_t* gm = gmask[wid];
  uint16_t* gp = gpre[wid];
  for (uint32_t i = 0; i < r.n && j < L.nmatch; ++i) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous tile's LDS reads precede these writes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t ts = r.lo + (uint64_t)i * kLTile;
    const __amdgpu_buffer_rsrc_t rs = ltile(L.g + r.lo, i, r.rel16);
    uint32_t c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t o = 16u * lane + 1024u * k;
      const uint32_t m = nl16(lload16(rs, o)) & granule_valid(r.rel, i * (uint32_t)kLTile + o);
      gm[64 * k + lane] = (uint16_t)m;
      c[k] = __popc(m);
    }
    // exclusive prefix over granules g = 64 k + lane (tile order)
    uint32_t base = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t incl = lscan_add(c[k]);
      gp[64 * k + lane] = (uint16_t)(base + incl - c[k]);
      base += (uint32_t)__builtin_amdgcn_readlane(incl, 63);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t tend = ts + kLTile < r.hi ? ts + kLTile : r.hi;
    for (;;) {  // matches starting in this tile, 64 at a time
      const uint64_t idx = j + (uint64_t)lane;
      const uint64_t s = idx < L.nmatch ? L.starts[idx] : ~0ull;
      const bool in = s < tend;
      const uint64_t mb = __ballot(in);
      if (!mb) break;
      uint64_t ln = 0;
      if (in) {
        const uint32_t o = (uint32_t)(s - ts), g = o >> 4;
        ln = line + gp[g] + __popc((uint32_t)gm[g] & ((1u << (o & 15)) - 1u));
        if (L.lines) L.lines[idx] = ln;
      }
      st.add(ln, in, mb, lane);
      const uint32_t k = (uint32_t)__popcll(mb);
      j += k;
      if (k < 64) break;
    }
    line += base;
    if (j >= L.nmatch || L.starts[j] >= r.hi) break;  // no further match in this range
  }
  st.store(L.recs + gw, lane);
}

__global__ __launch_bounds__(kLWaves * 64) void nl_assign_sparse_kernel(LinesParams L)
{
  const int lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * kLWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw >= L.nwaves) return;
  const LRange r = lrange(L, gw);
  uint64_t j = first_match(L, r.lo, lane);
  uint64_t line = 1 + L.prefix[gw];
  LineStats st;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(L.g + r.lo), (short)0, __builtin_amdgcn_readfirstlane((int)r.rel16), 0x00020000);
  const uint32_t nquart = (r.rel + kLinesQuarter - 1) / kLinesQuarter;
  const uint16_t* qc = L.qcount + r.lo / kLinesQuarter;
  for (uint32_t qb = 0; qb < nquart && j < L.nmatch; qb += 64) {
    uint64_t s = L.starts[j];
    if (s >= r.hi) break;
    // line offsets of the next 64 quarters
    const uint32_t nq = nquart - qb < 64u ? nquart - qb : 64u;
    const uint32_t c = (uint32_t)lane < nq ? qc[qb + lane] : 0u;
    const uint32_t incl = lscan_add(c);
    const uint32_t excl = incl - c;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
    const uint64_t bend0 = r.lo + (uint64_t)(qb + nq) * kLinesQuarter;
    const uint64_t bend = bend0 < r.hi ? bend0 : r.hi;
    while (s < bend) {  // each quarter holding a match start
      const uint32_t q = (uint32_t)((s - r.lo) / kLinesQuarter);
      const uint32_t qo = q * kLinesQuarter;
      const uint64_t qs = r.lo + qo;
      const uint64_t qe = qs + kLinesQuarter < r.hi ? qs + kLinesQuarter : r.hi;
      const uint64_t qline = line + (uint32_t)__builtin_amdgcn_readlane(excl, (int)(q - qb));
      const uint32_t go = qo + 16u * lane;
      const uint32_t m = nl16(lload16(rs, go)) & granule_valid(r.rel, go);
      const uint32_t cm = __popc(m);
      const uint32_t pre = lscan_add(cm) - cm;
      for (;;) {  // matches in this quarter, 64 at a time
        const uint64_t idx = j + (uint64_t)lane;
        const uint64_t sl = idx < L.nmatch ? L.starts[idx] : ~0ull;
        const bool in = sl < qe;
        const uint64_t mb = __ballot(in);
        if (!mb) break;  // the quarter held a multiple of 64 starts
        const uint32_t o = in ? (uint32_t)(sl - qs) : 0u;
        const int g = (int)(o >> 4);
        const uint32_t pg = (uint32_t)__shfl((int)pre, g, 64);  // all lanes take part
        const uint32_t mg = (uint32_t)__shfl((int)m, g, 64);
        const uint64_t ln = in ? qline + pg + __popc(mg & ((1u << (o & 15)) - 1u)) : 0ull;
        if (in && L.lines) L.lines[idx] = ln;
        st.add(ln, in, mb, lane);
        const uint32_t k = (uint32_t)__popcll(mb);
        j += k;
        if (k < 64) break;
      }
      s = j < L.nmatch ? L.starts[j] : ~0ull;
    }
    line += total;
  }
  st.store(L.recs + gw, lane);
}

hipError_t launch_nl_count(const LinesParams& L, bool sparse, hipStream_t stream)
{
  const uint32_t grid = (uint32_t)((L.nwaves + kLWaves - 1) / kLWaves);
  if (sparse)
    hipLaunchKernelGGL(nl_count_kernel<true>, dim3(grid), dim3(kLWaves * 64), 0, stream, L);
  else
    hipLaunchKernelGGL(nl_count_kernel<false>, dim3(grid), dim3(kLWaves * 64), 0, stream, L);
  return hipGetLastError();
}

hipError_t launch_nl_assign(const LinesParams& L, bool sparse, hipStream_t stream)
{
  const uint32_t grid = (uint32_t)((L.nwaves + kLWaves - 1) / kLWaves);
  if (sparse)
    hipLaunchKernelGGL(nl_assign_sparse_kernel, dim3(grid), dim3(kLWaves * 64), 0, stream, L);
  else
    hipLaunchKernelGGL(nl_assign_kernel, dim3(grid), dim3(kLWaves * 64), 0, stream, L);
  return hipGetLastError();
}

uint32_t lines_tile() { return kLTile; }

}  // namespace ugpu
