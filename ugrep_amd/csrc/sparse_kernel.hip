// sparse_kernel.hip -- wave-persistent FIND kernel for prefiltered patterns
// (needle-like first bytes: C1 -F lorem, C2 foo|bar|baz).
//
// Replaces the reference's adv_ prefilter loop + per-candidate DFA walk
// (lib/matcher_avx2.cpp:475-527 ADV_PAT_PIN, lib/matcher.cpp:42-750) for byte
// tables whose first bytes have a small exact term cover (tables.hpp).
//
// Each wave owns a contiguous range of 4 KiB wave-tiles and walks it alone, so
// the main loop has no workgroup barrier:
//   1. 4 KiB wave-tiles arrive by coalesced 16 B/lane loads, one tile ahead in
//      registers, and are stored to the wave's LDS slice;
//   2. the SWAR prefilter reads chunk k of lane l = bytes [1024k + 16l, +16)
//      -> 16-bit candidate mask per chunk (walks read the same LDS tile);
//   3. candidates are compacted in position order (packed DPP scans) into
//      an LDS list, and up to 64 are walked at once, one per lane: a walk from
//      c is independent of the chain, so all walks run in parallel;
//   4. the FIND chain over candidates is the greedy rule "keep the match at c
//      iff c >= end of the last kept match" (Appendix A: a non-candidate
//      position only steps p+1).  With an exclusive prefix-max of match ends
//      the rule is exact unless two candidate matches overlap; those batches
//      fall back to a 64-step in-wave sequential pass.
// Per-wave chain records (entry, exit, counts) are stitched by fix_kernel.
#include "device_common.hpp"

namespace ugpu {

namespace {

// 16-bit candidate mask of one 16-byte chunk (bytes 4j..4j+3 = wd[j]); `nx`
// holds the 4 bytes that follow the chunk; when `nx_known` is false the
// second-byte test of the chunk's last byte passes (a superset is safe).
// Prefilter bucket bits of the 4 bytes of x (tables.hpp): three v_perm_b32
// byte-table lookups on the lo3 / mid3 / hi2 fields of every byte, ANDed;
// then U = R | R >> 1 folds each set's two buckets (B -> bit 1, C -> bit 3,
// D -> bit 5; A stays bit 0 of R).
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

// 16-bit candidate mask of one 16-byte chunk: bit i set iff byte i passes
// A(i) | (B(i) & C(i+1) & D(i+2)).  R[j] = bucket_bits of dword j of the
// chunk, R[4] = of the 4 bytes after it (all ones when unknown: they pass).
__device__ __forceinline__ uint32_t chunk_mask(const uint32_t (&R)[5])
{
  uint32_t U[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) U[j] = R[j] | (R[j] >> 1);
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // byte i of alignbyte(next, cur, s) = byte i+s of the pair (cur, next);
    // every term is moved to bit 5 of its byte (no carries cross bytes)
    const uint32_t bcd = (U[j] << 4) & (__builtin_amdgcn_alignbyte(U[j + 1], U[j], 1) << 2) &
                         __builtin_amdgcn_alignbyte(U[j + 1], U[j], 2);
    const uint32_t cand = (bcd | (R[j] << 5)) & 0x20202020u;
    m |= ((((cand >> 5) * 0x00204081u) >> 21) & 0xfu) << (4 * j);
  }
  return m;
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

}  // namespace

template <bool WRITE>
__global__ __launch_bounds__(kSpWaves * 64) void sparse_kernel(ScanParams P)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar control flow
  uint8_t* wt = smem + wid * kWaveTile;
  uint16_t* cl = reinterpret_cast<uint16_t*>(smem + kSpWaves * kWaveTile) + wid * kCandCap;
  uint16_t* ltrans = reinterpret_cast<uint16_t*>(smem + kSpWaves * (kWaveTile + 2 * kCandCap));
  uint32_t* lcaps = reinterpret_cast<uint32_t*>(ltrans + P.ntrans_pad);
  {
    const uint4* src = reinterpret_cast<const uint4*>(P.trans);
    uint4* dst = reinterpret_cast<uint4*>(ltrans);
    for (uint32_t i = tid; i < P.ntrans_pad / 8; i += kSpWaves * 64) dst[i] = src[i];
    for (uint32_t i = tid; i < P.nstates; i += kSpWaves * 64) lcaps[i] = P.caps[i];
  }
  __syncthreads();  // the only workgroup barrier: tables staged
  const Tab<0> T{ltrans, nullptr, P.start, P.accb};
  const Ctx C{lcaps, P.log_row, P.delta};
  const FTab F{P.ft[0], P.ft[1], P.ft[2], P.ft[3], P.ft[4]};

  const uint64_t gw = (uint64_t)blockIdx.x * kSpWaves + wid;
  uint64_t tb = P.t0 + gw * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * kWaveTile, P.lo, P.hi);
  const uint64_t whi = clampu(te * kWaveTile, P.lo, P.hi);
  uint64_t x = WRITE ? P.entries[gw] : wlo;  // chain position (wave-uniform)

  Win w;
  w.lds = wt;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0, wover = 0;
  CountEm acc;
  uint64_t widx = WRITE ? P.out_base[gw] : 0;

  // 1. each tile arrives by coalesced 16 B/lane loads one tile ahead in
  //    registers; the current tile is stored to the wave's LDS slice, which the
  //    prefilter and the walks read.
  const uint64_t last16 = (P.rend - 1) & ~uint64_t(15);  // clamp: bytes >= rend are never consulted
  // (unconditional loads into named registers: a conditionally written array
  // captured by a lambda was demoted to scratch by hipcc)
  // Two tiles in flight per wave (r* = tile t+1, q* = tile t+2 at the top of
  // iteration t): 24 waves x 8 KiB per CU cover the loaded HBM latency.
  uint4 r0, r1, r2, r3, q0, q1, q2, q3;
  {
    const uint64_t p = (tb < te ? tb : 0) * kWaveTile + 16u * lane;
    r0 = load16(P.g, p, last16);
    r1 = load16(P.g, p + 1024, last16);
    r2 = load16(P.g, p + 2048, last16);
    r3 = load16(P.g, p + 3072, last16);
    const uint64_t p2 = (tb + 1 < te ? tb + 1 : tb) * kWaveTile + 16u * lane;
    q0 = load16(P.g, p2, last16);
    q1 = load16(P.g, p2 + 1024, last16);
    q2 = load16(P.g, p2 + 2048, last16);
    q3 = load16(P.g, p2 + 3072, last16);
  }
  for (uint64_t t = tb; t < te; ++t) {
    const uint64_t ts = t * kWaveTile;
    *reinterpret_cast<uint4*>(wt + 16 * lane) = r0;
    *reinterpret_cast<uint4*>(wt + 1024 + 16 * lane) = r1;
    *reinterpret_cast<uint4*>(wt + 2048 + 16 * lane) = r2;
    *reinterpret_cast<uint4*>(wt + 3072 + 16 * lane) = r3;
    w.base = ts;
    w.lend = ts + kWaveTile;

    // 2. prefilter on the registers: chunk k of this lane = bytes
    //    [1024k + 16l, +16); the 4 bytes after it are the next lane's first
    //    dword (DPP wave_shl:1), or lane 0's of chunk k+1 for lane 63.
    uint32_t m[4];
    if (P.ablate != 1) {
      const uint32_t h0 = bucket_bits(r0.x, F), h1 = bucket_bits(r1.x, F), h2 = bucket_bits(r2.x, F),
                     h3 = bucket_bits(r3.x, F);
      const uint32_t n0 = __builtin_amdgcn_update_dpp(0, h0, 0x130, 0xf, 0xf, false);
      const uint32_t n1 = __builtin_amdgcn_update_dpp(0, h1, 0x130, 0xf, 0xf, false);
      const uint32_t n2 = __builtin_amdgcn_update_dpp(0, h2, 0x130, 0xf, 0xf, false);
      const uint32_t n3 = __builtin_amdgcn_update_dpp(0, h3, 0x130, 0xf, 0xf, false);
      const bool l63 = lane == 63;
      const uint32_t R0[5] = {h0, bucket_bits(r0.y, F), bucket_bits(r0.z, F), bucket_bits(r0.w, F),
                              l63 ? (uint32_t)__builtin_amdgcn_readlane(h1, 0) : n0};
      m[0] = chunk_mask(R0);
      const uint32_t R1[5] = {h1, bucket_bits(r1.y, F), bucket_bits(r1.z, F), bucket_bits(r1.w, F),
                              l63 ? (uint32_t)__builtin_amdgcn_readlane(h2, 0) : n1};
      m[1] = chunk_mask(R1);
      const uint32_t R2[5] = {h2, bucket_bits(r2.y, F), bucket_bits(r2.z, F), bucket_bits(r2.w, F),
                              l63 ? (uint32_t)__builtin_amdgcn_readlane(h3, 0) : n2};
      m[2] = chunk_mask(R2);
      const uint32_t R3[5] = {h3, bucket_bits(r3.y, F), bucket_bits(r3.z, F), bucket_bits(r3.w, F),
                              l63 ? 0xffffffffu : n3};  // bytes past the wave-tile: unknown, pass
      m[3] = chunk_mask(R3);
    }
    r0 = q0;
    r1 = q1;
    r2 = q2;
    r3 = q3;
    {
      const uint64_t p = (t + 2 < te ? t + 2 : t) * kWaveTile + 16u * lane;  // tail: harmless re-read
      q0 = load16(P.g, p, last16);
      q1 = load16(P.g, p + 1024, last16);
      q2 = load16(P.g, p + 2048, last16);
      q3 = load16(P.g, p + 3072, last16);
    }
    wave_lds_sync();
    if (P.ablate == 1) {  // benchmarking only: staging alone
      acc.cnt += wt[lane];
      x = ts + kWaveTile < whi ? ts + kWaveTile : whi;
      wave_lds_sync();
      continue;
    }
    if (ts < wlo || ts + kWaveTile > whi) {  // first/last tile: clip to [wlo, whi)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t p0 = ts + 1024u * k + 16u * lane;
        const uint64_t a = wlo > p0 ? (wlo - p0 > 16 ? 16 : wlo - p0) : 0;
        const uint64_t z = whi > p0 ? (whi - p0 > 16 ? 16 : whi - p0) : 0;
        m[k] &= (uint32_t)((lowbits(z) & ~lowbits(a)) & 0xffffu);
      }
    }

    if (P.ablate == 2) {  // benchmarking only: staging + prefilter
      acc.cnt += __popc(m[0] | m[1] | m[2] | m[3]);
      x = ts + kWaveTile < whi ? ts + kWaveTile : whi;
      wave_lds_sync();
      continue;
    }
    if (__ballot((m[0] | m[1] | m[2] | m[3]) != 0)) {
      // 3. compact candidates in position order (k-major, then lane, then byte):
      //    two packed DPP scans of the per-chunk counts (16-bit fields)
      const uint32_t c01 = __popc(m[0]) | (__popc(m[1]) << 16), c23 = __popc(m[2]) | (__popc(m[3]) << 16);
      const uint32_t i01 = dpp_scan_add(c01), i23 = dpp_scan_add(c23);
      const uint32_t t01 = __builtin_amdgcn_readlane(i01, 63), t23 = __builtin_amdgcn_readlane(i23, 63);
      const uint32_t e01 = i01 - c01, e23 = i23 - c23;
      const uint32_t tot0 = t01 & 0xffffu, tot1 = t01 >> 16, tot2 = t23 & 0xffffu, tot3 = t23 >> 16;
      const uint32_t base[4] = {e01 & 0xffffu, tot0 + (e01 >> 16), tot0 + tot1 + (e23 & 0xffffu),
                                tot0 + tot1 + tot2 + (e23 >> 16)};
      const uint32_t ncand = tot0 + tot1 + tot2 + tot3;
      for (uint32_t win = 0; win < ncand; win += kCandCap) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t mk = m[k], rank = base[k];
          while (mk) {
            const uint32_t bit = __builtin_ctz(mk);
            mk &= mk - 1;
            if (rank - win < (uint32_t)kCandCap) cl[rank - win] = (uint16_t)(1024 * k + 16 * lane + bit);
            ++rank;
          }
        }
        wave_lds_sync();
        const uint32_t nwin = ncand - win < (uint32_t)kCandCap ? ncand - win : (uint32_t)kCandCap;
        // 4. walk up to 64 candidates at once, then apply the greedy chain rule
        for (uint32_t i0 = 0; i0 < nwin; i0 += 64) {
          const uint32_t j = i0 + lane;
          uint32_t coff = 0, le = 0;
          uint64_t len = 0;
          if (j < nwin) {
            coff = cl[j];
            if (P.ablate != 3) len = walk<0>(T, w, ts + coff, le, ovf);  // 3: benchmarking, no walks
          }
          const uint64_t c = ts + coff;
          const bool vm = len != 0 && c >= x;
          // match ends relative to the tile start (clamped; only order matters)
          const uint64_t endr = c + len - ts;
          const uint32_t er = vm ? (endr > 0xffffffffull ? 0xffffffffu : (uint32_t)endr) : 0u;
          const uint32_t xr = x > ts ? (x - ts > 0xffffffffull ? 0xffffffffu : (uint32_t)(x - ts)) : 0u;
          const uint32_t pm = umax32(dpp_prev_lane(dpp_scan_max(er)), xr);
          bool kept = vm && coff >= pm;
          if (__ballot(vm && coff < pm)) {
            // overlapping candidate matches: exact sequential greedy pass
            uint64_t xx = x;
            kept = false;
            for (int i = 0; i < 64; ++i) {
              const uint64_t ci = __shfl(c, i, 64);
              const uint64_t ei = __shfl(vm ? c + len : 0ull, i, 64);
              if (ei != 0 && ci >= xx) {
                if (lane == i) kept = true;
                xx = ei;
              }
            }
          }
          const uint64_t kb = __ballot(kept);
          if (kb) {
            if constexpr (WRITE) {
              WriteEm we{widx + lanes_below(kb), P.out_capacity, P.out_start, P.out_len, P.out_cap};
              if (kept) we.put(C, c, len, le, +1);
              wover |= we.overflow;
              widx += __popcll(kb);
            } else {
              if (kept) acc.put(C, c, len, le, +1);
            }
            // kept matches are disjoint and ordered: the last one ends last
            const int ll = 63 - __builtin_clzll(kb);
            const uint64_t e = c + len;
            const uint32_t ehi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(e >> 32), ll);
            const uint32_t elo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)e, ll);  // readlane is int: no sign extension
            x = ((uint64_t)ehi << 32) | elo;
          }
        }
        wave_lds_sync();  // the list is rewritten by the next window
      }
    }
    const uint64_t tend = ts + kWaveTile < whi ? ts + kWaveTile : whi;
    x = x > tend ? x : tend;
    wave_lds_sync();  // reads of this tile precede the next tile's stores
  }
  if (tb == te) x = wlo;

  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (wover) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  if constexpr (!WRITE) {
    const uint64_t c = wave_sum(acc.cnt), d = wave_sum(acc.dg), dc = wave_sum(acc.dc);
    if (lane == 0) {
      BlockRec rec;
      rec.entry = wlo;
      rec.exit = x;
      rec.cnt = c;
      rec.dg = d;
      rec.dc = dc;
      rec.pad0 = rec.pad1 = rec.pad2 = 0;
      P.recs[gw] = rec;
    }
  }
}

// ---------------------------------------------------------------- launchers
size_t sparse_smem_bytes(uint32_t ntrans_pad, uint32_t nstates)
{
  size_t b = (size_t)kSpWaves * (kWaveTile + 2 * kCandCap) + 2 * (size_t)ntrans_pad + 4 * (size_t)nstates;
  return (b + 15) & ~size_t(15);
}

namespace {

template <bool WRITE>
hipError_t sparse_one(const ScanParams& P, size_t smem, hipStream_t stream)
{
  static size_t attr_smem = 65536;
  if (smem > attr_smem) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sparse_kernel<WRITE>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_smem = smem;
  }
  hipLaunchKernelGGL((sparse_kernel<WRITE>), dim3(P.grid), dim3(kSpWaves * 64), smem, stream, P);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_sparse(const ScanParams& P, bool write, size_t smem, hipStream_t stream)
{
  return write ? sparse_one<true>(P, smem, stream) : sparse_one<false>(P, smem, stream);
}

hipError_t sparse_occupancy(const ScanParams& P, size_t smem, int* n)
{
  (void)P;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, sparse_kernel<false>, kSpWaves * 64, smem);
}

}  // namespace ugpu
