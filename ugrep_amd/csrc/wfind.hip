// wfind.hip -- FIND with Matcher option W (ugrep -w), SURVEY §8 a10 / §8f row 4.
//
// Option W changes two things in the reference's FIND loop
// (lib/matcher.cpp:107, :142, :208, :664): a walk starts at p only where
// at_wb() holds, and a TAKE counts only where at_we() holds at the match end
// (include/reflex/matcher.h:1194-1237).  Both predicates look at up to four
// bytes around a position and at the Unicode Word table, so they do not fit the
// transducer kernels' one-lookup-per-byte steps.  This kernel runs the exact W
// chain (walk<FMT, true>, device_common.hpp):
//
//   * one chain record per wave; its range is cut into 64 lane segments;
//   * every lane walks its segment's chain speculatively from the segment
//     start, then the lanes are stitched in rounds: a lane whose entry differs
//     from its predecessor's exit re-walks with merge() (two chains in lock
//     step until they meet) -- word text resyncs within a word, so one round;
//   * fix_kernel stitches the wave records the same way;
//   * the OFFSETS pass repeats the lane stitch from the record's exact entry,
//     scans the lane counts into output bases and re-walks, writing records.
//
// The tables (transitions, accept indices, classes, Word ranges) are staged in
// LDS once per workgroup of kWWaves records.  Bound: one dependent global byte
// read plus one LDS table lookup per step along one chain per lane; see
// DESIGN.md §3.8.
#include "device_common.hpp"

namespace ugpu {

namespace {

constexpr uint32_t kWUnit = 4096;   // bytes per tile (records hold whole tiles)
#ifndef UGPU_WF_WAVES
#define UGPU_WF_WAVES 16
#endif
constexpr int kWWaves = UGPU_WF_WAVES;  // waves (records) per workgroup: one staged table copy

// LDS image: transitions (u16, ntrans_pad), accept indices (u32 per state;
// mode kWalkCtx: acap, P.acap_n entries), the per-state acap rows of word
// boundary tables (u32, nmap), Word ranges (2 x u32 each), class bytes (256)
__host__ __device__ inline size_t wfind_smem(uint32_t ntrans_pad, uint32_t nwtab, uint32_t nacap, uint32_t nmap)
{
  return 2 * (size_t)ntrans_pad + 4 * ((size_t)nacap + nmap) + 8 * (size_t)nwtab + 256;
}

// M: kWalkWord (option W) or kWalkCtx (line anchors / option N): the same
// exact chain machinery, with that mode's walk rules
template <int FMT, bool WRITE, int M>
__global__ __launch_bounds__(kWWaves * 64) void wfind_kernel(ScanParams P)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  const uint32_t ncaps = M == kWalkCtx ? P.acap_n : P.nstates;
  const uint32_t nmap = M == kWalkCtx && P.ctx_word ? P.nstates : 0u;
  const uint32_t nwt = M == kWalkCtx && !P.ctx_word ? 0u : P.nwtab;
  {
    // stage the tables once per workgroup (the walks look them up per byte)
    uint16_t* tr = reinterpret_cast<uint16_t*>(wsm);
    uint32_t* cp = reinterpret_cast<uint32_t*>(wsm + 2 * (size_t)P.ntrans_pad);
    uint32_t* wt = cp + ncaps + nmap;
    uint8_t* cl = reinterpret_cast<uint8_t*>(wt + 2 * nwt);
    const uint32_t* caps = M == kWalkCtx ? P.acap : P.caps;
    if constexpr (FMT != 2)  // (wide tables stay in global memory)
      for (uint32_t i = threadIdx.x; i < P.ntrans_pad; i += blockDim.x) tr[i] = P.trans[i];
    for (uint32_t i = threadIdx.x; i < ncaps; i += blockDim.x) cp[i] = caps[i];
    for (uint32_t i = threadIdx.x; i < nmap; i += blockDim.x) cp[ncaps + i] = P.amap[i];
    for (uint32_t i = threadIdx.x; i < 2 * nwt; i += blockDim.x) wt[i] = P.wtab[i];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) cl[i] = P.cls[i];
    __syncthreads();
  }
  const uint16_t* s_trans = reinterpret_cast<const uint16_t*>(wsm);
  const uint32_t* s_caps = reinterpret_cast<const uint32_t*>(wsm + 2 * (size_t)P.ntrans_pad);
  const uint32_t* s_wtab = s_caps + ncaps + nmap;
  const uint8_t* s_cls = reinterpret_cast<const uint8_t*>(s_wtab + 2 * nwt);
  const int lane = threadIdx.x & 63;
  const uint64_t r = (uint64_t)blockIdx.x * kWWaves + (threadIdx.x >> 6);
  if (r >= P.nrec) return;  // wave-uniform
  uint64_t tb = P.t0 + r * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t wlo = clampu(tb * P.unit, P.lo, P.hi);
  const uint64_t whi = clampu(te * P.unit, P.lo, P.hi);
  const uint64_t seg = (whi - wlo + 63) / 64;
  const uint64_t slo = wlo + seg * lane < whi ? wlo + seg * lane : whi;
  const uint64_t shi = slo + seg < whi ? slo + seg : whi;
  Tab<FMT> T;
  if constexpr (FMT == 2)
    T = Tab<2>{P.trans32, s_cls, P.start, P.accb};
  else
    T = Tab<FMT>{s_trans, s_cls, P.start, P.accb};
  const Ctx C{s_caps, M == kWalkCtx ? 0u : P.log_row, P.delta};
  Win w = win_of(P);
  w.wtab = s_wtab;
  w.acap = s_caps;
  w.amap = s_caps + ncaps;
  uint32_t ovf = 0;

  // speculative lane chains (lane 0 enters at the record's entry)
  uint64_t ent = (WRITE && lane == 0) ? P.entries[r] : slo;
  CountEm acc;
  uint64_t p = ent;
  while (p < shi) p = chain_step<FMT, CountEm, M>(T, w, C, p, acc, +1, ovf);
  uint64_t exi = p;  // first chain position >= shi (the entry itself when it lies beyond)
  // lane stitch rounds (a wrong entry moves one lane per round; chains that do
  // not resynchronise give up after 24 rounds: UGPU_FLAG_BUDGET, and the host
  // resolves the range with the forest FIND, forest.hip)
  for (int round = 0;;) {
    uint64_t nx = __shfl_up(exi, 1, 64);
    const bool ch = lane > 0 && nx != ent;
    if (!__ballot(ch)) break;
    if (__ballot(ch && ent < shi) && ++round > 24) {
      if (lane == 0) atomicOr(P.flags, UGPU_FLAG_BUDGET);
      break;
    }
    if (ch) {
      uint64_t ne;
      if (!merge<FMT, M>(T, w, C, ent, nx, shi, acc, ne, ovf)) exi = ne;
      ent = nx;
    }
  }
  if constexpr (WRITE) {
    // exclusive scan of lane counts -> output index of the lane's first match
    uint64_t incl = acc.cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    WriteEm em{P.out_base[r] + incl - acc.cnt, P.out_capacity, P.out_start, P.out_len, P.out_cap};
    uint64_t q = ent;
    while (q < shi) q = chain_step<FMT, WriteEm, M>(T, w, C, q, em, +1, ovf);
    if (em.overflow) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  } else {
    const uint64_t c = wave_sum(acc.cnt), d = wave_sum(acc.dg), dc = wave_sum(acc.dc);
    const uint64_t x = __shfl(exi, 63, 64);
    if (lane == 0) {
      BlockRec rec;
      rec.entry = wlo;
      rec.exit = whi > wlo ? (x > whi ? x : whi) : wlo;
      rec.cnt = c;
      rec.dg = d;
      rec.dc = dc;
      rec.pad0 = rec.pad1 = rec.pad2 = 0;
      P.recs[r] = rec;
    }
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
}

template <int FMT, bool WRITE, int M>
hipError_t wfind_one(const ScanParams& P, hipStream_t stream)
{
  const size_t smem = wfind_smem(P.ntrans_pad, P.nwtab, M == kWalkCtx ? P.acap_n : P.nstates,
                                 M == kWalkCtx && P.ctx_word ? P.nstates : 0u);
  static size_t attr_smem = 65536;
  if (smem > attr_smem) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wfind_kernel<FMT, WRITE, M>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_smem = smem;
  }
  hipLaunchKernelGGL((wfind_kernel<FMT, WRITE, M>), dim3(P.grid), dim3(kWWaves * 64), smem, stream, P);
  return hipGetLastError();
}

template <int M>
hipError_t wfind_mode(const ScanParams& P, uint32_t format, bool write, hipStream_t stream)
{
  if (format == 0) return write ? wfind_one<0, true, M>(P, stream) : wfind_one<0, false, M>(P, stream);
  if (format == 1) return write ? wfind_one<1, true, M>(P, stream) : wfind_one<1, false, M>(P, stream);
  return write ? wfind_one<2, true, M>(P, stream) : wfind_one<2, false, M>(P, stream);
}

}  // namespace

uint32_t wfind_unit() { return kWUnit; }
uint32_t wfind_waves() { return kWWaves; }
size_t wfind_smem_bytes(uint32_t ntrans_pad, uint32_t nstates, uint32_t nwtab, uint32_t nacap, uint32_t nmap)
{
  (void)nstates;
  return wfind_smem(ntrans_pad, nwtab, nacap, nmap);
}

// option W (P.wtab), line anchors / option N (P.acap), or neither (wide
// tables: the plain walk over transitions in global memory)
hipError_t launch_wfind(const ScanParams& P, uint32_t format, bool write, hipStream_t stream)
{
  if (P.acap) return wfind_mode<kWalkCtx>(P, format, write, stream);
  if (P.look) return wfind_mode<kWalkLook>(P, format, write, stream);  // (with or without option W)
  if (P.wtab) return wfind_mode<kWalkWord>(P, format, write, stream);
  return wfind_mode<kWalkPlain>(P, format, write, stream);
}

}  // namespace ugpu
