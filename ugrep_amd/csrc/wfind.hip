// wfind.hip -- FIND with Matcher option W (ugrep -w), SURVEY §8 a10 / §8f row 4.
//
// Option W changes two things in the reference's FIND loop
// (lib/matcher.cpp:107, :142, :208, :664): a walk starts at p only where
// at_wb() holds, and a TAKE counts only where at_we() holds at the match end
// (include/reflex/matcher.h:1194-1237).  Both predicates look at up to four
// bytes around a position and at the Unicode Word table, so they do not fit the
// transducer kernels' one-lookup-per-byte steps.  This kernel runs the exact W
// chain (walk<FMT, true>, device_common.hpp) with one chain record per lane:
// lane r walks the chain of its byte range from the range start
// (speculatively), and fix_kernel stitches the records exactly as for the
// dense kernel's wave records.  The OFFSETS pass re-walks each range from its
// exact entry and writes the records at the range's output base.
//
// Bound: dependent global byte reads along one chain per lane (latency, not
// HBM bandwidth); word text resyncs the chains within a word, so fix_kernel
// needs one round.
#include "device_common.hpp"

namespace ugpu {

namespace {

constexpr uint32_t kWUnit = 4096;  // bytes per tile (records hold whole tiles)

template <int FMT, bool WRITE>
__global__ __launch_bounds__(kWfindLanes) void wfind_kernel(ScanParams P)
{
  const uint64_t r = (uint64_t)blockIdx.x * kWfindLanes + threadIdx.x;
  if (r >= P.nrec) return;
  uint64_t tb = P.t0 + r * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t blo = clampu(tb * P.unit, P.lo, P.hi);
  const uint64_t bhi = clampu(te * P.unit, P.lo, P.hi);
  const Tab<FMT> T{P.trans, P.cls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  Win w;
  w.lds = nullptr;
  w.base = 0;
  w.lend = 0;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  w.wtab = P.wtab;
  w.nwtab = P.nwtab;
  w.bob = P.bob;
  uint32_t ovf = 0;
  uint64_t p = WRITE ? P.entries[r] : blo;
  if constexpr (WRITE) {
    WriteEm em{P.out_base[r], P.out_capacity, P.out_start, P.out_len, P.out_cap};
    while (p < bhi) p = chain_step<FMT, WriteEm, true>(T, w, C, p, em, +1, ovf);
    if (em.overflow) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  } else {
    CountEm em;
    while (p < bhi) p = chain_step<FMT, CountEm, true>(T, w, C, p, em, +1, ovf);
    BlockRec rec;
    rec.entry = blo;
    rec.exit = bhi > blo ? p : blo;
    rec.cnt = em.cnt;
    rec.dg = em.dg;
    rec.dc = em.dc;
    rec.pad0 = rec.pad1 = rec.pad2 = 0;
    P.recs[r] = rec;
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
}

template <int FMT, bool WRITE>
hipError_t wfind_one(const ScanParams& P, hipStream_t stream)
{
  hipLaunchKernelGGL((wfind_kernel<FMT, WRITE>), dim3(P.grid), dim3(kWfindLanes), 0, stream, P);
  return hipGetLastError();
}

}  // namespace

uint32_t wfind_unit() { return kWUnit; }

hipError_t launch_wfind(const ScanParams& P, uint32_t format, bool write, hipStream_t stream)
{
  if (format == 0) return write ? wfind_one<0, true>(P, stream) : wfind_one<0, false>(P, stream);
  return write ? wfind_one<1, true>(P, stream) : wfind_one<1, false>(P, stream);
}

}  // namespace ugpu
