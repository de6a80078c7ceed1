// scan_kernels.hip -- CDNA4 (gfx950) kernels of the FIND engine.  See
// scan_kernels.hpp for the chain/stitch scheme.
//
// Reference hot loops replaced here:
//   * needle prefilter simd_advance_pattern_pinN_*_avx2 (lib/matcher_avx2.cpp:
//     303-799) / simd_advance_string_* (lib/matcher_avx512bw.cpp:281-463):
//     per-lane SWAR test of the segment's 64 staged bytes against the DFA's
//     first/second-byte terms -> 64-bit candidate mask (filter_mask);
//   * DFA opcode interpreter (lib/matcher.cpp:125-546): one dependent LDS
//     lookup per byte in the flattened table (walk);
//   * FIND restart/accept logic (lib/matcher.cpp:621-746): chain_step.
#include "device_common.hpp"

namespace ugpu {

// ---------------------------------------------------------------- scan kernel
template <int FMT, int FC, bool WRITE>
__global__ __launch_bounds__(kBlock) void scan_kernel(ScanParams P)
{
  constexpr bool FILT = FC != 0;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint64_t* ex = reinterpret_cast<uint64_t*>(smem + kTile + kHalo);
  uint64_t* red = ex + kBlock;  // 3 * 4 u64 reduction scratch
  uint16_t* ltrans = reinterpret_cast<uint16_t*>(red + 16);
  uint8_t* lcls = reinterpret_cast<uint8_t*>(ltrans + P.ntrans_pad);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;

  // stage the transition table (and class map) once per block
  {
    const uint4* src = reinterpret_cast<const uint4*>(P.trans);
    uint4* dst = reinterpret_cast<uint4*>(ltrans);
    for (uint32_t i = tid; i < P.ntrans_pad / 8; i += kBlock) dst[i] = src[i];
    if constexpr (FMT == 1) {
      if (tid < 16) reinterpret_cast<uint4*>(lcls)[tid] = reinterpret_cast<const uint4*>(P.cls)[tid];
    }
  }
  const Tab<FMT> T{ltrans, lcls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  static_assert(!FILT, "prefiltered patterns use sparse_kernel.hip");

  const uint64_t b = blockIdx.x;
  uint64_t tb = P.t0 + b * P.tpb;
  uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
  if (tb > te) tb = te;
  const uint64_t blo = clampu(tb * kTile, P.lo, P.hi);
  const uint64_t bhi = clampu(te * kTile, P.lo, P.hi);
  uint64_t x0 = WRITE ? P.entries[b] : blo;

  Win w;
  w.lds = tile;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0;
  CountEm tot;
  uint64_t wbase = WRITE ? P.out_base[b] : 0;
  uint32_t wover = 0;

  uint4 pf[4], ph = make_uint4(0, 0, 0, 0);
  auto prefetch = [&](uint64_t t) {
    const uint64_t ts = t * kTile;
#pragma unroll
    for (int k = 0; k < 4; ++k) pf[k] = load_chunk(P.g, ts + 16ull * (tid + k * kBlock), P.rend);
    if (tid < kHalo / 16) ph = load_chunk(P.g, ts + kTile + 16ull * tid, P.rend);
  };
  if (tb < te) prefetch(tb);

  for (uint64_t t = tb; t < te; ++t) {
    const uint64_t ts = t * kTile;
    __syncthreads();  // previous tile fully consumed
    {
      uint4* d = reinterpret_cast<uint4*>(tile);
#pragma unroll
      for (int k = 0; k < 4; ++k) d[tid + k * kBlock] = pf[k];
      if (tid < kHalo / 16) d[kTile / 16 + tid] = ph;
    }
    __syncthreads();
    if (t + 1 < te) prefetch(t + 1);

    w.base = ts;
    w.lend = ts + kTile + kHalo;
    const uint64_t sa = ts + (uint64_t)tid * kSeg;
    const uint64_t s = clampu(sa, blo, bhi);
    const uint64_t e = clampu(sa + kSeg, blo, bhi);
    uint64_t mask = 0;
    if (P.ablate == 1) {  // keep x0 consistent so fix_kernel has nothing to stitch
      tot.cnt += tile[tid];
      x0 = clampu(ts + kTile, blo, bhi);
      continue;
    }
    if (P.ablate == 2) {
      tot.cnt += __popcll(mask);
      x0 = clampu(ts + kTile, blo, bhi);
      continue;
    }
    uint64_t x = (tid == 0) ? x0 : s;
    CountEm la;
    const uint64_t xe = run_seg<FMT, FILT>(T, w, C, x, sa, e, mask, la, ovf);
    // The true chain enters lane k at lane k-1's exit.  It differs from the
    // speculative entry s_k only where some lane's chain left its segment past
    // the segment end (a match crossing the boundary).
    if (__syncthreads_or(xe > e)) {
      ex[tid] = xe;
      // resolve the true chain entry of every lane (rounds propagate left->right)
      for (;;) {
        __syncthreads();
        const uint64_t nx = (tid == 0) ? x0 : ex[tid - 1];
        const bool ch = nx != x;
        __syncthreads();
        if (ch) {
          uint64_t ne;
          if (!merge<FMT, FILT>(T, w, C, x, nx, sa, e, mask, la, ne, ovf)) ex[tid] = ne;
          x = nx;
        }
        if (!__syncthreads_or(ch)) break;
      }
      x0 = ex[kBlock - 1];
    } else {
      x0 = clampu(ts + kTile, blo, bhi);  // == exit of the last lane
    }
    if constexpr (WRITE) {
      // exclusive prefix of the lanes' match counts, then re-walk and store
      uint64_t v = la.cnt, incl = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      if (lane == 63) red[wid] = incl;
      __syncthreads();
      uint64_t off = 0, all = 0;
#pragma unroll
      for (int k = 0; k < kBlock / 64; ++k) {
        off += (k < wid) ? red[k] : 0;
        all += red[k];
      }
      WriteEm we{wbase + off + incl - v, P.out_capacity, P.out_start, P.out_len, P.out_cap};
      run_seg<FMT, FILT>(T, w, C, x, sa, e, mask, we, ovf);
      wover |= we.overflow;
      wbase += all;
      __syncthreads();  // red reused next tile
    } else {
      tot.cnt += la.cnt;
      tot.dg += la.dg;
      tot.dc += la.dc;
    }
  }

  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (wover) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  if constexpr (!WRITE) {
    const uint64_t c = wave_sum(tot.cnt), d = wave_sum(tot.dg), dc = wave_sum(tot.dc);
    __syncthreads();
    if (lane == 0) {
      red[wid] = c;
      red[4 + wid] = d;
      red[8 + wid] = dc;
    }
    __syncthreads();
    if (tid == 0) {
      BlockRec r;
      r.entry = blo;
      r.exit = x0;
      r.cnt = red[0] + red[1] + red[2] + red[3];
      r.dg = red[4] + red[5] + red[6] + red[7];
      r.dc = red[8] + red[9] + red[10] + red[11];
      r.pad0 = r.pad1 = r.pad2 = 0;
      P.recs[b] = r;
    }
  }
}

// ---------------------------------------------------------------- fix kernel
// One workgroup re-enters every block whose speculative entry differs from its
// predecessor's exit (merge over the block's byte range, bytes from global),
// repeating until no exit changes; then reduces the totals and produces the
// exact block entries and output bases for the OFFSETS pass.
template <int FMT>
__global__ __launch_bounds__(kFixThreads) void fix_kernel(ScanParams P)
{
  __shared__ uint64_t ent[kMaxRec], exi[kMaxRec];
  __shared__ uint64_t wred[3][kFixThreads / 64];
  __shared__ uint64_t wscan[kFixThreads / 64];
  constexpr int PER = kMaxRec / kFixThreads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = (int)P.nrec;
  const Tab<FMT> T{P.trans, P.cls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  Win w;
  w.lds = nullptr;
  w.base = 0;
  w.lend = 0;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0;

  uint64_t cnt[PER], dg[PER], dc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = tid * PER + j;
    if (b < G) {
      BlockRec r = P.recs[b];
      ent[b] = r.entry;
      exi[b] = r.exit;
      cnt[j] = r.cnt;
      dg[j] = r.dg;
      dc[j] = r.dc;
    } else {
      cnt[j] = dg[j] = dc[j] = 0;
    }
  }
  uint32_t rounds = 0;
  for (;;) {
    __syncthreads();
    uint64_t nx[PER];
    bool ch[PER], any = false;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int b = tid * PER + j;
      ch[j] = false;
      if (b > 0 && b < G) {
        nx[j] = exi[b - 1];
        ch[j] = nx[j] != ent[b];
        any |= ch[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (!ch[j]) continue;
      const uint64_t b = tid * PER + j;
      uint64_t tb = P.t0 + b * P.tpb;
      uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
      if (tb > te) tb = te;
      const uint64_t bhi = clampu(te * P.unit, P.lo, P.hi);
      CountEm d;
      uint64_t ne;
      if (!merge<FMT, 0>(T, w, C, ent[b], nx[j], 0, bhi, 0, d, ne, ovf)) exi[b] = ne;
      ent[b] = nx[j];
      cnt[j] += d.cnt;
      dg[j] += d.dg;
      dc[j] += d.dc;
    }
    if (!__syncthreads_or(any)) break;
    ++rounds;
  }
  // totals + exclusive scan of block counts
  uint64_t mc = 0, md = 0, mdc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    mc += cnt[j];
    md += dg[j];
    mdc += dc[j];
  }
  uint64_t incl = mc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const uint64_t sd = wave_sum(md), sdc = wave_sum(mdc);
  if (lane == 63) wscan[wid] = incl;
  if (lane == 0) {
    wred[1][wid] = sd;
    wred[2][wid] = sdc;
  }
  __syncthreads();
  uint64_t off = 0;
  for (int k = 0; k < wid; ++k) off += wscan[k];
  uint64_t run = off + incl - mc;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = tid * PER + j;
    if (b < G) {
      P.out_base_out[b] = run;
      P.entries_out[b] = ent[b];
      run += cnt[j];
    }
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (tid == 0) {
    uint64_t c = 0, d = 0, e = 0;
    for (int k = 0; k < kFixThreads / 64; ++k) {
      c += wscan[k];
      d += wred[1][k];
      e += wred[2][k];
    }
    DevTotals* t = P.totals;
    t->count = c;
    t->digest = d;
    t->dcap = e;
    t->entry = ent[0];
    t->exit = exi[G - 1];
    t->rounds = rounds;
  }
}

// Shard-boundary stitch (multi-GPU): re-enter [lo, hi) at new_entry.
template <int FMT>
__global__ void chain_fix_kernel(ScanParams P, uint64_t old_entry, uint64_t new_entry)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const Tab<FMT> T{P.trans, P.cls, P.start, P.accb};
  const Ctx C{P.caps, P.log_row, P.delta};
  Win w;
  w.lds = nullptr;
  w.base = 0;
  w.lend = 0;
  w.g = P.g;
  w.rend = P.rend;
  w.eof = P.at_eof;
  uint32_t ovf = 0;
  CountEm d;
  uint64_t ne = 0;
  bool met = merge<FMT, 0>(T, w, C, old_entry, new_entry, 0, P.hi, 0, d, ne, ovf);
  DevTotals* t = P.totals;
  t->count = d.cnt;
  t->digest = d.dg;
  t->dcap = d.dc;
  t->entry = new_entry;
  t->exit = met ? ~0ull : ne;  // ~0 = exit unchanged
  t->flags = ovf ? UGPU_FLAG_HALO : 0;
  t->rounds = met ? 1 : 0;
}

// ---------------------------------------------------------------- launchers
template <int FMT, int FC, bool WRITE>
static hipError_t launch_one(const ScanParams& P, size_t smem, hipStream_t stream)
{
  static size_t attr_smem = 65536;
  if (smem > attr_smem) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&scan_kernel<FMT, FC, WRITE>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_smem = smem;
  }
  hipLaunchKernelGGL((scan_kernel<FMT, FC, WRITE>), dim3(P.grid), dim3(kBlock), smem, stream, P);
  return hipGetLastError();
}

hipError_t launch_scan(const ScanParams& P, uint32_t format, bool filter, bool write, size_t smem,
                       hipStream_t stream)
{
  (void)filter;  // prefiltered patterns run sparse_kernel
  if (format == 0) return write ? launch_one<0, 0, true>(P, smem, stream) : launch_one<0, 0, false>(P, smem, stream);
  return write ? launch_one<1, 0, true>(P, smem, stream) : launch_one<1, 0, false>(P, smem, stream);
}

hipError_t launch_fix(const ScanParams& P, uint32_t format, hipStream_t stream)
{
  if (format == 0)
    hipLaunchKernelGGL(fix_kernel<0>, dim3(1), dim3(kFixThreads), 0, stream, P);
  else
    hipLaunchKernelGGL(fix_kernel<1>, dim3(1), dim3(kFixThreads), 0, stream, P);
  return hipGetLastError();
}

hipError_t launch_chain_fix(const ScanParams& P, uint32_t format, uint64_t old_entry, uint64_t new_entry,
                            hipStream_t stream)
{
  if (format == 0)
    hipLaunchKernelGGL(chain_fix_kernel<0>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  else
    hipLaunchKernelGGL(chain_fix_kernel<1>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  return hipGetLastError();
}

template <int FMT, int FC>
static hipError_t occ_one(size_t smem, int* n)
{
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, scan_kernel<FMT, FC, false>, kBlock, smem);
}

hipError_t scan_occupancy(uint32_t format, bool filter, size_t smem, int* n)
{
  (void)filter;
  if (format == 0) return occ_one<0, 0>(smem, n);
  return occ_one<1, 0>(smem, n);
}

size_t scan_smem_bytes(uint32_t ntrans_pad, uint32_t format)
{
  size_t b = kTile + kHalo + sizeof(uint64_t) * (kBlock + 16) + sizeof(uint16_t) * ntrans_pad;
  if (format == 1) b += 256;
  return (b + 15) & ~size_t(15);
}

}  // namespace ugpu
