// scan_kernels.hip -- chain-record stitching kernels of the FIND engine (see
// scan_kernels.hpp for the chain/stitch scheme).  The scan kernels themselves
// are sparse_kernel.hip (prefiltered patterns) and dense_kernel.hip.
#include "device_common.hpp"

namespace ugpu {


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
  const Tab<FMT> T = tab_global<FMT>(P);
  const Ctx C = P.acap ? Ctx{P.acap, 0u, P.delta} : Ctx{P.caps, P.log_row, P.delta};
  const Win w = win_of(P);
  uint32_t ovf = 0, over = 0;
  // the scan kernel already gave up on these chains (UGPU_FLAG_BUDGET): the host
  // resolves the range with the forest FIND, nothing to stitch
  if (__hip_atomic_load(P.flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & UGPU_FLAG_BUDGET) return;

  uint64_t cnt[PER], dg[PER], dc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = j * kFixThreads + tid;
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
      const int b = j * kFixThreads + tid;
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
      const uint64_t b = (uint64_t)j * kFixThreads + tid;
      uint64_t tb = P.t0 + b * P.tpb;
      uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
      if (tb > te) tb = te;
      const uint64_t bhi = clampu(te * P.unit, P.lo, P.hi);
      CountEm d;
      uint64_t ne;
      const bool met =
          P.acap   ? merge<FMT, kWalkCtx>(T, w, C, ent[b], nx[j], bhi, d, ne, ovf, P.merge_budget, &over)
          : P.wtab ? merge<FMT, kWalkWord>(T, w, C, ent[b], nx[j], bhi, d, ne, ovf, P.merge_budget, &over)
                   : merge<FMT>(T, w, C, ent[b], nx[j], bhi, d, ne, ovf, P.merge_budget, &over);
      if (!met) exi[b] = ne;
      ent[b] = nx[j];
      cnt[j] += d.cnt;
      dg[j] += d.dg;
      dc[j] += d.dc;
    }
    if (!__syncthreads_or(any)) break;
    if (__syncthreads_or(over) || ++rounds >= P.max_rounds) {  // chains that do not resynchronise
      over = 1;
      break;
    }
  }
  // totals + exclusive scan of block counts (block order b = j * kFixThreads + tid:
  // one workgroup scan per j, carried across j)
  uint64_t md = 0, mdc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    md += dg[j];
    mdc += dc[j];
  }
  const uint64_t sd = wave_sum(md), sdc = wave_sum(mdc);
  if (lane == 0) {
    wred[1][wid] = sd;
    wred[2][wid] = sdc;
  }
  uint64_t carry = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    uint64_t incl = cnt[j];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) wscan[wid] = incl;
    __syncthreads();
    uint64_t off = carry, tot = 0;
    for (int k = 0; k < kFixThreads / 64; ++k) {
      if (k < wid) off += wscan[k];
      tot += wscan[k];
    }
    const int b = j * kFixThreads + tid;
    if (b < G) {
      P.out_base_out[b] = off + incl - cnt[j];
      P.entries_out[b] = ent[b];
    }
    carry += tot;
  }
  if (ovf) atomicOr(P.flags, UGPU_FLAG_HALO);
  if (over && tid == 0) atomicOr(P.flags, UGPU_FLAG_BUDGET);
  __syncthreads();
  if (tid == 0) {
    uint64_t d = 0, e = 0;
    for (int k = 0; k < kFixThreads / 64; ++k) {
      d += wred[1][k];
      e += wred[2][k];
    }
    const uint64_t c = carry;
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
  const Tab<FMT> T = tab_global<FMT>(P);
  const Ctx C = P.acap ? Ctx{P.acap, 0u, P.delta} : Ctx{P.caps, P.log_row, P.delta};
  // (option W: at_wb reads the bytes before a walk start; the caller's buffer
  // holds the code point before lo -- shard and stream prefixes, engine.hip)
  const Win w = win_of(P);
  uint32_t ovf = 0, over = 0;
  CountEm d;
  uint64_t ne = 0;
  bool met = P.acap   ? merge<FMT, kWalkCtx>(T, w, C, old_entry, new_entry, P.hi, d, ne, ovf, P.merge_budget, &over)
             : P.wtab ? merge<FMT, kWalkWord>(T, w, C, old_entry, new_entry, P.hi, d, ne, ovf, P.merge_budget, &over)
                      : merge<FMT>(T, w, C, old_entry, new_entry, P.hi, d, ne, ovf, P.merge_budget, &over);
  DevTotals* t = P.totals;
  t->count = d.cnt;
  t->digest = d.dg;
  t->dcap = d.dc;
  t->entry = new_entry;
  t->exit = met ? ~0ull : ne;  // ~0 = exit unchanged
  t->flags = (ovf ? UGPU_FLAG_HALO : 0) | (over ? UGPU_FLAG_BUDGET : 0);
  t->rounds = met ? 1 : 0;
}

// Host-path record packing (ugpu_find_records): n records (u64 start, u32
// len, u32 cap) of one chunk into u32 start - base, u16 len and (caps != 0)
// u16 cap; a len or cap >= 0xFFFF is written as 0xFFFF and its record's
// (index, len | cap << 32) appended to esc through a counter (rare: the host
// sorts them).  One record per thread, fully coalesced.
//
// dense (one accept index, many records per byte -- identifiers, words): u8
// gap from the previous record's end (the chunk base for the first) and u8
// len, 2 B per record; a gap or len >= 0xFF is written as 0xFF and the
// record's (index, start - base | len << 32) escapes.
__global__ void pack_records_kernel(const uint64_t* start, const uint32_t* len, const uint32_t* cap, uint64_t n,
                                    uint64_t base, uint8_t* out, int caps, int dense, uint64_t* esc, uint32_t* nesc)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (dense) {
    const uint64_t s = start[i] - base;
    const uint32_t l = len[i];
    const uint64_t pe = i ? start[i - 1] - base + len[i - 1] : 0;  // (FIND matches do not overlap: s >= pe)
    const uint64_t g = s - pe;
    const bool ok = g < 0xFFu && l < 0xFFu;
    out[i] = (uint8_t)(ok ? g : 0xFFu);
    out[n + i] = (uint8_t)(ok ? l : 0xFFu);
    if (!ok) {
      const uint32_t k = atomicAdd(nesc, 1u);
      esc[2 * k] = i;
      esc[2 * k + 1] = (s & 0xffffffffull) | ((uint64_t)l << 32);
    }
    return;
  }
  uint32_t* o_start = reinterpret_cast<uint32_t*>(out);
  uint16_t* o_len = reinterpret_cast<uint16_t*>(out + 4 * n);
  uint16_t* o_cap = reinterpret_cast<uint16_t*>(out + 6 * n);
  const uint32_t l = len[i], c = caps ? cap[i] : 0u;
  o_start[i] = (uint32_t)(start[i] - base);
  o_len[i] = (uint16_t)(l >= 0xFFFFu ? 0xFFFFu : l);
  if (caps) o_cap[i] = (uint16_t)(c >= 0xFFFFu ? 0xFFFFu : c);
  if (l >= 0xFFFFu || c >= 0xFFFFu) {
    const uint32_t k = atomicAdd(nesc, 1u);
    esc[2 * k] = i;
    esc[2 * k + 1] = (uint64_t)l | ((uint64_t)c << 32);
  }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_pack_records(const uint64_t* start, const uint32_t* len, const uint32_t* cap, uint64_t n,
                               uint64_t base, uint8_t* out, int caps, int dense, uint64_t* esc, uint32_t* nesc,
                               hipStream_t stream)
{
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(pack_records_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, start, len, cap, n, base,
                     out, caps, dense, esc, nesc);
  return hipGetLastError();
}

hipError_t launch_fix(const ScanParams& P, uint32_t format, hipStream_t stream)
{
  if (format == 0)
    hipLaunchKernelGGL(fix_kernel<0>, dim3(1), dim3(kFixThreads), 0, stream, P);
  else if (format == 1)
    hipLaunchKernelGGL(fix_kernel<1>, dim3(1), dim3(kFixThreads), 0, stream, P);
  else
    hipLaunchKernelGGL(fix_kernel<2>, dim3(1), dim3(kFixThreads), 0, stream, P);
  return hipGetLastError();
}

hipError_t launch_chain_fix(const ScanParams& P, uint32_t format, uint64_t old_entry, uint64_t new_entry,
                            hipStream_t stream)
{
  if (format == 0)
    hipLaunchKernelGGL(chain_fix_kernel<0>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  else if (format == 1)
    hipLaunchKernelGGL(chain_fix_kernel<1>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  else
    hipLaunchKernelGGL(chain_fix_kernel<2>, dim3(1), dim3(64), 0, stream, P, old_entry, new_entry);
  return hipGetLastError();
}

}  // namespace ugpu
