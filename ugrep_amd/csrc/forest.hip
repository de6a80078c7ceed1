// forest.hip -- exact FIND for chains that do not resynchronise.
//
// The FIND loop (lib/matcher.cpp:42-750) moves from a
// chain position p to N(p) = p + (length of the longest match at p, or 1 when
// there is none).  N(p) depends on p alone, so the chain from any entry e is
// the orbit e, N(e), N(N(e)), ... in the forest of parent pointers N (N(p) > p).
// The speculative pipelines (sparse/dense kernels + fix_kernel) guess a piece's
// entry and merge the true chain into the guessed one; when the chains never
// meet (\D\D over text without digits, 'aa' over runs of a) every piece is
// re-walked serially and fix_kernel gives up (UGPU_FLAG_BUDGET).  This path
// needs no such assumption:
//
//   forest_exit_kernel   one workgroup per block of kFB chain positions: N(p)
//                        for every p of the block by the exact walk (bytes and
//                        tables in LDS), then pointer jumping in LDS gives every
//                        p's exit = the first orbit element >= the block end.
//                        Stored per position as (exit - block end), u32.
//   forest_stitch_kernel one wave follows the true chain across blocks: the
//                        entry of block k+1 is the exit of block k from its
//                        entry.  Entries fall in a block's first 64 positions
//                        unless a match is longer than that, so lane j holds
//                        that exit for entry j (the other waves stage the next
//                        blocks' 256-byte heads in LDS) and a step is one
//                        v_readlane; farther entries read their exit from HBM.
//   forest_walk_kernel   every block resolves its FIND chain from its exact
//                        entry the same way one level down (64 sub-blocks, one
//                        lane each): match count and digests (COUNT) or the
//                        match records (WRITE).
//   forest_sum_kernel    totals and per-block output bases (exclusive scan).
//
// The range is processed in chunks of at most kFChunk positions (the exits take
// 4 B per position), the chain entry carried on the device from chunk to chunk.
// A walk's HALO (readable end reached before EOF) counts only on the chain.
#include "device_common.hpp"

namespace ugpu {

namespace {

constexpr int kFB = 4096;          // chain positions per block
constexpr int kFHalo = 256;        // bytes staged past the block end
constexpr int kFThreads = 1024;    // forest_exit_kernel
constexpr int kFStage = kFB + kFHalo;
constexpr int kFGroup = 16;        // stitch: blocks per batch of LDS reads
constexpr int kFWin = 128;         // stitch: blocks per LDS window

// Tables into LDS: trans u16[ntrans_pad] then cls[256]; returns the LDS bytes used.
template <int FMT>
__device__ __forceinline__ Tab<FMT> fstage_tables(const ScanParams& P, uint8_t* smem, int tid, int nthr)
{
  uint16_t* lt = reinterpret_cast<uint16_t*>(smem);
  uint8_t* lc = smem + 2 * (size_t)P.ntrans_pad;
  if constexpr (FMT != 2) {
    const uint4* src = reinterpret_cast<const uint4*>(P.trans);
    uint4* dst = reinterpret_cast<uint4*>(lt);
    for (uint32_t i = tid; i < P.ntrans_pad / 8; i += nthr) dst[i] = src[i];
  }
  if constexpr (FMT != 0)
    for (int i = tid; i < 256; i += nthr) lc[i] = P.cls[i];
  if constexpr (FMT == 2)
    return Tab<2>{P.trans32, lc, P.start, P.accb};  // (wide: transitions from global memory)
  else
    return Tab<FMT>{lt, lc, P.start, P.accb};
}

__device__ __forceinline__ size_t ftab_bytes(const ScanParams& P) { return ((2 * (size_t)P.ntrans_pad + 256) + 15) & ~size_t(15); }

// Stage bytes [bs, min(bs + kFStage, rend)) of the chunk into `dst`; returns the window.
__device__ __forceinline__ Win fstage_bytes(const ScanParams& P, uint8_t* dst, uint64_t bs, int tid, int nthr)
{
  const uint64_t lend = bs + kFStage < P.rend ? bs + kFStage : (P.rend > bs ? P.rend : bs);
  const uint32_t n = (uint32_t)(lend - bs);
  for (uint32_t i = tid; i < n; i += nthr) dst[i] = P.g[bs + i];
  Win w = win_of(P);
  w.lds = dst;
  w.base = bs;
  w.lend = lend;
  return w;
}

constexpr uint32_t kFMatch = 0x80000000u;  // N entry: a match starts here (else N = p + 1)
constexpr uint32_t kFOvf = 0x40000000u;    // N entry: the walk reached the readable end before EOF
constexpr uint32_t kFEmpty = 0x20000000u;  // N entry: the match is empty (option N; N = p + 1)
constexpr uint32_t kFNMask = 0x1fffffffu;  // N entry: N(p) - block start
constexpr int kFSub = 64;                  // forest_walk_kernel: positions per lane sub-block

// N(p) - bs (with the flags above) for the block's positions, and the walk's
// last accepting entry (its row gives the accept index) when LE is set.
// Neighbouring threads walk neighbouring positions: similar bytes, similar rows.
template <int FMT, int W, bool LE>
__device__ __forceinline__ void forest_n(const Tab<FMT>& T, const Win& w, uint64_t bs, uint32_t nb, uint32_t* N,
                                         uint32_t* le_out, int tid, int nthr)
{
  for (uint32_t r = tid; r < nb; r += nthr) {
    uint32_t le, ovf = 0;
    const uint64_t len = walk<FMT, W>(T, w, bs + r, le, ovf);
    // (lookahead under option W: a TAIL without a TAKE is no match, and the
    // chain goes on one past its end, as chain_step)
    const bool tail_only = W == kWalkLook && len && !le;
    uint64_t nx = (uint64_t)r + (len ? len + (tail_only ? 1u : 0u) : 1);
    if (nx > kFNMask) {
      // a match longer than 512 MiB does not fit the entry: fail loudly (the
      // HALO flag: the caller gets UGPU_HALO and, in the drop-in adapter, the
      // CPU matcher) instead of a wrong length
      nx = kFNMask;
      ovf = 1;
    }
    const bool empty = W == kWalkCtx && !len && le && w.nul;  // option N: the empty match at p
    N[r] = (uint32_t)nx | ((len && !tail_only) || empty ? kFMatch : 0u) | (empty ? kFEmpty : 0u) | (ovf ? kFOvf : 0u);
    if constexpr (LE) le_out[r] = le;
  }
}

}  // namespace

template <int FMT, int W>
__global__ __launch_bounds__(kFThreads) void forest_exit_kernel(ScanParams P, ForestArgs A)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t fsm[];
  const int tid = threadIdx.x;
  const Tab<FMT> T = fstage_tables<FMT>(P, fsm, tid, kFThreads);
  uint8_t* bytes = fsm + ftab_bytes(P);
  uint32_t* J = reinterpret_cast<uint32_t*>(bytes + kFStage);
  const uint64_t blk = blockIdx.x;
  const uint64_t bs = A.c_lo + blk * kFB;
  const uint64_t be = bs + kFB < A.c_hi ? bs + kFB : A.c_hi;
  const uint32_t nb = (uint32_t)(be - bs);
  const Win w = fstage_bytes(P, bytes, bs, tid, kFThreads);
  __syncthreads();
  forest_n<FMT, W, false>(T, w, bs, nb, J, nullptr, tid, kFThreads);
  __syncthreads();
  for (uint32_t r = tid; r < nb; r += kFThreads) J[r] &= kFNMask;
  __syncthreads();
  // pointer jumping: J[r] -> the first orbit element >= nb (in-place updates
  // only ever replace a pointer by a later element of the same orbit)
  for (;;) {
    bool ch = false;
    for (uint32_t r = tid; r < nb; r += kFThreads) {
      const uint32_t j = J[r];
      if (j < nb) {
        J[r] = J[j];
        ch = true;
      }
    }
    if (!__syncthreads_or(ch)) break;
  }
  uint32_t* ex = A.ex + blk * kFB;
  for (uint32_t r = tid; r < nb; r += kFThreads) ex[r] = J[r] - nb;
}

// One workgroup.  The chunk entry is *A.entry; on return *A.entry is the chunk
// exit.  Windows of kFWin blocks: waves 1-15 load the next window's first-64
// exits into LDS while wave 0 follows the chain through the current one (per
// block one independent LDS read, then a v_readlane at the entry offset).
__global__ __launch_bounds__(kFThreads) void forest_stitch_kernel(ForestArgs A)
{
  __shared__ uint32_t win[2][kFWin][64];
  __shared__ uint64_t went[2][kFWin];  // block entries, written to HBM by the loader waves
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  auto load_window = [&](uint32_t k0, int buf, int t0, int nt) {
    for (int i = t0; i < kFWin * 64; i += nt) {
      const uint32_t k = k0 + (uint32_t)(i >> 6), j = (uint32_t)(i & 63);
      const uint64_t bs = A.c_lo + (uint64_t)k * kFB;
      win[buf][i >> 6][j] = (k < A.nblk && bs + j < A.c_hi) ? A.ex[(uint64_t)k * kFB + j] : 0u;
    }
  };
  auto flush_entries = [&](uint32_t k0, int buf, int t0, int nt) {
    for (int i = t0; i < kFWin; i += nt)
      if (k0 + i < A.nblk) A.bentry[k0 + i] = went[buf][i];
  };
  load_window(0, 0, tid, kFThreads);
  __syncthreads();
  uint64_t e = *A.entry;
  uint32_t k0 = 0, buf = 0;
  for (; k0 < A.nblk; k0 += kFWin, buf ^= 1) {
    if (wid != 0) {
      if (k0 > 0) flush_entries(k0 - kFWin, buf ^ 1, tid - 64, kFThreads - 64);
      if (k0 + kFWin < A.nblk) load_window(k0 + kFWin, buf ^ 1, tid - 64, kFThreads - 64);
    } else {
      // (no global memory traffic in this loop: a pending store or load would
      // make every step wait for it)
      for (uint32_t g0 = 0; g0 < (uint32_t)kFWin && k0 + g0 < A.nblk; g0 += kFGroup) {
        uint32_t v[kFGroup];
#pragma unroll
        for (int g = 0; g < kFGroup; ++g) v[g] = win[buf][g0 + g][lane];
#pragma unroll
        for (int g = 0; g < kFGroup; ++g) {
          const uint32_t k = k0 + g0 + g;
          const uint64_t bs = A.c_lo + (uint64_t)k * kFB;
          const uint64_t be = bs + kFB < A.c_hi ? bs + kFB : A.c_hi;
          if (lane == 0) went[buf][g0 + g] = e;
          if (k < A.nblk && e < be) {
            const uint32_t j = (uint32_t)__builtin_amdgcn_readfirstlane((int)(e - bs));
            if (j < 64) {
              e = be + (uint32_t)__builtin_amdgcn_readlane((int)v[g], (int)j);
            } else {
              e = be + A.ex[(uint64_t)k * kFB + j];  // an entry past a long match
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (k0 > 0) flush_entries(k0 - kFWin, buf ^ 1, tid, kFThreads);
  if (tid == 0) *A.entry = e;
}

// One workgroup per block: the FIND chain from the block's exact entry.  N(p)
// for every position again (as forest_exit_kernel), then 64 lane sub-blocks of
// kFSub positions: pointer jumping to each position's first orbit element past
// its sub-block, one thread follows the chain across the sub-blocks (64
// dependent LDS reads), and lane i walks sub-block i from its entry along N,
// summing matches (COUNT) or writing them from the block's output base plus
// the lane prefix (WRITE).
template <int FMT, int W, bool WRITE>
__global__ __launch_bounds__(kFThreads) void forest_walk_kernel(ScanParams P, ForestArgs A)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t fsm[];
  __shared__ uint64_t sent[kFB / kFSub];
  const int tid = threadIdx.x, lane = tid & 63;
  const Tab<FMT> T = fstage_tables<FMT>(P, fsm, tid, kFThreads);
  uint8_t* bytes = fsm + ftab_bytes(P);
  uint32_t* N = reinterpret_cast<uint32_t*>(bytes + kFStage);
  uint32_t* J = N + kFB;
  uint32_t* LE = J + kFB;
  const uint64_t k = blockIdx.x;
  const uint64_t bs = A.c_lo + k * kFB;
  const uint64_t be = bs + kFB < A.c_hi ? bs + kFB : A.c_hi;
  const uint32_t nb = (uint32_t)(be - bs);
  const uint64_t e0 = A.bentry[k];
  if (e0 >= be) {  // a long match covers the whole block
    if (!WRITE && tid == 0) A.bsum[3 * k] = A.bsum[3 * k + 1] = A.bsum[3 * k + 2] = 0;
    return;
  }
  const Win w = fstage_bytes(P, bytes, bs, tid, kFThreads);
  __syncthreads();
  forest_n<FMT, W, true>(T, w, bs, nb, N, LE, tid, kFThreads);
  __syncthreads();
  // J[r]: first orbit element >= the end of r's sub-block (block-relative)
  for (uint32_t r = tid; r < nb; r += kFThreads) J[r] = N[r] & kFNMask;
  __syncthreads();
  for (;;) {
    bool ch = false;
    for (uint32_t r = tid; r < nb; r += kFThreads) {
      const uint32_t se = (r / kFSub + 1) * kFSub < nb ? (r / kFSub + 1) * kFSub : nb;  // sub-block end
      const uint32_t j = J[r];
      if (j < se) {
        J[r] = J[j];
        ch = true;
      }
    }
    if (!__syncthreads_or(ch)) break;
  }
  if (tid == 0) {
    uint64_t e = e0;
    for (uint32_t i = 0; i < kFB / kFSub; ++i) {
      const uint64_t se = bs + (uint64_t)(i + 1) * kFSub;
      sent[i] = e;
      if (e < se && e < be) e = bs + J[e - bs];
    }
  }
  __syncthreads();
  if (tid >= 64) return;
  // lane = sub-block
  const uint64_t sa = bs + (uint64_t)lane * kFSub;
  const uint64_t sb = sa + kFSub < be ? sa + kFSub : be;
  const Ctx C = W == kWalkCtx ? Ctx{P.acap, 0u, P.delta} : Ctx{P.caps, P.log_row, P.delta};
  uint32_t ovf = 0;
  CountEm em;
  for (uint64_t p = sent[lane]; p < sb;) {
    const uint32_t nv = N[p - bs];
    const uint64_t q = bs + (nv & kFNMask);
    if (nv & kFMatch) em.put(C, p, nv & kFEmpty ? 0 : q - p, LE[p - bs], +1);
    ovf |= nv & kFOvf;
    p = q;
  }
  if constexpr (WRITE) {
    uint64_t incl = em.cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    WriteEm we{A.bbase[k] + incl - em.cnt, P.out_capacity, P.out_start, P.out_len, P.out_cap};
    for (uint64_t p = sent[lane]; p < sb;) {
      const uint32_t nv = N[p - bs];
      const uint64_t q = bs + (nv & kFNMask);
      if (nv & kFMatch) we.put(C, p, nv & kFEmpty ? 0 : q - p, LE[p - bs], +1);
      p = q;
    }
    if (__ballot(we.overflow) && lane == 0) atomicOr(P.flags, UGPU_FLAG_CAPACITY);
  } else {
    const uint64_t c = wave_sum(em.cnt), d = wave_sum(em.dg), x = wave_sum(em.dc);
    if (lane == 0) {
      A.bsum[3 * k] = c;
      A.bsum[3 * k + 1] = d;
      A.bsum[3 * k + 2] = x;
    }
  }
  if (__ballot(ovf != 0) && lane == 0) atomicOr(P.flags, UGPU_FLAG_HALO);
}

// One workgroup: running totals += the chunk's block sums; bbase = exclusive
// prefix of the block counts, starting at the matches before this chunk.
// last: also write the DevTotals of the whole range.
__global__ __launch_bounds__(kFixThreads) void forest_sum_kernel(ForestArgs A, DevTotals* tot, uint64_t lo, int last)
{
  __shared__ uint64_t wsum[3][kFixThreads / 64];
  __shared__ uint64_t wscan[kFixThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t per = (A.nblk + kFixThreads - 1) / kFixThreads;
  const uint32_t k0 = tid * per, k1 = k0 + per < A.nblk ? k0 + per : A.nblk;
  uint64_t c = 0, d = 0, x = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    c += A.bsum[3 * k];
    d += A.bsum[3 * k + 1];
    x += A.bsum[3 * k + 2];
  }
  uint64_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const uint64_t sd = wave_sum(d), sx = wave_sum(x);
  if (lane == 63) wscan[wid] = incl;
  if (lane == 0) {
    wsum[1][wid] = sd;
    wsum[2][wid] = sx;
  }
  __syncthreads();
  const uint64_t run = A.run[0];
  uint64_t off = run, tc = 0, td = 0, tx = 0;
  for (int w = 0; w < kFixThreads / 64; ++w) {
    if (w < wid) off += wscan[w];
    tc += wscan[w];
    td += wsum[1][w];
    tx += wsum[2][w];
  }
  uint64_t b = off + incl - c;
  for (uint32_t k = k0; k < k1; ++k) {
    A.bbase[k] = b;
    b += A.bsum[3 * k];
  }
  __syncthreads();
  if (tid == 0) {
    A.run[0] = run + tc;
    A.run[1] += td;
    A.run[2] += tx;
    if (last) {
      tot->count = A.run[0];
      tot->digest = A.run[1];
      tot->dcap = A.run[2];
      tot->entry = lo;
      tot->exit = *A.entry;
      tot->rounds = 0;
    }
  }
}

__global__ void forest_init_kernel(ForestArgs A, uint64_t entry)
{
  if (threadIdx.x == 0) {
    *A.entry = entry;
    A.run[0] = A.run[1] = A.run[2] = 0;
  }
}

// ---------------------------------------------------------------- launcher
namespace {

template <int FMT, int W>
hipError_t forest_fmt(const ScanParams& P, ForestArgs A, uint64_t entry, bool write, DevTotals* tot,
                      hipStream_t st)
{
  const size_t tab = ((2 * (size_t)P.ntrans_pad + 256) + 15) & ~size_t(15);
  const size_t sm1 = tab + kFStage + 4 * (size_t)kFB;
  const size_t sm2 = tab + kFStage + 12 * (size_t)kFB;
  hipError_t e;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(forest_exit_kernel<FMT, W>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm1)) != hipSuccess)
    return e;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(forest_walk_kernel<FMT, W, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm2)) != hipSuccess)
    return e;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(forest_walk_kernel<FMT, W, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm2)) != hipSuccess)
    return e;
  const uint64_t lo = entry, hi = P.hi;
  hipLaunchKernelGGL(forest_init_kernel, dim3(1), dim3(64), 0, st, A, entry);
  if (lo >= hi) {
    A.nblk = 0;
    hipLaunchKernelGGL(forest_sum_kernel, dim3(1), dim3(kFixThreads), 0, st, A, tot, P.lo, 1);
    return hipGetLastError();
  }
  for (uint64_t c = lo; c < hi; c += kFChunk) {
    A.c_lo = c;
    A.c_hi = c + kFChunk < hi ? c + kFChunk : hi;
    A.nblk = (uint32_t)((A.c_hi - A.c_lo + kFB - 1) / kFB);
    const int last = A.c_hi == hi;
    hipLaunchKernelGGL((forest_exit_kernel<FMT, W>), dim3(A.nblk), dim3(kFThreads), sm1, st, P, A);
    hipLaunchKernelGGL(forest_stitch_kernel, dim3(1), dim3(kFThreads), 0, st, A);
    hipLaunchKernelGGL((forest_walk_kernel<FMT, W, false>), dim3(A.nblk), dim3(kFThreads), sm2, st, P, A);
    hipLaunchKernelGGL(forest_sum_kernel, dim3(1), dim3(kFixThreads), 0, st, A, tot, P.lo, last);
    if (write)
      hipLaunchKernelGGL((forest_walk_kernel<FMT, W, true>), dim3(A.nblk), dim3(kFThreads), sm2, st, P, A);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

uint64_t forest_block() { return kFB; }

hipError_t launch_forest(const ScanParams& P, uint32_t format, const ForestArgs& A, uint64_t entry, bool write,
                         DevTotals* tot, hipStream_t st)
{
  if (P.acap)
    return format == 0   ? forest_fmt<0, kWalkCtx>(P, A, entry, write, tot, st)
           : format == 1 ? forest_fmt<1, kWalkCtx>(P, A, entry, write, tot, st)
                         : forest_fmt<2, kWalkCtx>(P, A, entry, write, tot, st);
  if (P.look)  // (lookahead, with or without option W)
    return format == 0   ? forest_fmt<0, kWalkLook>(P, A, entry, write, tot, st)
           : format == 1 ? forest_fmt<1, kWalkLook>(P, A, entry, write, tot, st)
                         : forest_fmt<2, kWalkLook>(P, A, entry, write, tot, st);
  if (P.wtab)
    return format == 0   ? forest_fmt<0, kWalkWord>(P, A, entry, write, tot, st)
           : format == 1 ? forest_fmt<1, kWalkWord>(P, A, entry, write, tot, st)
                         : forest_fmt<2, kWalkWord>(P, A, entry, write, tot, st);
  return format == 0   ? forest_fmt<0, kWalkPlain>(P, A, entry, write, tot, st)
         : format == 1 ? forest_fmt<1, kWalkPlain>(P, A, entry, write, tot, st)
                       : forest_fmt<2, kWalkPlain>(P, A, entry, write, tot, st);
}

}  // namespace ugpu
