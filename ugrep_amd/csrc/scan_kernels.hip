// scan_kernels.hip -- chain-record stitching kernels of the FIND engine (see
// scan_kernels.hpp for the chain/stitch scheme).  The scan kernels themselves
// are sparse_kernel.hip (prefiltered patterns) and dense_kernel.hip.
#include "device_common.hpp"

namespace ugpu {


// ---------------------------------------------------------------- fix kernel
// Open walks (sparse_kernel walk truncation, OpenRec): a wave whose chain
// ended in a walk still alive at its range end `lim` counted no match for it.
// The walk W is resolved from the records of the waves after it:
//   R1 (one thread per open wave k): walk W on from lim, and from the first
//      match start c1 of wave k+1 on, the walk V of c1 beside it; when both
//      are alive in the same state at the same position they are the same
//      walk from there on (kOpenConv), so W's accepts after that point are
//      V's: V's end e1 (a closed first match) or, when V is wave k+1's own
//      open walk, that walk's resolved end.  W may die first (kOpenDead).
//      A walk that neither dies nor converges within kOpenConvBudget bytes
//      is left to R1b.
//   R1b (one wave per such walk, when there are few): W walked on by the whole
//      wave, 1 KiB a round (coop_continue), until it dies or reaches the end
//      of the readable bytes (kOpenDead), within kOpenCoopBudget bytes; past
//      that it gives up (kOpenUnres: UGPU_FLAG_BUDGET, the forest FIND).  The
//      last open wave of a run of candidate bytes that crosses many waves
//      (a needle-free letter run under [a-z]+(ing|ed)) is resolved here; the
//      waves before it converge with their successors in R1.
//   R2 (wave 0, open waves in descending order, 64 at a time): the ends, each
//      from the next one's (a run of candidate bytes across many waves is one
//      chain of converged open walks).
//   R3 (one thread per open wave): the match [c, e) joins the wave's counts
//      and its exit becomes e; an end before lim re-walks the rest of the
//      wave's chain from there (the COUNT pass had dropped those candidates).
// Afterwards every record is what an untruncated walk would have given, and
// the stitch below runs as for any kernel.
// fix_kernel applies each block's corrections to its record in place (count,
// digest, dcap; the owner thread only): the stitch loop keeps no per-block
// arrays in registers, and the records' entries and pads (the sparse
// kernel's first-match shortcut, its open walks) stay as the scan wrote them.
__device__ __forceinline__ void rec_add(const ScanParams& P, uint64_t b, uint64_t dcnt, uint64_t ddg, uint64_t ddc)
{
  uint64_t* r = reinterpret_cast<uint64_t*>(P.recs + b);
  r[2] += dcnt;
  r[3] += ddg;
  r[4] += ddc;
}

// R1b: walk W on with the whole wave from DFA entry s before byte q, up to
// lim (<= rend).  Each round lane l walks the 16 bytes at (q & ~15) + 16 l
// from a guessed entry (W's entry run over the 4 bytes before them: exact when
// the state depends on the last few bytes, as in a letter loop); the guesses
// are checked in lane order against the previous lane's exit, and W advances
// to the first lane whose guess was wrong, or dies in the first dying lane
// before it (as sparse_kernel's coop_walk, bytes from registers instead of
// LDS).  Returns true when W died (q = the byte it died on) or reached the
// readable end (q = rend); lastw / lew = W's last accept (unchanged if none).
template <int FMT>
__device__ __forceinline__ bool coop_continue(const Tab<FMT>& T, const Win& w, uint32_t& s, uint64_t& q, uint64_t lim,
                                              uint64_t& lastw, uint32_t& lew)
{
  const int lane = threadIdx.x & 63;
  while (q < lim) {
    const uint64_t base = q & ~uint64_t(15);
    const uint64_t sa = base + 16u * (uint32_t)lane;
    uint32_t d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint64_t i = sa + 4 * k + b;
        x |= (i < w.rend ? (uint32_t)w.g[i] : 0u) << (8 * b);
      }
      d[k] = x;
    }
    const uint32_t pw = (uint32_t)__shfl_up((int)d[3], 1, 64);  // the 4 bytes before the lane's 16
    uint32_t spec = s;
    if (lane != 0) {
      uint32_t t = s;
#pragma unroll
      for (int b = 0; b < 4; ++b) t = t ? T.step(t, (pw >> (8 * b)) & 0xffu) : 0u;
      spec = t ? t : s;
    }
    const uint64_t a = sa > q ? sa : q;
    const uint64_t z = sa + 16 < lim ? sa + 16 : lim;
    uint32_t cur = spec, lel = 0;
    uint64_t lastl = 0, dl = 0;
    for (uint64_t i = a; i < z; ++i) {
      const uint32_t byte = (d[(i - sa) >> 2] >> (8 * ((i - sa) & 3))) & 0xffu;
      const uint32_t e = T.step(cur, byte);
      if (e == 0) {
        dl = i + 1;
        break;
      }
      cur = e;
      if (e >= T.accb) {
        lastl = i + 1;
        lel = e;
      }
    }
    const uint32_t prev = (uint32_t)__shfl_up((int)cur, 1, 64);
    const bool seg = a < z;
    const int nl = __popcll(__ballot(seg));
    const uint64_t bad = __ballot(seg && lane != 0 && spec != prev);
    const uint64_t dead = __ballot(seg && dl != 0);
    const uint64_t accm = __ballot(lastl != 0);
    const int j = bad ? __builtin_ctzll(bad) : nl;
    const int dd = dead ? __builtin_ctzll(dead) : 64;
    const uint64_t m = accm & lowbits((uint64_t)(dd < j ? dd + 1 : j));
    if (m) {
      const int k = 63 - __builtin_clzll(m);
      lastw = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(lastl >> 32), k, 64) << 32) |
              (uint32_t)__shfl((int)(uint32_t)lastl, k, 64);
      lew = (uint32_t)__shfl((int)lel, k, 64);
    }
    if (dd < j) {
      const uint64_t dp = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(dl >> 32), dd, 64) << 32) |
                          (uint32_t)__shfl((int)(uint32_t)dl, dd, 64);
      q = dp - 1;
      return true;
    }
    s = (uint32_t)__shfl((int)cur, j - 1, 64);
    const uint64_t qn = base + 16u * (uint32_t)j;
    q = (j < nl || qn < lim) ? qn : lim;
  }
  return q >= w.rend;
}

constexpr uint64_t kOpenCoopBudget = 64ull << 20;  // bytes R1b walks one open walk on
constexpr int kOpenCoopMax = 256;                  // open walks R1b takes at most (else the forest FIND)

template <int FMT>
__device__ __forceinline__ void resolve_open(const ScanParams& P, const Tab<FMT>& T, const Ctx& C, const Win& w, int G,
                                             int tid, uint64_t* exi, const uint32_t* openm, uint32_t& ovf, uint32_t& over)
{
  constexpr int PER = kMaxRec / kFixThreads;
  const int lane = tid & 63, wid = tid >> 6;
  // R1
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = j * kFixThreads + tid;
    if (b >= G || !((openm[b >> 5] >> (b & 31)) & 1u)) continue;
    OpenRec* o = P.open + b;
    uint32_t s = o->s, v = 0, lew = 0, type = kOpenUnres;
    uint64_t q = o->lim, lastw = 0;
    uint64_t c1 = ~0ull;
    if (b + 1 < G) {
      const BlockRec nr = P.recs[b + 1];
      if ((nr.pad2 & kRecFirst) && nr.pad1 != 0) c1 = nr.pad0;
    }
    const uint64_t qmax = q + kOpenConvBudget;
    if (c1 != ~0ull && c1 < q) {
      // (W stands kOpenSlack past the range end: bring V there first)
      v = T.start;
      for (uint64_t p = c1; p < q && v; ++p) v = T.step(v, w.g[p]);
    }
    for (;;) {
      if (q == c1) v = T.start;
      if (v != 0 && v == s) {
        type = kOpenConv;
        break;
      }
      if (q >= w.rend) {  // the end of the readable bytes: the walk ends here
        if (!w.eof) ovf = 1;
        type = kOpenDead;
        break;
      }
      if (q >= qmax) break;
      const uint32_t byte = w.g[q];
      s = T.step(s, byte);
      if (v) v = T.step(v, byte);
      if (s == 0) {
        type = kOpenDead;
        break;
      }
      ++q;
      if (s >= T.accb) {
        lastw = q;
        lew = s;
      }
    }
    o->q = q;
    o->lastw = lastw;
    o->lew = lew;
    o->sq = s;  // (R1b goes on from here)
    o->type = type;
  }
  __threadfence_block();
  __syncthreads();
  // R1b: the walks R1 left unresolved, one wave each, when there are few
  {
    __shared__ uint32_t nunres;
    if (tid == 0) nunres = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int b = j * kFixThreads + tid;
      if (b < G && ((openm[b >> 5] >> (b & 31)) & 1u) && P.open[b].type == kOpenUnres) atomicAdd(&nunres, 1u);
    }
    __syncthreads();
    if (nunres && nunres <= (uint32_t)kOpenCoopMax) {
      for (int b = 0, k = 0; b < G; ++b) {
        if (!((openm[b >> 5] >> (b & 31)) & 1u)) continue;
        OpenRec* o = P.open + b;
        if (o->type != kOpenUnres) continue;
        if ((k++ % (kFixThreads / 64)) != wid) continue;
        uint32_t s = o->sq, lew = o->lew;
        uint64_t q = o->q, lastw = o->lastw;
        const uint64_t lim = q + kOpenCoopBudget < w.rend ? q + kOpenCoopBudget : w.rend;
        const bool done = s != 0 && coop_continue<FMT>(T, w, s, q, lim, lastw, lew);
        if (lane == 0 && done) {
          if (q >= w.rend && !w.eof) ovf = 1;
          o->q = q;
          o->lastw = lastw;
          o->lew = lew;
          o->type = kOpenDead;
        }
      }
    }
    __threadfence_block();
    __syncthreads();
  }
  // R2
  if (wid == 0) {
    uint64_t carry = 0;
    uint32_t carry_le = 0;
    for (int base = (G - 1) & ~63; base >= 0; base -= 64) {
      const int b = base + lane;
      const bool op = b < G && ((openm[b >> 5] >> (b & 31)) & 1u);
      const uint64_t om = __ballot(op);
      if (!om) continue;
      uint64_t oc = 0, olast = 0, oq = 0, olastw = 0, ne1 = 0;
      uint32_t ole = 0, olew = 0, otype = 0, nle1 = 0;
      if (op) {
        const OpenRec o = P.open[b];
        oc = o.c;
        olast = o.last;
        ole = o.le;
        oq = o.q;
        olastw = o.lastw;
        olew = o.lew;
        otype = o.type;
        if (b + 1 < G) {
          const BlockRec nr = P.recs[b + 1];
          ne1 = nr.pad1;
          nle1 = (uint32_t)nr.pad2;
        }
      }
      uint64_t mye = 0;
      uint32_t myle = 0;
      for (uint64_t m = om; m;) {
        const int k = 63 - __builtin_clzll(m);
        m &= ~(1ull << k);
        auto rl64 = [k](uint64_t x) {
          return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), k) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((uint32_t)x, k);
        };
        const uint32_t ty = (uint32_t)__builtin_amdgcn_readlane(otype, k);
        const uint64_t lw = rl64(olastw);
        // W's own last accept: after lim, else before it (== c: none)
        uint64_t e = lw ? lw : rl64(olast);
        uint32_t le = lw ? (uint32_t)__builtin_amdgcn_readlane(olew, k) : (uint32_t)__builtin_amdgcn_readlane(ole, k);
        if (ty == kOpenConv) {
          // after the convergence point W accepts where V does
          const uint64_t n1 = rl64(ne1);
          const uint64_t ve = n1 == kOpenEnd ? carry : n1;  // (wave b+1 was resolved just before)
          const uint32_t vle = n1 == kOpenEnd ? carry_le : (uint32_t)__builtin_amdgcn_readlane(nle1, k);
          if (ve > rl64(oq)) {
            e = ve;
            le = vle;
          }
        } else if (ty == kOpenUnres) {
          over = 1;
        }
        (void)oc;
        carry = e;
        carry_le = le;
        if (lane == k) {
          mye = e;
          myle = le;
        }
      }
      if (op) {
        P.open[b].e = mye;
        P.open[b].le_e = myle;
      }
    }
  }
  __threadfence_block();
  __syncthreads();
  // R3
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = j * kFixThreads + tid;
    if (b >= G || !((openm[b >> 5] >> (b & 31)) & 1u)) continue;
    const OpenRec o = P.open[b];
    uint64_t tb = P.t0 + (uint64_t)b * P.tpb;
    uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
    if (tb > te) tb = te;
    const uint64_t bhi = clampu(te * P.unit, P.lo, P.hi);
    CountEm d;
    uint64_t p = o.c + 1;
    if (o.e > o.c) {
      d.put(C, o.c, o.e - o.c, o.le_e, +1);
      p = o.e;
    } else if (w.dom && !P.acap && !P.wtab) {
      // the open walk accepts nowhere: the positions it crossed in dominating
      // states start nothing either (tables.hpp dom), up to the block end --
      // all of them when every non-accepting state dominates (dom_all: the
      // walk never accepted, so it crossed the block in such states)
      p = P.dom_all ? (bhi > o.c + 1 ? bhi : o.c + 1) : dom_restart<FMT>(T, w, o.c, bhi);
    }
    // an end before the range end: the chain goes on from there (those
    // candidates were dropped by the COUNT pass)
    const uint64_t lim = p + P.merge_budget;
    while (p < bhi) {
      if (p > lim) {
        over = 1;
        break;
      }
      p = chain_step<FMT, CountEm>(T, w, C, p, d, +1, ovf, bhi);
    }
    exi[b] = p;
    rec_add(P, (uint64_t)b, d.cnt, d.dg, d.dc);
  }
  __threadfence_block();
  __syncthreads();
}

// Block b re-entered at nx instead of its entry `ent` (one fix_kernel round):
// its record's counts corrected in place; returns whether its exit is
// unchanged, else sets `exit`.
template <int FMT>
__device__ __forceinline__ bool fix_block(const ScanParams& P, const Tab<FMT>& T, const Ctx& C, const Win& w, uint64_t b,
                                          uint64_t ent, uint64_t nx, uint64_t bhi, uint64_t& exit, uint32_t& ovf,
                                          uint32_t& over)
{
  uint64_t* r = reinterpret_cast<uint64_t*>(P.recs + b);  // entry, exit, cnt, dg, dc, pad0, pad1, pad2
  if (nx >= bhi) {
    // the true chain enters at or past the block's end (a long match covers
    // it): no chain position in the block, no matches
    if (ent < bhi) r[2] = r[3] = r[4] = 0;
    exit = nx;
    return false;
  }
  CountEm d;
  uint64_t ne = 0, po = ent;
  bool met = false, done = false;
  if constexpr (FMT == 0) {
    const uint64_t pad2 = r[7];
    if (po == r[0] && (pad2 & kRecFirst)) {
      // the speculative chain from the record's entry visits every position
      // up to its first kept match c1 and then its end e1: a true entry there
      // meets it
      uint64_t c1 = r[5], e1 = r[6];
      uint32_t le1 = (uint32_t)pad2;
      if (e1 == kOpenEnd) {
        const OpenRec o = P.open[b];
        e1 = o.e > o.c ? o.e : 0;  // (no match: the chain went on at c1 + 1)
        le1 = o.le_e;
        if (e1 == 0) c1 = 0;  // (no shortcut past c1)
      }
      if (r[6] == 0 || nx <= c1) {
        met = done = true;
      } else if (e1 != 0) {
        d.put(C, c1, e1 - c1, le1, -1);  // the first match is not on the true chain
        if (nx == e1)
          met = done = true;
        else
          po = e1;
      }
    }
  }
  if (!done)
    met = P.acap   ? merge<FMT, kWalkCtx>(T, w, C, po, nx, bhi, d, ne, ovf, P.merge_budget, &over)
          : P.look ? merge<FMT, kWalkLook>(T, w, C, po, nx, bhi, d, ne, ovf, P.merge_budget, &over)
          : P.wtab ? merge<FMT, kWalkWord>(T, w, C, po, nx, bhi, d, ne, ovf, P.merge_budget, &over)
                   : merge<FMT>(T, w, C, po, nx, bhi, d, ne, ovf, P.merge_budget, &over);
  r[2] += d.cnt;
  r[3] += d.dg;
  r[4] += d.dc;
  exit = ne;
  return met;
}

// One workgroup re-enters every block whose speculative entry differs from its
// predecessor's exit (merge over the block's byte range, bytes from global),
// repeating until no exit changes; then reduces the totals and produces the
// exact block entries and output bases for the OFFSETS pass.  A block the
// true chain enters at or past its end is skipped in one step (a long match
// covers it); a sparse_kernel record whose first kept match the true entry
// reaches or ends at is corrected without a walk (BlockRec pads).
template <int FMT>
__global__ __launch_bounds__(kFixThreads) void fix_kernel(ScanParams P)
{
  __shared__ uint64_t ent[kMaxRec], exi[kMaxRec];
  __shared__ uint64_t wred[3][kFixThreads / 64];
  __shared__ uint64_t wscan[kFixThreads / 64];
  __shared__ uint32_t openm[kMaxRec / 32];
  constexpr int PER = kMaxRec / kFixThreads;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = (int)P.nrec;
  const Tab<FMT> T = tab_global<FMT>(P);
  const Ctx C = P.acap ? Ctx{P.acap, 0u, P.delta} : Ctx{P.caps, P.log_row, P.delta};
  const Win w = win_of(P);
  uint32_t ovf = 0, over = 0;
  // the scan kernel already gave up on these chains (UGPU_FLAG_BUDGET): the host
  // resolves the range with the forest FIND, nothing to stitch
  const uint32_t fl = __hip_atomic_load(P.flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (fl & UGPU_FLAG_BUDGET) return;
  const bool any_open = FMT == 0 && P.open && (fl & UGPU_FLAG_OPEN);
  if (any_open)
    for (int i = tid; i < kMaxRec / 32; i += kFixThreads) openm[i] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = j * kFixThreads + tid;
    if (b < G) {
      const uint64_t* r = reinterpret_cast<const uint64_t*>(P.recs + b);
      ent[b] = r[0];
      exi[b] = r[1];
      if (any_open && (r[7] & kRecOpen)) atomicOr(&openm[b >> 5], 1u << (b & 31));
    }
  }
  if (any_open) {
    __syncthreads();
    resolve_open<FMT>(P, T, C, w, G, tid, exi, openm, ovf, over);
    over = __syncthreads_or(over) ? 1u : 0u;
  }
  uint32_t rounds = 0;
  for (;;) {
    __syncthreads();
    uint32_t chm = 0;  // bit j: block j * kFixThreads + tid changed
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int b = j * kFixThreads + tid;
      if (b > 0 && b < G && exi[b - 1] != ent[b]) chm |= 1u << j;
    }
    __syncthreads();
    // (a block's new entry is its predecessor's exit as read here: one that a
    // merge of this round already moved only brings the fixpoint closer)
    for (uint32_t m = chm; m;) {
      const int j = __builtin_ctz(m);
      m &= m - 1;
      const uint64_t b = (uint64_t)j * kFixThreads + tid;
      const uint64_t nx = exi[b - 1];
      if (nx == ent[b]) continue;
      uint64_t tb = P.t0 + b * P.tpb;
      uint64_t te = tb + P.tpb < P.t1 ? tb + P.tpb : P.t1;
      if (tb > te) tb = te;
      const uint64_t bhi = clampu(te * P.unit, P.lo, P.hi);
      uint64_t ne = 0;
      if (!fix_block<FMT>(P, T, C, w, b, ent[b], nx, bhi, ne, ovf, over)) exi[b] = ne;
      ent[b] = nx;
    }
    if (!__syncthreads_or(chm != 0)) break;
    if (__syncthreads_or(over) || ++rounds >= P.max_rounds) {  // chains that do not resynchronise
      over = 1;
      break;
    }
  }
  __threadfence_block();
  __syncthreads();
  uint64_t cnt[PER];
  uint64_t md = 0, mdc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = j * kFixThreads + tid;
    cnt[j] = 0;
    if (b < G) {
      const uint64_t* r = reinterpret_cast<const uint64_t*>(P.recs + b);
      cnt[j] = r[2];
      md += r[3];
      mdc += r[4];
    }
  }
  // totals + exclusive scan of block counts (block order b = j * kFixThreads + tid:
  // one workgroup scan per j, carried across j)
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
             : P.look ? merge<FMT, kWalkLook>(T, w, C, old_entry, new_entry, P.hi, d, ne, ovf, P.merge_budget, &over)
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
