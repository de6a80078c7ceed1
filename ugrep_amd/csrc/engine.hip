// engine.hip -- host side of the C ABI declared in include/ugpu.h.
//
// Pipeline of one whole-buffer FIND (what Matcher::find() computes lazily, one
// match per call, lib/matcher.cpp:42-750):
//   sparse_kernel / dense_kernel <WRITE=false>
//                                 wave-persistent grid, speculative per-wave chains,
//                                 per-wave (entry, exit, count, digests)
//   fix_kernel                    stitch wave entries, totals, output bases
//   sparse_kernel / dense_kernel <WRITE=true>
//                                 (OFFSETS only) re-walk from exact entries and
//                                 store (start, len, cap) records
// The prefiltered sparse kernel serves tables with a selective three-byte
// prefilter (tables.hpp); every other table runs the dense kernel.
// Tables are uploaded once per ugpu_dfa (one Pattern), shared by all scanners.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <future>
#include <vector>

#include "../../include/ugpu.h"
#include "plan.hpp"
#include "scan_kernels.hpp"
#include "tables.hpp"

// Geometry of a UTF-8 / NUL scan of the device bytes dbuf[0, len) (U.out unset).
ugpu::Utf8Params utf8_params(const uint8_t* dbuf, uint64_t len)
{
  // CU count of the calling thread's device (cached per device id)
  static std::atomic<int> cached[64];
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if (dev < 64 && cached[dev].load(std::memory_order_relaxed) > 0) {
    cus = cached[dev].load(std::memory_order_relaxed);
  } else {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (dev < 64) cached[dev].store(cus, std::memory_order_relaxed);
  }
  ugpu::Utf8Params U{};
  U.head = reinterpret_cast<uintptr_t>(dbuf) & 15u;
  U.g = dbuf - U.head;
  U.len = len;
  U.span = (U.head + len + 15u) & ~15ull;
  const uint64_t tile = ugpu::utf8_tile();
  const uint64_t tiles = (U.span + tile - 1) / tile;
  const uint64_t want = (uint64_t)cus * 16;  // about 16 waves per CU
  const uint64_t tpw = (tiles + want - 1) / want;
  U.per = tpw * tile;
  U.nwaves = (tiles + tpw - 1) / tpw;
  return U;
}


using namespace ugpu;

struct ugpu_dfa {
  DfaTables t;
  // the plan the tables were uploaded with (lookback, option-W route); the
  // kernel-choice test knobs (UGPU_SPARSE, UGPU_XI, ...) stay live: scanners
  // and ugpu_dfa_info_get read them when they are called
  DfaPlan plan;
  int device = 0;
  uint32_t ntrans_pad = 0;
  uint16_t* d_trans = nullptr;
  uint32_t* d_trans32 = nullptr;  // wide tables (FMT_WIDE)
  uint16_t* d_xtrans = nullptr;  // FIND transducer (restart-local tables on the dense path)
  uint8_t* d_xid = nullptr;      // immediate transducer ids (xi_kernel), COUNT scans
  uint16_t* d_xg = nullptr;      // gap transducer (xg_kernel), COUNT scans
  uint8_t* d_xu = nullptr;       // code-point run tables (xc_kernel U mode): kXuTab bytes, then kXuBm3 dwords
  uint8_t* d_xg_sync = nullptr;
  uint8_t* d_cls = nullptr;
  uint32_t* d_caps = nullptr;
  uint32_t* d_wtab = nullptr;  // option W: Unicode Word ranges (UGPU_PAT_WORD)
  uint32_t nwtab = 0;
  // option W on a table equivalent to \w+: on valid UTF-8 the W
  // rules remove nothing, so such scans run the non-W kernels (xg_kernel)
  bool wplus = false;
  bool wsparse = false;  // option W on the sparse kernel without a selective prefilter (DfaPlan::wsparse)
  // option W on a two-state table whose X is the ASCII word bytes: xc_kernel
  // applies the W rules itself (non-ASCII input falls back to wfind_kernel)
  bool xcw = false;
  // line anchors / option N (UGPU_PAT_EMPTY): amode = the table has anchors,
  // or matches the empty string under N; its scans run the context walk
  // (wfind_kernel, device_common.hpp kWalkCtx) on the per-context accepts
  bool nul = false, amode = false;
  uint32_t* d_acap = nullptr;  // acap, or (word boundaries) acap_rows then acap_map
  // no match starts right after a word character (ScanParams::wstart)
  bool wstart = false;
  // loop-needle tables (C+N, ScanParams::lb_cls): the prefilter finds N, and
  // each candidate walks back to its C-run's start (host_api.cpp loop_needle)
  bool lb = false;
  uint8_t lb_ft[20] = {};
  uint32_t* d_lbcls = nullptr;  // 256-bit mask of C
  uint32_t* d_dom = nullptr;    // dominated restarts (tables.hpp dom), or NULL
  uint32_t* d_look = nullptr;   // lookahead TAIL / HEAD masks per state (tables.hpp look), or NULL
  // idle scanners of ugpu_find_all calls on this table (reused: creating one
  // costs device allocations and property queries)
  std::mutex pool_mu;
  std::vector<ugpu_scanner*> pool;
  std::vector<ugpu_scanner*> pool_w;  // scanners that prefer kernels with a record-writing pass (records path)
  // the opcode words and flags it was built from, and its copies on other
  // devices (ugpu_find_all_multi), created on first use
  std::vector<uint32_t> opc;
  uint32_t pflags = 0;
  std::mutex rep_mu;
  std::vector<ugpu_dfa*> reps;
};

struct ugpu_scanner {
  const ugpu_dfa* dfa = nullptr;
  int device = 0;
  int max_rec = 0;       // chain records per scan (blocks or waves)
  bool sparse = false;   // prefiltered wave-persistent kernel (sparse_kernel.hip)
  bool xi = false;       // COUNT scans run xi_kernel (immediate tables); OFFSETS use the dense kernel
  bool xg = false;       // COUNT scans run xg_kernel (gap tables); OFFSETS use the dense kernel
  bool xc = false;       // COUNT and OFFSETS scans run xc_kernel (two-state and, U mode, code-point run tables)
  bool xu_xi = false, xu_xg = false;  // U mode: the kernels a range goes to when it flags UGPU_FLAG_USLOW
  bool xu = false;       // xc_kernel runs in U mode (code-point run tables)
  bool pref_write = false;  // created for a records consumer (scanner_acquire)
  bool last_xc = false;  // the last ugpu_scan ran xc_kernel
  bool word = false;     // option W: every pass runs wfind_kernel (wfind.hip) (per scan when wfast)
  bool wfast = false;    // option W on a \w+ table: non-W kernels when the scanned bytes are valid UTF-8
  bool wu = false;       // ... and those scans run xc_kernel's U mode with the run-edge check (no isutf8 pass)
  bool wforce = false;   // (the next scan of a wfast scanner runs wfind_kernel)
  bool xu_exact = false; // U mode: scans run the exact kernel (after a range that flagged UGPU_FLAG_UMIX)
  int word_rec = 0;      // chain records of a wfind scan
  bool wxc = false;      // option W on xc_kernel (dfa->xcw), wfind_kernel when it flags UGPU_FLAG_WSLOW
  uint32_t bol0 = 1;     // dbuf[0] begins a line (ugpu_scanner_context; anchored tables)
  size_t smem = 0;       // sparse / dense kernel
  size_t xi_smem = 0;
  int xi_rec = 0;        // chain records of an xi scan
  bool last_xi = false;  // the last ugpu_scan ran xi_kernel
  const uint8_t* last_buf = nullptr;
  uint64_t last_args[5] = {0, 0, 0, 0, 0};  // lo, hi, read_end, at_eof, bias of the last scan
  BlockRec* d_recs = nullptr;
  uint64_t* d_entries = nullptr;
  uint64_t* d_obase = nullptr;
  // xc_kernel COUNT passes of record scanners also write the In bits
  // (ScanParams::inbits) unless UGPU_XC_BITMAP=0; OFFSETS then expands them
  uint16_t* d_inbits = nullptr;
  uint64_t inbits_cap = 0;  // bytes
  uint64_t* d_fix = nullptr;  // xc_kernel OFFSETS: per wave, the record whose start an earlier wave wrote
  OpenRec* d_open = nullptr;  // sparse_kernel: per wave, its open walk (walk truncation)
  uint32_t* d_susp = nullptr;  // sparse_kernel: per wave, suspended at a long walk (resume launch)
  SuspRec* d_srec = nullptr;   // ... and its suspended state
  DevTotals* d_tot = nullptr;
  uint32_t* d_flags = nullptr;
  DevTotals* h_tot = nullptr;  // pinned
  uint32_t* h_flags = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipStream_t stream = nullptr;
  ScanParams last{};
  uint64_t off = 0;  // alignment shift of the last scan
  bool have_scan = false;
  // forest FIND (forest.hip): scratch, allocated on first use, and whether the
  // last scan was resolved by it (its OFFSETS pass then runs the forest too)
  bool forest = false;
  uint64_t f_cap = 0;  // chain positions the scratch covers
  uint32_t* d_fex = nullptr;
  uint64_t* d_fvar = nullptr;  // entry, run[3]
  uint64_t* d_fent = nullptr;
  uint64_t* d_fsum = nullptr;
  uint64_t* d_fbase = nullptr;
  // single-pass OFFSETS (sparse tables): the COUNT pass stages each wave's
  // records (ugpu_scanner_stage, or a ugpu_find_all in OFFSETS mode)
  bool stage = false, stage_once = false, staged_last = false;
  uint64_t* d_st_start = nullptr;
  uint32_t* d_st_len = nullptr;
  uint32_t* d_st_cap = nullptr;
  uint32_t* d_st_n = nullptr;
};

namespace {

const char* const kBudgetMsg =
    "the FIND chains of this table do not resynchronise on this input (stitch budget exceeded): use the CPU matcher";

// (the error string lives in the host library, libugpu_host.so: ugpu_last_error)
int fail(int code, const std::string& msg) { return ugpu::host_fail(code, msg); }

int hip_fail(hipError_t e, const char* what)
{
  return ugpu::host_fail(UGPU_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                              \
  do {                                             \
    hipError_t _e = (expr);                        \
    if (_e != hipSuccess) return hip_fail(_e, #expr); \
  } while (0)

// Process exit.  A caller may release handles from its own static
// destructors (ugrep keeps its matcher in a global unique_ptr,
// src/ugrep.cpp:4491, so the drop-in adapter's last stream and tables are
// released after main returns).  Those run after this library's pools are
// destroyed and after the HIP runtime's own exit teardown, both registered
// later than such a global: a release there wrote into the freed pool vectors
// and called into a torn-down runtime (an intermittent "corrupted
// double-linked list" abort at ugrep_gpu's exit).  The first HIP call of the
// process arms an atexit handler, registered after the runtime's, so it runs
// before both; from then on the release calls free nothing (the process is
// ending, the driver reclaims its device memory) and ugpu_select_device makes
// no HIP call.
std::atomic<bool> g_exiting{false};

void on_process_exit() { g_exiting.store(true, std::memory_order_release); }

void exit_guard_arm()
{
  static std::once_flag once;
  std::call_once(once, [] { (void)std::atexit(on_process_exit); });
}

bool exiting() { return g_exiting.load(std::memory_order_acquire); }

// UGPU_TRACE=1: one stderr line per pipeline step (debugging)
bool trace_on()
{
  static const bool on = std::getenv("UGPU_TRACE") && std::getenv("UGPU_TRACE")[0] == '1';
  return on;
}
#define UGPU_TRACE(...)                  \
  do {                                   \
    if (trace_on()) {                    \
      std::fprintf(stderr, "[ugpu] " __VA_ARGS__); \
      std::fflush(stderr);               \
    }                                    \
  } while (0)

uint64_t env_u64(const char* name, uint64_t dflt)
{
  const char* v = std::getenv(name);
  return v && *v ? std::strtoull(v, nullptr, 0) : dflt;
}

// context tables on sparse_kernel: the acap (+ amap) entries it stages in LDS
// (0: too large, or no context accepts; they stay in global memory)
uint32_t acap_lds_n(const ugpu_dfa* d)
{
  if (!d->amode) return 0;
  const size_t n = d->t.ctx_word ? d->t.acap_rows.size() + d->t.states : d->t.acap.size();
  return n <= kSpAcapLds ? (uint32_t)n : 0u;
}

// fix_kernel rounds allowed for a geometry before it gives up and the forest
// FIND (forest.hip) resolves the range: resynchronising tables need 0-1 rounds
// (more only for matches spanning several records), each round walks serially,
// so about 256 KiB of re-walks in total (UGPU_FIX_BUDGET), 4 to 16 rounds
uint32_t fix_rounds_for(const ScanParams& P)
{
  const uint64_t rec = P.tpb * P.unit ? P.tpb * P.unit : 1;
  uint64_t r = env_u64("UGPU_FIX_BUDGET", 256ull << 10) / rec;
  if (r < 4) r = 4;
  if (r > 16) r = 16;
  return (uint32_t)r;
}

int utf8_scan(const uint8_t* dbuf, uint64_t len, bool nul, uint64_t* pos, void* stream);

// two-state tables run xc_kernel for COUNT scans (UGPU_XC=0: xi/xg/dense)
bool dfa_xc(const ugpu_dfa* d)
{
  const char* env = std::getenv("UGPU_XC");
  return d->t.xc && !d->t.filter && !d->lb && d->t.cap1 != 0 && (!d->d_wtab || d->xcw) && !(env && env[0] == '0');
}

// code-point run tables run xc_kernel's U mode for COUNT and OFFSETS scans
// when they have no gap transducer: on C4 (\w+) xg_kernel measured 3.0 ms
// against U mode's 3.17.  UGPU_XU=1 prefers U mode, UGPU_XU=0
// never takes it.  Under option W only on \w+ (the W fast path).
// code-point run tables take xc_kernel's U mode, also when they have a gap
// transducer (C4 \w+: xu_kernel 2.30 ms, xg_kernel 2.94 ms; UGPU_XU=0 keeps
// xg_kernel / the table's other kernel)
bool dfa_xu(const ugpu_dfa* d)
{
  const char* env = std::getenv("UGPU_XU");
  const bool off = env && env[0] == '0';
  return d->d_xu && (!d->d_wtab || d->wplus) && !off;
}

void fill_tables(ScanParams& P, const ugpu_dfa* d)
{
  P.trans = d->d_trans;
  P.trans32 = d->d_trans32;
  P.xtrans = d->d_xtrans;
  P.xid = d->d_xid;
  P.xid_rows = d->t.xid_rows;
  P.xg = d->d_xg;
  P.xg_sync = d->d_xg_sync;
  P.xg_cls = d->d_xg_sync ? d->d_xg_sync + 256 : nullptr;
  P.xg_stride = 2 * d->t.xg2_pad;
  P.xg_entries = (uint32_t)((d->t.xg2.size() + 7) & ~size_t(7));
  P.cls = d->d_cls;
  P.caps = d->d_caps;
  P.ntrans_pad = d->ntrans_pad;
  P.start = d->t.start;
  P.accb = d->t.accb;
  P.log_row = d->t.log_row;
  P.nstates = d->t.states;
  P.cap1 = d->t.cap1;
  P.wtab = d->d_wtab;
  P.nwtab = d->nwtab;
  P.xc_cls = d->d_cls + 256;
  // (option W on xc_kernel: 1 = X is the ASCII word bytes, 2 = a subset of them)
  P.xc_w = d->xcw ? (d->t.xc_w ? 1u : 2u) : 0u;
  P.xu_tab = dfa_xu(d) ? d->d_xu : nullptr;
  P.xu_bm3 = d->d_xu ? reinterpret_cast<const uint32_t*>(d->d_xu + kXuTab) : nullptr;
  P.xu_null = d->t.xu_null;
  P.acap = d->amode ? d->d_acap : nullptr;
  P.ctx_word = d->amode && d->t.ctx_word ? 1u : 0u;
  P.acap_n = (uint32_t)(P.ctx_word ? d->t.acap_rows.size() : d->t.acap.size());
  P.acap_lds = acap_lds_n(d) != 0 && env_u64("UGPU_SP_ACAP_LDS", 1) != 0 ? 1u : 0u;
  P.amap = P.ctx_word ? d->d_acap + d->t.acap_rows.size() : nullptr;
  P.nul = d->nul ? 1u : 0u;
  P.wstart = d->wstart && env_u64("UGPU_WSTART", 1) != 0 ? 1u : 0u;
  P.bol0 = 1;
  // chain bytes one stitch merge may cross before the chains count as not
  // resynchronising (two chains of a resynchronising table meet within a match
  // or two; longer merges go to the forest FIND)
  P.merge_budget = env_u64("UGPU_MERGE_BUDGET", 4096);
  const uint8_t* ft = d->lb ? d->lb_ft : d->t.ft;
  for (int i = 0; i < 5; ++i)
    P.ft[i] = (uint32_t)ft[4 * i] | ((uint32_t)ft[4 * i + 1] << 8) | ((uint32_t)ft[4 * i + 2] << 16) |
              ((uint32_t)ft[4 * i + 3] << 24);
  P.lb_cls = d->lb ? d->d_lbcls : nullptr;
  P.dom = d->d_dom;
  P.look = d->d_look;
  P.dom_all = d->d_dom && d->t.dom_all ? 1u : 0u;
  if (d->lb) P.wstart = 0;  // (the candidates are needle positions, not match starts)
}

// Translate a byte range of dbuf into the 16-byte aligned base coordinates
// the kernels use, and fix the geometry: `unit`-byte tiles, dealt in equal
// contiguous runs to at most max_rec chain records (per = records per block).
void geometry(ScanParams& P, const uint8_t* dbuf, uint64_t lo, uint64_t hi, uint64_t read_end, int max_rec,
              uint32_t unit, uint32_t per, uint64_t& off)
{
  off = reinterpret_cast<uintptr_t>(dbuf) & 15u;
  P.g = dbuf - off;
  P.lo = lo + off;
  P.hi = hi + off;
  P.rend = read_end + off;
  const uint64_t t0 = P.lo / unit;
  uint64_t t1 = (P.hi + unit - 1) / unit;
  if (t1 <= t0) t1 = t0 + 1;
  const uint64_t nt = t1 - t0;
  uint64_t nrec = nt < (uint64_t)max_rec ? nt : (uint64_t)max_rec;
  if (nrec == 0) nrec = 1;
  // the kernels address a record's bytes with 32-bit offsets
  const uint64_t min_rec = (nt * unit + kMaxRecBytes - 1) / kMaxRecBytes;
  if (nrec < min_rec) nrec = min_rec < nt ? min_rec : nt;
  const uint64_t tpr = (nt + nrec - 1) / nrec;
  nrec = (nt + tpr - 1) / tpr;
  const uint64_t grid = (nrec + per - 1) / per;
  P.bob = off;  // dbuf[0]: the buffer's first byte (option W: at_wb there)
  P.t0 = t0;
  P.t1 = t1;
  P.tpb = tpr;
  P.unit = unit;
  P.grid = (uint32_t)grid;
  P.nrec = (uint32_t)(grid * per);
  P.max_rounds = fix_rounds_for(P);
}

void geometry_for(ScanParams& P, const ugpu_scanner* s, const uint8_t* dbuf, uint64_t lo, uint64_t hi,
                  uint64_t read_end, uint64_t& off, bool xi = false)
{
  if (s->word)
    geometry(P, dbuf, lo, hi, read_end, s->word_rec, wfind_unit(), wfind_waves(), off);
  else if (xi && s->xc)
    geometry(P, dbuf, lo, hi, read_end, s->xi_rec, xc_unit(s->xu), xc_waves(), off);
  else if (xi && s->xg)
    geometry(P, dbuf, lo, hi, read_end, s->xi_rec, xg_unit(), xg_waves(), off);
  else if (xi)
    geometry(P, dbuf, lo, hi, read_end, s->xi_rec, xi_unit(), xi_waves(), off);
  else if (s->sparse)
    geometry(P, dbuf, lo, hi, read_end, s->max_rec, kWaveTile, kSpWaves, off);
  else
    geometry(P, dbuf, lo, hi, read_end, s->max_rec, dense_unit(s->dfa->t.format), dense_waves(s->dfa->t.format), off);
}

hipError_t launch_main(const ugpu_scanner* s, const ScanParams& P, bool write, hipStream_t st, bool xi = false)
{
  if (s->word) return launch_wfind(P, s->dfa->t.format, write, st);
  if (xi && s->xc) return launch_xc(P, write, st);
  if (xi && s->xg) return launch_xg(P, st);
  if (xi) return launch_xi(P, s->xi_smem, st);
  if (s->sparse) return launch_sparse(P, write, s->smem, st);
  return launch_dense(P, s->dfa->t.format, write, s->smem, st);
}

bool is_device_ptr(const void* p)
{
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

void forest_free(ugpu_scanner* s)
{
  (void)hipFree(s->d_fex);
  (void)hipFree(s->d_fvar);
  (void)hipFree(s->d_fent);
  (void)hipFree(s->d_fsum);
  (void)hipFree(s->d_fbase);
  s->d_fex = nullptr;
  s->d_fvar = s->d_fent = s->d_fsum = s->d_fbase = nullptr;
  s->f_cap = 0;
}

// Forest FIND over chain positions [entry, P.hi) of P's buffer (COUNT, or
// WRITE into P.out_*), synchronously; totals and flags land in h_tot / h_flags.
int forest_run(ugpu_scanner* s, ScanParams P, uint64_t entry, bool write, hipStream_t st)
{
  const uint64_t fb = forest_block();
  const uint64_t range = P.hi > entry ? P.hi - entry : 0;
  uint64_t pos = range < kFChunk ? range : kFChunk;
  pos = (pos + fb - 1) / fb * fb;
  if (pos == 0) pos = fb;
  if (pos > s->f_cap) {
    forest_free(s);
    const uint64_t nb = pos / fb;
    hipError_t e;
    if ((e = hipMalloc(&s->d_fex, pos * 4)) != hipSuccess || (e = hipMalloc(&s->d_fvar, 4 * 8)) != hipSuccess ||
        (e = hipMalloc(&s->d_fent, nb * 8)) != hipSuccess || (e = hipMalloc(&s->d_fsum, nb * 24)) != hipSuccess ||
        (e = hipMalloc(&s->d_fbase, nb * 8)) != hipSuccess) {
      forest_free(s);
      return hip_fail(e, "forest scratch");
    }
    s->f_cap = pos;
  }
  UGPU_TRACE("forest entry %llu hi %llu rend %llu write %d\n", (unsigned long long)entry,
             (unsigned long long)P.hi, (unsigned long long)P.rend, (int)write);
  ForestArgs A{};
  A.ex = s->d_fex;
  A.entry = s->d_fvar;
  A.run = s->d_fvar + 1;
  A.bentry = s->d_fent;
  A.bsum = s->d_fsum;
  A.bbase = s->d_fbase;
  P.flags = s->d_flags;
  HIP_TRY(hipMemsetAsync(s->d_flags, 0, sizeof(uint32_t), st));
  HIP_TRY(launch_forest(P, s->dfa->t.format, A, entry, write, s->d_tot, st));
  HIP_TRY(hipMemcpyAsync(s->h_tot, s->d_tot, sizeof(DevTotals), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(s->h_flags, s->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return UGPU_OK;
}

int dfa_on(const ugpu_dfa* d, int dev, const ugpu_dfa** out);

}  // namespace

extern "C" {

int ugpu_device_count(int* n)
{
  if (!n) return fail(UGPU_INVAL, "NULL argument");
  *n = 0;
  HIP_TRY(hipGetDeviceCount(n));
  exit_guard_arm();
  return UGPU_OK;
}

int ugpu_select_device(int dev)
{
  if (exiting()) return UGPU_OK;  // (only releases follow, and they free nothing)
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  exit_guard_arm();
  if (dev < 0 || dev >= n) return fail(UGPU_INVAL, "no such device");
  HIP_TRY(hipSetDevice(dev));
  return UGPU_OK;
}

int ugpu_dfa_create(const uint32_t* opc, uint32_t nop, uint32_t pattern_flags, ugpu_dfa** out)
{
  if (!out) return fail(UGPU_INVAL, "out is NULL");
  if (pattern_flags & ~(UGPU_PAT_WORD | UGPU_PAT_EMPTY)) return fail(UGPU_INVAL, "unknown pattern flags");
  *out = nullptr;
  ugpu_dfa* d = new (std::nothrow) ugpu_dfa();
  if (!d) return fail(UGPU_NOMEM, "host allocation");
  std::string err;
  int rc = build_tables(opc, nop, d->t, err);
  if (rc != 0) {
    delete d;
    return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  }
  const DfaPlan pl = dfa_plan(d->t, pattern_flags);
  if (!pl.ok) {
    delete d;
    return fail(UGPU_UNSUPPORTED, "option W with line anchors, empty matches or negative patterns");
  }
  hipError_t e = hipGetDevice(&d->device);
  if (e != hipSuccess) {
    delete d;
    return hip_fail(e, "hipGetDevice");
  }
  exit_guard_arm();
  d->opc.assign(opc, opc + nop);
  d->plan = pl;
  d->pflags = pattern_flags;
  d->nul = pl.nul;
  d->amode = pl.amode;
  d->wplus = pl.wplus;
  d->wsparse = pl.wsparse;
  d->xcw = pl.xcw;
  // option W: every match begins where at_wb holds (lib/matcher.cpp:107);
  // word-boundary tables: when no state accepts in a context without CTX_WB
  if (pattern_flags & UGPU_PAT_WORD) {
    d->wstart = !d->amode;
  } else if (d->amode && d->t.ctx_word && d->t.format != FMT_WIDE) {
    // a candidate right after a letter has WB = 0 and BW = whether its first
    // character is a word character: droppable when no state accepts in such
    // a context.  BW = 1 for every first byte of the pattern that is an ASCII
    // word byte; any other first byte (non-ASCII included) may give BW = 0.
    auto asc_word = [](uint32_t b) {
      return (b >= '0' && b <= '9') || (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == '_';
    };
    bool bw0 = false;
    for (uint32_t b = 0; b < 256 && !bw0; ++b) {
      const uint32_t col = d->t.format == FMT_BYTE ? b : d->t.cls[b];
      if (d->t.trans[d->t.start + col] != 0 && !asc_word(b)) bw0 = true;
    }
    bool any = false;
    for (size_t i = 0; i < d->t.acap.size() && !any; ++i) {
      const uint32_t c = (uint32_t)(i & 63);
      any = !(c & CTX_WB) && ((c & CTX_BW) || bw0) && d->t.acap[i] != 0;
    }
    d->wstart = !any && !d->t.acap.empty();
  }
  const uint32_t* lbcls = pl.lb_cls;
  if (pl.lb) {
    // the prefilter over the strings of N (tables.cpp needle_filter)
    d->lb = true;
    std::copy(pl.lb_ft, pl.lb_ft + 20, d->lb_ft);
  }
  const size_t n = d->t.trans.size();
  d->ntrans_pad = (uint32_t)((n + 7) & ~size_t(7));
  std::vector<uint16_t> tr(d->ntrans_pad, 0);
  std::copy(d->t.trans.begin(), d->t.trans.end(), tr.begin());
  if ((e = hipMalloc(&d->d_trans, tr.size() * 2)) != hipSuccess ||
      (e = hipMalloc(&d->d_cls, 512)) != hipSuccess ||  // cls, then the xc byte classes
      (e = hipMalloc(&d->d_caps, d->t.caps.size() * 4)) != hipSuccess ||
      (e = hipMemcpy(d->d_trans, tr.data(), tr.size() * 2, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(d->d_cls, d->t.cls.data(), 256, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(d->d_cls + 256, d->t.xc ? d->t.xc_tab.data() : d->t.cls.data(), 256, hipMemcpyHostToDevice)) !=
          hipSuccess ||
      (e = hipMemcpy(d->d_caps, d->t.caps.data(), d->t.caps.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
    ugpu_dfa_destroy(d);
    return hip_fail(e, "table upload");
  }
  if (d->lb && ((e = hipMalloc(&d->d_lbcls, 32)) != hipSuccess ||
                (e = hipMemcpy(d->d_lbcls, lbcls, 32, hipMemcpyHostToDevice)) != hipSuccess)) {
    ugpu_dfa_destroy(d);
    return hip_fail(e, "loop class upload");
  }
  if (d->t.lookahead &&
      ((e = hipMalloc(&d->d_look, d->t.look.size() * 4)) != hipSuccess ||
       (e = hipMemcpy(d->d_look, d->t.look.data(), d->t.look.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)) {
    ugpu_dfa_destroy(d);
    return hip_fail(e, "lookahead upload");
  }
  // (UGPU_DOM=0: no dominated-restart skips; testing)
  const char* domenv = std::getenv("UGPU_DOM");
  if (!d->t.dom.empty() && !(domenv && domenv[0] == '0') &&
      ((e = hipMalloc(&d->d_dom, d->t.dom.size() * 4)) != hipSuccess ||
       (e = hipMemcpy(d->d_dom, d->t.dom.data(), d->t.dom.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)) {
    ugpu_dfa_destroy(d);
    return hip_fail(e, "dominance upload");
  }
  if (d->t.format == FMT_WIDE &&
      ((e = hipMalloc(&d->d_trans32, d->t.trans32.size() * 4)) != hipSuccess ||
       (e = hipMemcpy(d->d_trans32, d->t.trans32.data(), d->t.trans32.size() * 4, hipMemcpyHostToDevice)) !=
           hipSuccess)) {
    ugpu_dfa_destroy(d);
    return hip_fail(e, "wide table upload");
  }
  if (d->amode &&
      ((e = hipMalloc(&d->d_acap, d->t.ctx_word ? (d->t.acap_rows.size() + d->t.acap_map.size()) * 4
                                                : d->t.acap.size() * 4)) != hipSuccess ||
       (e = d->t.ctx_word
                ? hipMemcpy(d->d_acap, d->t.acap_rows.data(), d->t.acap_rows.size() * 4, hipMemcpyHostToDevice)
                : hipMemcpy(d->d_acap, d->t.acap.data(), d->t.acap.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
       (d->t.ctx_word &&
        (e = hipMemcpy(d->d_acap + d->t.acap_rows.size(), d->t.acap_map.data(), d->t.acap_map.size() * 4,
                       hipMemcpyHostToDevice)) != hipSuccess))) {
    // the per-context accepts; every scan runs the context walk (no transducers)
    ugpu_dfa_destroy(d);
    return hip_fail(e, "context accept upload");
  }
  if (pl.wtab || (d->amode && d->t.ctx_word)) {
    // (option W, and word-boundary meta edges: both test Unicode word characters)
    std::vector<uint32_t> wt;
    ugpu_word_ranges(wt);
    d->nwtab = (uint32_t)(wt.size() / 2);
    if ((e = hipMalloc(&d->d_wtab, wt.size() * 4)) != hipSuccess ||
        (e = hipMemcpy(d->d_wtab, wt.data(), wt.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
      ugpu_dfa_destroy(d);
      return hip_fail(e, "word table upload");
    }
  }
  if (pl.xtrans) {
    std::vector<uint16_t> xt(d->ntrans_pad, 0);
    std::copy(d->t.xtrans.begin(), d->t.xtrans.end(), xt.begin());
    if ((e = hipMalloc(&d->d_xtrans, xt.size() * 2)) != hipSuccess ||
        (e = hipMemcpy(d->d_xtrans, xt.data(), xt.size() * 2, hipMemcpyHostToDevice)) != hipSuccess) {
      ugpu_dfa_destroy(d);
      return hip_fail(e, "transducer table upload");
    }
  }
  if (pl.xid) {
    if ((e = hipMalloc(&d->d_xid, d->t.xid.size())) != hipSuccess ||
        (e = hipMemcpy(d->d_xid, d->t.xid.data(), d->t.xid.size(), hipMemcpyHostToDevice)) != hipSuccess) {
      ugpu_dfa_destroy(d);
      return hip_fail(e, "immediate transducer upload");
    }
  }
  if (pl.xu) {
    if ((e = hipMalloc(&d->d_xu, kXuTab + 4 * kXuBm3)) != hipSuccess ||
        (e = hipMemcpy(d->d_xu, d->t.xu_tab.data(), kXuTab, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(d->d_xu + kXuTab, d->t.xu_bm3.data(), 4 * kXuBm3, hipMemcpyHostToDevice)) != hipSuccess) {
      ugpu_dfa_destroy(d);
      return hip_fail(e, "code-point run table upload");
    }
  }
  if (pl.xg) {
    // device form: the class-major product table (tables.hpp xg2), padded to 8 entries
    std::vector<uint16_t> xg((d->t.xg2.size() + 7) & ~size_t(7), 0);
    std::copy(d->t.xg2.begin(), d->t.xg2.end(), xg.begin());
    if ((e = hipMalloc(&d->d_xg, xg.size() * 2)) != hipSuccess ||
        (e = hipMemcpy(d->d_xg, xg.data(), xg.size() * 2, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMalloc(&d->d_xg_sync, 512)) != hipSuccess ||
        (e = hipMemcpy(d->d_xg_sync, d->t.xg_sync.data(), 256, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(d->d_xg_sync + 256, d->t.xg2_cls.data(), 256, hipMemcpyHostToDevice)) != hipSuccess) {
      ugpu_dfa_destroy(d);
      return hip_fail(e, "gap transducer upload");
    }
  }
  *out = d;
  return UGPU_OK;
}

int ugpu_dfa_destroy(ugpu_dfa* d)
{
  if (!d || exiting()) return UGPU_OK;
  for (ugpu_dfa* r : d->reps) {
    if (r) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(r->device);
      ugpu_dfa_destroy(r);
      (void)hipSetDevice(cur);
    }
  }
  for (ugpu_scanner* s : d->pool) ugpu_scanner_destroy(s);
  for (ugpu_scanner* s : d->pool_w) ugpu_scanner_destroy(s);
  if (d->d_trans) (void)hipFree(d->d_trans);
  if (d->d_trans32) (void)hipFree(d->d_trans32);
  if (d->d_xtrans) (void)hipFree(d->d_xtrans);
  if (d->d_wtab) (void)hipFree(d->d_wtab);
  if (d->d_xid) (void)hipFree(d->d_xid);
  if (d->d_xg) (void)hipFree(d->d_xg);
  if (d->d_xu) (void)hipFree(d->d_xu);
  if (d->d_xg_sync) (void)hipFree(d->d_xg_sync);
  if (d->d_cls) (void)hipFree(d->d_cls);
  if (d->d_caps) (void)hipFree(d->d_caps);
  if (d->d_acap) (void)hipFree(d->d_acap);
  if (d->d_lbcls) (void)hipFree(d->d_lbcls);
  if (d->d_dom) (void)hipFree(d->d_dom);
  if (d->d_look) (void)hipFree(d->d_look);
  delete d;
  return UGPU_OK;
}

extern const char* ugpu_build_id_str;  // (build/build_id.cpp, written by the Makefile)
const char* ugpu_build_id(void) { return ugpu_build_id_str; }

int ugpu_dfa_info_get(const ugpu_dfa* d, ugpu_dfa_info* info)
{
  if (!d || !info) return fail(UGPU_INVAL, "NULL argument");
  // (the plan the tables were uploaded with -- lookback and option-W route,
  // whatever UGPU_LB / UGPU_WSPARSE / UGPU_WFAST say now)
  dfa_info_fill(d->t, d->plan, info);
  return UGPU_OK;
}

namespace {
int scanner_create(const ugpu_dfa* dfa, ugpu_scanner** out, bool prefer_write);
}

int ugpu_scanner_create(const ugpu_dfa* dfa, ugpu_scanner** out) { return scanner_create(dfa, out, false); }

int ugpu_scanner_create_ex(const ugpu_dfa* dfa, uint32_t flags, ugpu_scanner** out)
{
  if (flags & ~UGPU_SCANNER_RECORDS) return fail(UGPU_INVAL, "unknown scanner flags");
  return scanner_create(dfa, out, (flags & UGPU_SCANNER_RECORDS) != 0);
}

namespace {

// prefer_write: code-point run tables take xc_kernel's U mode, which writes
// its own records, also where xg_kernel (no record pass: OFFSETS rebuilt on
// dense_kernel) counts a little faster -- the choice of a records consumer
int scanner_create(const ugpu_dfa* dfa, ugpu_scanner** out, bool prefer_write)
{
  if (!dfa || !out) return fail(UGPU_INVAL, "NULL argument");
  *out = nullptr;
  {
    // the table copy on the calling thread's device (ugpu_select_device)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(UGPU_DEVICE, "hipGetDevice");
    const int rc = dfa_on(dfa, dev, &dfa);
    if (rc) return rc;
  }
  ugpu_scanner* s = new (std::nothrow) ugpu_scanner();
  if (!s) return fail(UGPU_NOMEM, "host allocation");
  s->pref_write = prefer_write;
  s->dfa = dfa;
  // every failure below releases what was allocated so far
#define HIP_TRY_S(expr)                      \
  do {                                       \
    hipError_t _e = (expr);                  \
    if (_e != hipSuccess) {                  \
      const int _rc = hip_fail(_e, #expr);   \
      ugpu_scanner_destroy(s);               \
      return _rc;                            \
    }                                        \
  } while (0)
  HIP_TRY_S(hipGetDevice(&s->device));
  // option W: prefiltered tables keep sparse_kernel (its candidate walks check
  // the W rules); every other table runs wfind_kernel (tables through the caches)
  // line anchors / option N: every scan runs the context walk on wfind_kernel
  // wide tables: the exact walk on wfind_kernel, transitions from global memory
  // context accepts (word boundaries, line anchors) on a prefiltered table:
  // sparse_kernel's candidate walks run the context walk, the
  // prefilter's candidates stay a superset; without a prefilter (or with
  // UGPU_SPARSE=0) wfind_kernel's chain of context walks
  // (option W: also loop-needle tables and DfaPlan::wsparse; UGPU_SPARSE=0:
  // wfind_kernel, which applies the W rules)
  const char* senv0 = std::getenv("UGPU_SPARSE");
  const bool sp_off = senv0 && senv0[0] == '0';
  const bool ctx_sparse = dfa->amode && dfa->t.filter && dfa->t.format == FMT_BYTE && !sp_off;
  const bool w_sparse = (dfa->t.filter || dfa->lb || dfa->wsparse) && dfa->t.format == FMT_BYTE && !sp_off;
  // lookahead tables: the lookahead walk (kWalkLook) on wfind_kernel
  if ((dfa->amode && !ctx_sparse) || dfa->t.format == FMT_WIDE || dfa->t.lookahead ||
      (dfa->d_wtab && !dfa->amode && !w_sparse)) {
    const uint32_t nacap = !dfa->amode ? dfa->t.states
                           : dfa->t.ctx_word ? (uint32_t)dfa->t.acap_rows.size() : (uint32_t)dfa->t.acap.size();
    const uint32_t nmap = dfa->amode && dfa->t.ctx_word ? dfa->t.states : 0u;
    if (wfind_smem_bytes(dfa->ntrans_pad, dfa->t.states, dfa->nwtab, nacap, nmap) > 160 * 1024) {
      delete s;
      return fail(UGPU_UNSUPPORTED, "tables do not fit in LDS");
    }
    s->word = true;
    s->word_rec = kMaxRec;
    if (const char* env = std::getenv("UGPU_MAX_GRID")) {
      int v = std::atoi(env);
      if (v >= 1 && v <= kMaxRec) s->word_rec = v;
    }
    s->max_rec = s->word_rec;
  }
  if (s->word && dfa->wplus) {
    // \w+ under option W: set up the non-W kernels too; ugpu_scan picks per scan
    s->word = false;
    s->wfast = true;
  } else if (s->word && dfa->xcw) {
    s->word = false;  // xc_kernel with the W rules; wfind_kernel when it flags non-ASCII bytes
    s->wxc = true;
  }
  if (s->word) {
    HIP_TRY_S(hipMalloc(&s->d_recs, sizeof(BlockRec) * kMaxRec));
    HIP_TRY_S(hipMalloc(&s->d_entries, sizeof(uint64_t) * kMaxRec));
    HIP_TRY_S(hipMalloc(&s->d_obase, sizeof(uint64_t) * kMaxRec));
    HIP_TRY_S(hipMalloc(&s->d_fix, sizeof(uint64_t) * kMaxRec));
    HIP_TRY_S(hipMalloc(&s->d_tot, sizeof(DevTotals)));
    HIP_TRY_S(hipMalloc(&s->d_flags, sizeof(uint32_t)));
    HIP_TRY_S(hipHostMalloc(&s->h_tot, sizeof(DevTotals)));
    HIP_TRY_S(hipHostMalloc(&s->h_flags, sizeof(uint32_t)));
    HIP_TRY_S(hipEventCreate(&s->ev0));
    HIP_TRY_S(hipEventCreate(&s->ev1));
    *out = s;
    return UGPU_OK;
  }
  // (UGPU_SPARSE=0: prefiltered tables take the dense-pattern kernels; testing)
  const char* senv = std::getenv("UGPU_SPARSE");
  s->sparse = (dfa->t.filter || dfa->lb || dfa->wsparse) && dfa->t.format == FMT_BYTE && !(senv && senv[0] == '0');
  s->smem = s->sparse ? sparse_smem_bytes(dfa->ntrans_pad, dfa->t.states, acap_lds_n(dfa))
                      : dense_smem_bytes(dfa->t.format, dfa->ntrans_pad, dfa->t.states);
  if (s->smem > 160 * 1024) {
    delete s;
    return fail(UGPU_UNSUPPORTED, "tables do not fit in LDS");
  }
  int per_cu = 0;
  if (s->sparse) {
    ScanParams probe{};
    HIP_TRY_S(sparse_occupancy(probe, s->smem, &per_cu));
  } else {
    HIP_TRY_S(dense_occupancy(dfa->t.format, dfa->t.cap1 != 0, dfa->d_xtrans != nullptr, s->smem, &per_cu));
  }
  hipDeviceProp_t prop;
  HIP_TRY_S(hipGetDeviceProperties(&prop, s->device));
  if (per_cu < 1) per_cu = 1;
  int g = prop.multiProcessorCount * per_cu * (s->sparse ? kSpWaves : dense_waves(dfa->t.format));
  if (g > kMaxRec) g = kMaxRec;
  s->max_rec = g;
  if (const char* env = std::getenv("UGPU_MAX_GRID")) {
    int v = std::atoi(env);
    if (v >= 1 && v <= kMaxRec) s->max_rec = v;
  }
  // immediate tables: COUNT scans on xi_kernel (UGPU_XI=0 keeps the dense kernel);
  // gap tables: xg_kernel (UGPU_XG=0 keeps the dense kernel)
  const char* xenv = std::getenv("UGPU_XI");
  const char* genv = std::getenv("UGPU_XG");
  if (!s->sparse && !(dfa->d_xid && !(xenv && xenv[0] == '0')) && dfa->d_xg && !(genv && genv[0] == '0')) {
    int gpc = 0;
    HIP_TRY_S(xg_occupancy((uint32_t)((dfa->t.xg2.size() + 7) & ~size_t(7)), &gpc));
    if (gpc >= 1) {
      s->xg = true;
      int gg = prop.multiProcessorCount * gpc * (int)xg_waves();
      s->xi_rec = gg > kMaxRec ? kMaxRec : gg;
      if (const char* env = std::getenv("UGPU_MAX_GRID")) {
        int v = std::atoi(env);
        if (v >= 1 && v <= kMaxRec) s->xi_rec = v;
      }
    }
  }
  if (!s->sparse && dfa->d_xid && !(xenv && xenv[0] == '0')) {
    s->xi_smem = (size_t)dfa->t.xid_rows * 256;
    int xpc = 0;
    HIP_TRY_S(xi_occupancy(s->xi_smem, &xpc));
    if (xpc >= 1) {
      s->xi = true;
      int xg = prop.multiProcessorCount * xpc * (int)xi_waves();
      s->xi_rec = xg > kMaxRec ? kMaxRec : xg;
      if (const char* env = std::getenv("UGPU_MAX_GRID")) {
        int v = std::atoi(env);
        if (v >= 1 && v <= kMaxRec) s->xi_rec = v;
      }
    }
  }
  // two-state tables: COUNT scans on xc_kernel, ahead of xi/xg (UGPU_XC=0
  // keeps those)
  const char* uenv = std::getenv("UGPU_XU");
  // option W on \w+ (wfast): U mode checks the run edges itself, one pass
  // instead of isutf8 + xg_kernel (UGPU_XUW=0 keeps those)
  const char* wuenv = std::getenv("UGPU_XUW");
  const bool wu = s->wfast && dfa->d_xu && !(wuenv && wuenv[0] == '0') && !(uenv && uenv[0] == '0');
  const bool xu = dfa_xu(dfa) || wu ||
                  (prefer_write && dfa->d_xu && (!dfa->d_wtab || dfa->wplus) && !(uenv && uenv[0] == '0'));
  if (!s->sparse && (dfa_xc(dfa) || xu)) {
    int cpc = 0;
    HIP_TRY_S(xc_occupancy(xu, &cpc));
    if (cpc >= 1) {
      s->xc = true;
      s->xu = xu;
      s->wu = wu;
      s->xu_xi = s->xi;
      s->xu_xg = s->xg;
      s->xi = s->xg = false;
      const int cg = prop.multiProcessorCount * cpc * (int)xc_waves();
      s->xi_rec = cg > kMaxRec ? kMaxRec : cg;
      if (const char* env = std::getenv("UGPU_MAX_GRID")) {
        int v = std::atoi(env);
        if (v >= 1 && v <= kMaxRec) s->xi_rec = v;
      }
    }
  }
  HIP_TRY_S(hipMalloc(&s->d_recs, sizeof(BlockRec) * kMaxRec));
  HIP_TRY_S(hipMalloc(&s->d_entries, sizeof(uint64_t) * kMaxRec));
  HIP_TRY_S(hipMalloc(&s->d_obase, sizeof(uint64_t) * kMaxRec));
  HIP_TRY_S(hipMalloc(&s->d_fix, sizeof(uint64_t) * kMaxRec));
  if (s->sparse) {
    HIP_TRY_S(hipMalloc(&s->d_open, sizeof(OpenRec) * kMaxRec));
    HIP_TRY_S(hipMalloc(&s->d_susp, sizeof(uint32_t) * kMaxRec));
    HIP_TRY_S(hipMalloc(&s->d_srec, sizeof(SuspRec) * kMaxRec));
  }
  HIP_TRY_S(hipMalloc(&s->d_tot, sizeof(DevTotals)));
  HIP_TRY_S(hipMalloc(&s->d_flags, sizeof(uint32_t)));
  HIP_TRY_S(hipHostMalloc(&s->h_tot, sizeof(DevTotals)));
  HIP_TRY_S(hipHostMalloc(&s->h_flags, sizeof(uint32_t)));
  HIP_TRY_S(hipEventCreate(&s->ev0));
  HIP_TRY_S(hipEventCreate(&s->ev1));
  *out = s;
  return UGPU_OK;
#undef HIP_TRY_S
}

}  // namespace

int ugpu_scanner_destroy(ugpu_scanner* s)
{
  if (!s || exiting()) return UGPU_OK;
  (void)hipFree(s->d_recs);
  (void)hipFree(s->d_entries);
  (void)hipFree(s->d_obase);
  (void)hipFree(s->d_inbits);
  (void)hipFree(s->d_fix);
  (void)hipFree(s->d_open);
  (void)hipFree(s->d_susp);
  (void)hipFree(s->d_srec);
  (void)hipFree(s->d_tot);
  (void)hipFree(s->d_flags);
  (void)hipHostFree(s->h_tot);
  (void)hipHostFree(s->h_flags);
  forest_free(s);
  (void)hipFree(s->d_st_start);
  (void)hipFree(s->d_st_len);
  (void)hipFree(s->d_st_cap);
  (void)hipFree(s->d_st_n);
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  delete s;
  return UGPU_OK;
}

int ugpu_scan(ugpu_scanner* s, const uint8_t* dbuf, uint64_t lo, uint64_t hi, uint64_t read_end, int at_eof,
              uint64_t bias, void* stream)
{
  if (!s || !dbuf) return fail(UGPU_INVAL, "NULL argument");
  if (lo > hi || hi > read_end) return fail(UGPU_INVAL, "need lo <= hi <= read_end");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s->wxc) s->word = false;
  if (s->wfast) {
    // option W on \w+: matches are maximal runs of Word code points, so on valid
    // UTF-8 at_wb/at_we hold at every match edge -- provided the
    // chain enters at the buffer start or after an ASCII non-word byte
    bool fast = !s->wforce;
    if (fast && lo > 0) {
      uint8_t b = 0;
      HIP_TRY(hipMemcpyAsync(&b, dbuf + lo - 1, 1, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      fast = b == '\n' || (b < 0x80 && b != '_' && !((b | 0x20u) - 'a' < 26u) && !(b - '0' < 10u));
    }
    // isutf8 over [lo, read_end) first (run beside the scan on a second stream
    // it gained nothing: the two kernels slowed each other down)
    if (fast && read_end > lo && !s->wu) {
      uint64_t bad = ~0ull;
      const int rc = utf8_scan(dbuf + lo, read_end - lo, false, &bad, stream);
      if (rc) return rc;
      fast = bad == ~0ull;
    }
    s->word = !fast;
  }
  ScanParams P{};
  fill_tables(P, s->dfa);
  P.xu_tab = s->xu ? s->dfa->d_xu : nullptr;  // (the scanner's U mode choice)
  P.xu_w = s->wu && !s->word ? 1u : 0u;
  P.xu_exact = s->xu_exact ? 1u : 0u;
  P.bol0 = s->bol0;
  if (s->wfast && !s->word) P.wtab = nullptr, P.nwtab = 0;  // the non-W kernels, stitches and forest
  geometry_for(P, s, dbuf, lo, hi, read_end, s->off, s->xi || s->xg || s->xc);
  P.delta = (int64_t)bias - (int64_t)s->off;
  P.at_eof = at_eof ? 1u : 0u;
  if (const char* ab = std::getenv("UGPU_ABLATE")) P.ablate = (uint32_t)std::atoi(ab);
  P.recs = s->d_recs;
  P.flags = s->d_flags;
  P.totals = s->d_tot;
  P.entries_out = s->d_entries;
  P.out_base_out = s->d_obase;
  // sparse_kernel walks stop at their wave's range end (open walks, resolved
  // by fix_kernel): a long match costs each wave its own bytes only
  // (UGPU_TRUNC=0: walks run to the readable end)
  static const bool trunc = env_u64("UGPU_TRUNC", 1) != 0;
  P.open = s->sparse && !P.wtab && !P.acap && trunc ? s->d_open : nullptr;
  // walks longer than their window: the wave suspends, a resume launch of
  // the kernel completes it (coop_walk); option W and the context walks keep
  // their per-lane walks
  P.susp = s->sparse && !P.wtab && !P.acap ? s->d_susp : nullptr;
  P.srec = P.susp ? s->d_srec : nullptr;
  s->staged_last = false;
  if (s->sparse && (s->stage || s->stage_once)) {
    if (!s->d_st_n) {
      // all four or none (a partial failure frees what it got)
      const size_t n = (size_t)kMaxRec * kStagePer;
      uint64_t* a = nullptr;
      uint32_t *b = nullptr, *c = nullptr, *d = nullptr;
      hipError_t e = hipMalloc(&a, n * 8);
      if (e == hipSuccess) e = hipMalloc(&b, n * 4);
      if (e == hipSuccess) e = hipMalloc(&c, n * 4);
      if (e == hipSuccess) e = hipMalloc(&d, kMaxRec * 4);
      if (e != hipSuccess) {
        (void)hipFree(a);
        (void)hipFree(b);
        (void)hipFree(c);
        (void)hipFree(d);
        (void)hipGetLastError();
        return fail(UGPU_NOMEM, "staging buffers");
      }
      s->d_st_start = a;
      s->d_st_len = b;
      s->d_st_cap = c;
      s->d_st_n = d;
    }
    P.st_start = s->d_st_start;
    P.st_len = s->d_st_len;
    P.st_cap = s->d_st_cap;
    P.st_n = s->d_st_n;
    P.st_per = kStagePer;
    s->staged_last = true;
  }
  s->stage_once = false;
  P.inbits = nullptr;
  // (default on, round 4: with the expansion's coalesced length stores and
  // 12-byte records, C4 OFFSETS 6.4 ms against 8.1 ms for the WRITE pass, C3
  // 9.8 against 11.7 ms, profiles/r04_offsets_ab.txt; UGPU_XC_BITMAP=0 restores it)
  if (s->pref_write && s->xc && !s->word && !P.xc_w && !P.xu_w && env_u64("UGPU_XC_BITMAP", 1) != 0) {
    // one bit per byte up to the chunk after the readable end (the last wave
    // searches for the exit up to there)
    const uint64_t need = ((((P.rend + 15) & ~uint64_t(15)) + 2048) >> 3) + 64;
    if (need > s->inbits_cap) {
      (void)hipFree(s->d_inbits);
      s->d_inbits = nullptr;
      s->inbits_cap = 0;
      if (hipMalloc(&s->d_inbits, need + need / 8) == hipSuccess)
        s->inbits_cap = need + need / 8;
      else
        (void)hipGetLastError();  // (no bitmap: OFFSETS runs the WRITE pass)
    }
    if (s->d_inbits) P.inbits = s->d_inbits;
  }
  UGPU_TRACE("scan lo %llu hi %llu rend %llu eof %d grid %u xi %d xg %d sparse %d word %d\n", (unsigned long long)P.lo,
             (unsigned long long)P.hi, (unsigned long long)P.rend, at_eof, P.grid, (int)s->xi, (int)s->xg,
             (int)s->sparse, (int)s->word);
  HIP_TRY(hipMemsetAsync(s->d_flags, 0, sizeof(uint32_t), st));
  HIP_TRY(hipEventRecord(s->ev0, st));
  HIP_TRY(launch_main(s, P, false, st, s->xi || s->xg || s->xc));
  HIP_TRY(hipEventRecord(s->ev1, st));
  HIP_TRY(launch_fix(P, s->dfa->t.format, st));
  HIP_TRY(hipMemcpyAsync(s->h_tot, s->d_tot, sizeof(DevTotals), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(s->h_flags, s->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  s->last = P;
  s->last_xi = !s->word && (s->xi || s->xg || s->xc);
  s->last_xc = !s->word && s->xc;
  s->last_buf = dbuf;
  s->last_args[0] = lo;
  s->last_args[1] = hi;
  s->last_args[2] = read_end;
  s->last_args[3] = at_eof ? 1u : 0u;
  s->last_args[4] = bias;
  s->stream = st;
  s->have_scan = true;
  s->forest = false;
  return UGPU_OK;
}

int ugpu_scanner_context(ugpu_scanner* s, int bol0)
{
  if (!s) return fail(UGPU_INVAL, "NULL argument");
  s->bol0 = bol0 ? 1u : 0u;
  return UGPU_OK;
}

int ugpu_scan_totals(ugpu_scanner* s, ugpu_totals* out)
{
  if (!s || !out) return fail(UGPU_INVAL, "NULL argument");
  if (!s->have_scan) return fail(UGPU_INVAL, "no scan issued");
  HIP_TRY(hipStreamSynchronize(s->stream));
  if (s->last_xc && s->xu && (*s->h_flags & UGPU_FLAG_UMIX)) {
    // U mode's fast kernel met an XU_MIX or XU_SLOW lead: redo the range with
    // the exact U kernel (which flags UGPU_FLAG_USLOW for 4-byte tokens)
    // (and keeps it for the scanner's later scans: inputs with such leads
    // usually have many)
    s->xu_exact = true;
    const int rc = ugpu_scan(s, s->last_buf, s->last_args[0], s->last_args[1], s->last_args[2],
                             (int)s->last_args[3], s->last_args[4], s->stream);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
  }
  if (s->wu && !s->word && (*s->h_flags & (UGPU_FLAG_WSLOW | UGPU_FLAG_USLOW))) {
    // option W on U mode met a stray continuation byte right after a token
    // byte (at_wb may decode a word character there, xc_kernel.hip umask) or a
    // 4-byte token: redo the range with wfind_kernel
    s->wforce = true;
    const int rc = ugpu_scan(s, s->last_buf, s->last_args[0], s->last_args[1], s->last_args[2],
                             (int)s->last_args[3], s->last_args[4], s->stream);
    s->wforce = false;
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
  }
  if (s->wxc && !s->word && (*s->h_flags & UGPU_FLAG_WSLOW)) {
    // option W met bytes >= 0x80 (their at_wb/at_we need the UTF-8 decode):
    // redo the range with wfind_kernel
    s->wxc = false;
    s->word = true;
    const int rc = ugpu_scan(s, s->last_buf, s->last_args[0], s->last_args[1], s->last_args[2],
                             (int)s->last_args[3], s->last_args[4], s->stream);
    s->wxc = true;
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
  }
  if (s->last_xc && (*s->h_flags & UGPU_FLAG_USLOW)) {
    // U mode met a lead byte of a 4-byte token: redo the range with the
    // table's next kernel (xg / xi / dense)
    s->xc = false;
    s->xi = s->xu_xi;
    s->xg = s->xu_xg;
    const int rc = ugpu_scan(s, s->last_buf, s->last_args[0], s->last_args[1], s->last_args[2],
                             (int)s->last_args[3], s->last_args[4], s->stream);
    s->xc = true;
    s->xi = s->xg = false;
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
  }

  UGPU_TRACE("totals flags %u count %llu rounds %u\n", *s->h_flags, (unsigned long long)s->h_tot->count,
             s->h_tot->rounds);
  if ((*s->h_flags & UGPU_FLAG_BUDGET) && !s->forest) {
    // the speculative stitch gave up (chains that do not resynchronise):
    // resolve the same range exactly with the forest FIND
    const int rc = forest_run(s, s->last, s->last.lo, false, s->stream);
    if (rc) return rc;
    s->forest = true;
  }
  const DevTotals& t = *s->h_tot;
  out->count = t.count;
  out->digest = t.digest;
  out->dcap = t.dcap;
  out->entry = t.entry - s->off;
  out->exit = t.exit - s->off;
  out->flags = (*s->h_flags & ~(UGPU_FLAG_WSLOW | UGPU_FLAG_OPEN)) | (s->forest ? UGPU_TOT_FOREST : 0u) |
               ((s->wfast || s->wxc) && !s->word ? UGPU_TOT_WFAST : 0u);
  out->fix_rounds = t.rounds;
  if (out->flags & UGPU_FLAG_HALO) return fail(UGPU_HALO, "a match walked past the readable end of the shard");
  if (out->flags & UGPU_FLAG_BUDGET) return fail(UGPU_UNSUPPORTED, kBudgetMsg);
  return UGPU_OK;
}

int ugpu_scanner_stage(ugpu_scanner* s, int on)
{
  if (!s) return fail(UGPU_INVAL, "NULL argument");
  s->stage = on != 0;
  return UGPU_OK;
}

int ugpu_scan_kernel_ms(ugpu_scanner* s, float* ms)
{
  if (!s || !ms) return fail(UGPU_INVAL, "NULL argument");
  HIP_TRY(hipEventSynchronize(s->ev1));
  HIP_TRY(hipEventElapsedTime(ms, s->ev0, s->ev1));
  return UGPU_OK;
}

int ugpu_scan_offsets(ugpu_scanner* s, uint64_t* d_start, uint32_t* d_len, uint32_t* d_cap, uint64_t capacity,
                      void* stream)
{
  if (!s || !s->have_scan) return fail(UGPU_INVAL, "no scan issued");
  if (!d_cap && (s->dfa->t.cap1 == 0 || s->dfa->t.anchored))
    return fail(UGPU_INVAL, "the table has several accept indices: d_cap is needed");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipStreamSynchronize(s->stream));
  ScanParams P = s->last;
  bool forest = s->forest || (*s->h_flags & UGPU_FLAG_BUDGET);
  if (s->last_xc && !forest) {
    // xc_kernel writes its own records (starts, then lengths from the ends),
    // at the output bases of the COUNT pass's exact records
    P.out_base = s->d_obase;
    P.out_start = d_start;
    P.out_len = d_len;
    P.out_cap = d_cap;
    P.out_capacity = capacity;
    P.out_fix = s->d_fix;
    HIP_TRY(hipMemsetAsync(s->d_flags, 0, sizeof(uint32_t), st));
    if (P.inbits)
      HIP_TRY(launch_xc_expand(P, st, s->h_tot->count));  // (the COUNT pass wrote the In bits)
    else
      HIP_TRY(launch_xc(P, true, st, s->h_tot->count));
    HIP_TRY(hipMemcpyAsync(s->h_flags, s->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (*s->h_flags & UGPU_FLAG_CAPACITY) return fail(UGPU_CAPACITY, "output capacity exceeded");
    if (*s->h_flags & UGPU_FLAG_HALO) return fail(UGPU_HALO, "a match walked past the readable end of the shard");
    return UGPU_OK;
  }
  if (s->last_xi && s->wxc) s->word = true;  // (not reached: xc writes its own W records)
  if (s->last_xi && !forest) {
    // xi_kernel has no record-writing pass: redo the chain records with the
    // dense kernel's geometry (COUNT + fix), then its WRITE pass
    P = ScanParams{};
    fill_tables(P, s->dfa);
    P.bol0 = s->bol0;
    if (s->wfast) P.wtab = nullptr, P.nwtab = 0;  // (only a non-W scan gets here)
    uint64_t off = 0;
    geometry_for(P, s, s->last_buf, s->last_args[0], s->last_args[1], s->last_args[2], off, false);
    P.delta = (int64_t)s->last_args[4] - (int64_t)off;
    P.at_eof = (uint32_t)s->last_args[3];
    P.recs = s->d_recs;
    P.flags = s->d_flags;
    P.totals = s->d_tot;
    P.entries_out = s->d_entries;
    P.out_base_out = s->d_obase;
    HIP_TRY(hipMemsetAsync(s->d_flags, 0, sizeof(uint32_t), st));
    HIP_TRY(launch_main(s, P, false, st));
    HIP_TRY(launch_fix(P, s->dfa->t.format, st));
    HIP_TRY(hipMemcpyAsync(s->h_flags, s->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    forest = (*s->h_flags & UGPU_FLAG_BUDGET) != 0;
  }
  P.entries = s->d_entries;
  P.out_base = s->d_obase;
  P.out_start = d_start;
  P.out_len = d_len;
  P.out_cap = d_cap;
  P.out_capacity = capacity;
  UGPU_TRACE("offsets forest %d capacity %llu staged %d\n", (int)forest, (unsigned long long)capacity,
             (int)s->staged_last);
  if (!forest && s->staged_last && !s->last_xi) {
    // single pass: copy the staged records of waves whose speculative chain was
    // the true one; a WRITE pass (skipping the copied waves) covers the rest
    HIP_TRY(hipMemsetAsync(s->d_flags, 0, sizeof(uint32_t), st));
    HIP_TRY(launch_stage_copy(P, st));
    HIP_TRY(hipMemcpyAsync(s->h_flags, s->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    s->staged_last = false;  // (the staging slots now say which waves are done)
    if (*s->h_flags & UGPU_FLAG_CAPACITY) return fail(UGPU_CAPACITY, "output capacity exceeded");
    if (!(*s->h_flags & UGPU_FLAG_NEEDWRITE)) return UGPU_OK;
  } else {
    P.st_n = nullptr;  // no staged records: every wave writes
  }
  if (!forest) {
    HIP_TRY(hipMemsetAsync(s->d_flags, 0, sizeof(uint32_t), st));
    HIP_TRY(launch_main(s, P, true, st));
    HIP_TRY(hipMemcpyAsync(s->h_flags, s->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    forest = (*s->h_flags & UGPU_FLAG_BUDGET) != 0;  // a lane stitch ran past its round budget
  }
  if (forest) {
    const int rc = forest_run(s, P, P.lo, true, st);
    if (rc) return rc;
  }
  if (*s->h_flags & UGPU_FLAG_CAPACITY) return fail(UGPU_CAPACITY, "output capacity exceeded");
  if (*s->h_flags & UGPU_FLAG_HALO) return fail(UGPU_HALO, "a match walked past the readable end of the shard");
  return UGPU_OK;
}

int ugpu_chain_fix(ugpu_scanner* s, const uint8_t* dbuf, uint64_t lo, uint64_t hi, uint64_t read_end, int at_eof,
                   uint64_t bias, uint64_t old_entry, uint64_t new_entry, ugpu_totals* delta, void* stream)
{
  if (!s || !dbuf || !delta) return fail(UGPU_INVAL, "NULL argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // (option W: the exact W walk -- also for scanners whose scans take the
  // non-W kernels, wfast / wxc; at_wb at lo reads dbuf[lo - 4 .. lo))
  ScanParams P{};
  fill_tables(P, s->dfa);
  P.bol0 = s->bol0;
  uint64_t off = 0;
  geometry_for(P, s, dbuf, lo, hi, read_end, off);
  P.delta = (int64_t)bias - (int64_t)off;
  P.at_eof = at_eof ? 1u : 0u;
  P.totals = s->d_tot;
  HIP_TRY(launch_chain_fix(P, s->dfa->t.format, old_entry + off, new_entry + off, st));
  DevTotals t;
  HIP_TRY(hipMemcpyAsync(&t, s->d_tot, sizeof(DevTotals), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (t.flags & UGPU_FLAG_BUDGET) {
    // the two chains do not meet within the merge budget: the exact chains from
    // both entries by the forest FIND, and their difference
    int rc = forest_run(s, P, new_entry + off, false, st);
    if (rc) return rc;
    const DevTotals tn = *s->h_tot;
    const uint32_t fn = *s->h_flags;
    rc = forest_run(s, P, old_entry + off, false, st);
    if (rc) return rc;
    const DevTotals to = *s->h_tot;
    t.count = tn.count - to.count;
    t.digest = tn.digest - to.digest;
    t.dcap = tn.dcap - to.dcap;
    t.exit = tn.exit == to.exit ? ~0ull : tn.exit;
    t.flags = (fn | *s->h_flags) & UGPU_FLAG_HALO;
    t.rounds = 0;
  }
  delta->count = t.count;
  delta->digest = t.digest;
  delta->dcap = t.dcap;
  delta->entry = new_entry;
  delta->exit = (t.exit == ~0ull) ? ~0ull : t.exit - off;
  delta->flags = t.flags;
  delta->fix_rounds = t.rounds;
  if (t.flags & UGPU_FLAG_HALO) return fail(UGPU_HALO, "a match walked past the readable end of the shard");
  return UGPU_OK;
}

namespace {

// Per-device workspace of ugpu_find_all, pooled (no hipMalloc/hipFree per
// call: hipFree synchronises the device): a private non-blocking stream (calls
// from several host threads do not serialise on the null stream), the device
// copy of a host input and the device match arrays, grown on demand.
// Pinned host memory for a stream's match lists: ugpu_stream_feed copies the
// records there and its ugpu_result borrows the arrays (refs: results still
// alive; a block with live results is not written again).  Blocks live as long
// as the pooled workspace that holds them (the process).
struct PinBlk {
  uint8_t* p = nullptr;
  size_t bytes = 0;             // (a pinned_get block)
  uint64_t cap = 0;             // records
  uint64_t cap_n = 0;           // cap[0 .. cap_n) holds cap_v (single-accept tables: no cap copy)
  uint32_t cap_v = 0;
  std::atomic<int> refs{0};
};

struct FindWs {
  int dev = -1;
  hipStream_t st = nullptr;
  // ugpu_stream: the two device buffers (carry + chunk) and the pinned blocks
  uint8_t* d_sb[2] = {nullptr, nullptr};
  uint64_t sb_cap = 0;  // bytes of each (+ 16 padding allocated)
  PinBlk pin[2];
  uint8_t* d_in = nullptr;
  uint64_t in_cap = 0;
  uint64_t* d_start = nullptr;
  uint32_t* d_len = nullptr;
  uint32_t* d_cap = nullptr;
  uint64_t out_cap = 0;

  hipError_t reserve_in(uint64_t n)
  {
    if (n <= in_cap) return hipSuccess;
    (void)hipFree(d_in);
    d_in = nullptr;
    in_cap = 0;
    const uint64_t c = n + n / 4;
    hipError_t e = hipMalloc(&d_in, c + 16);
    if (e == hipSuccess) in_cap = c;
    return e;
  }
  hipError_t reserve_out(uint64_t n)
  {
    if (n <= out_cap) return hipSuccess;
    (void)hipFree(d_start);
    (void)hipFree(d_len);
    (void)hipFree(d_cap);
    d_start = nullptr;
    d_len = d_cap = nullptr;
    out_cap = 0;
    const uint64_t c = n + n / 4;
    hipError_t e;
    if ((e = hipMalloc(&d_start, c * 8)) != hipSuccess || (e = hipMalloc(&d_len, c * 4)) != hipSuccess ||
        (e = hipMalloc(&d_cap, c * 4)) != hipSuccess)
      return e;
    out_cap = c;
    return hipSuccess;
  }
};

std::mutex g_find_mu;
std::vector<FindWs*> g_find_pool;

FindWs* find_ws_acquire(int dev)
{
  {
    std::lock_guard<std::mutex> lk(g_find_mu);
    for (size_t i = 0; i < g_find_pool.size(); ++i)
      if (g_find_pool[i]->dev == dev) {
        FindWs* w = g_find_pool[i];
        g_find_pool.erase(g_find_pool.begin() + (long)i);
        return w;
      }
  }
  FindWs* w = new (std::nothrow) FindWs;
  if (!w) return nullptr;
  w->dev = dev;
  if (hipStreamCreateWithFlags(&w->st, hipStreamNonBlocking) != hipSuccess) {
    delete w;
    return nullptr;
  }
  exit_guard_arm();
  return w;
}

void find_ws_release(FindWs* w)
{
  std::lock_guard<std::mutex> lk(g_find_mu);
  g_find_pool.push_back(w);
}

// Every ugpu_result is the head of a ResBox: its arrays are malloc()ed, or
// (pin set) borrowed from a pinned block of a stream's workspace
struct ResBox {
  ugpu_result r;
  PinBlk* pin;
};

ugpu_result* result_alloc()
{
  ResBox* b = static_cast<ResBox*>(std::calloc(1, sizeof(ResBox)));
  return b ? &b->r : nullptr;
}

int scanner_acquire(const ugpu_dfa* dfa, ugpu_scanner** out, bool prefer_write = false)
{
  ugpu_dfa* d = const_cast<ugpu_dfa*>(dfa);
  {
    std::lock_guard<std::mutex> lk(d->pool_mu);
    std::vector<ugpu_scanner*>& pool = prefer_write ? d->pool_w : d->pool;
    if (!pool.empty()) {
      *out = pool.back();
      pool.pop_back();
      (*out)->bol0 = 1;  // (a pooled scanner may have served a shard)
      (*out)->xu_exact = false;  // (nor keep the exact U kernel an earlier input needed)
      return UGPU_OK;
    }
  }
  const int rc = scanner_create(dfa, out, prefer_write);
  if (!rc) (*out)->pref_write = prefer_write;
  return rc;
}

void scanner_release(const ugpu_dfa* dfa, ugpu_scanner* s)
{
  ugpu_dfa* d = const_cast<ugpu_dfa*>(dfa);
  std::lock_guard<std::mutex> lk(d->pool_mu);
  (s->pref_write ? d->pool_w : d->pool).push_back(s);
}

}  // namespace

int ugpu_find_all(const ugpu_dfa* dfa, const uint8_t* buf, uint64_t len, uint64_t start, uint32_t mode,
                  ugpu_result** out)
{
  if (!dfa || !out || (!buf && len)) return fail(UGPU_INVAL, "NULL argument");
  *out = nullptr;
  if (start > len) start = len;
  ugpu_result* r = result_alloc();
  if (!r) return fail(UGPU_NOMEM, "host allocation");
  if (len == 0) {
    *out = r;
    return UGPU_OK;
  }
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    std::free(r);
    return hip_fail(e, "hipGetDevice");
  }
  // (the calling thread's device: the table copy there, ugpu_select_device)
  int rc = dfa_on(dfa, dev, &dfa);
  if (rc) {
    std::free(r);
    return rc;
  }
  ugpu_scanner* s = nullptr;
  rc = scanner_acquire(dfa, &s, mode == UGPU_MODE_OFFSETS);
  if (rc) {
    std::free(r);
    return rc;
  }
  FindWs* ws = find_ws_acquire(dev);
  if (!ws) {
    scanner_release(dfa, s);
    std::free(r);
    return fail(UGPU_NOMEM, "find workspace");
  }
  const uint8_t* dbuf = buf;
  ugpu_totals tot{};
  if (!is_device_ptr(buf)) {
    if ((e = ws->reserve_in(len)) != hipSuccess || (e = hipMemcpyAsync(ws->d_in, buf, len, hipMemcpyHostToDevice,
                                                                        ws->st)) != hipSuccess)
      rc = hip_fail(e, "input copy");
    dbuf = ws->d_in;
  }
  s->stage_once = mode == UGPU_MODE_OFFSETS;  // single-pass OFFSETS for sparse tables
  if (!rc) rc = ugpu_scan(s, dbuf, start, len, len, 1, 0, ws->st);
  if (!rc) rc = ugpu_scan_totals(s, &tot);
  if (!rc) {
    r->count = tot.count;
    r->digest = tot.digest;
    r->dcap = tot.dcap;
  }
  if (!rc && mode == UGPU_MODE_OFFSETS && tot.count > 0) {
    const uint64_t n = tot.count;
    r->start = static_cast<uint64_t*>(std::malloc(n * 8));
    r->len = static_cast<uint32_t*>(std::malloc(n * 4));
    r->cap = static_cast<uint32_t*>(std::malloc(n * 4));
    if (!r->start || !r->len || !r->cap)
      rc = fail(UGPU_NOMEM, "match list allocation");
    else if ((e = ws->reserve_out(n)) != hipSuccess)
      rc = hip_fail(e, "match list");
    if (!rc) rc = ugpu_scan_offsets(s, ws->d_start, ws->d_len, ws->d_cap, n, ws->st);
    if (!rc && ((e = hipMemcpyAsync(r->start, ws->d_start, n * 8, hipMemcpyDeviceToHost, ws->st)) != hipSuccess ||
                (e = hipMemcpyAsync(r->len, ws->d_len, n * 4, hipMemcpyDeviceToHost, ws->st)) != hipSuccess ||
                (e = hipMemcpyAsync(r->cap, ws->d_cap, n * 4, hipMemcpyDeviceToHost, ws->st)) != hipSuccess ||
                (e = hipStreamSynchronize(ws->st)) != hipSuccess))
      rc = hip_fail(e, "hipMemcpy matches");
  }
  (void)hipStreamSynchronize(ws->st);
  find_ws_release(ws);
  scanner_release(dfa, s);
  if (rc) {
    ugpu_result_free(r);
    return rc;
  }
  *out = r;
  return UGPU_OK;
}

// ---------------------------------------------------------------- records (host path)
// ugpu_find_records: the FIND records of a host buffer for a consumer that pops
// them one by one (the drop-in matcher), as fast as PCIe moves the input.  The
// input goes H2D in chunks on a copy thread; each chunk is scanned from the true
// chain entry (the previous chunk's exit) as soon as it and the next one are on
// the device, its records are written, packed to 6 B (u32 start - chunk base,
// u16 len; + u16 cap when the table has several accept indices) -- or, for
// dense chunks of one accept index (a record per < 32 bytes), to 2 B (u8 gap
// from the previous record's end, u8 len) -- and copied asynchronously into
// pinned host memory -- H2D, scans and D2H overlap.  The records are decoded
// when popped.
struct ugpu_records {
  struct Piece {
    uint64_t base = 0, n = 0;
    uint8_t* host = nullptr;  // pinned: u32 start[n], u16 len[n], (caps) u16 cap[n]
    size_t host_bytes = 0;
    hipEvent_t landed = nullptr;  // the D2H into host has completed (NULL: already waited for)
    bool dense = false;           // host: u8 gap[n], u8 len[n] (pack_records_kernel dense)
    std::vector<std::pair<uint64_t, uint64_t>> esc;  // (index, len | cap << 32), sorted
  };
  // published by the pipeline thread (under mu; a deque keeps references)
  std::deque<Piece> pieces;
  size_t published = 0;
  bool done = false;
  bool input_free = false;  // the caller's host buffer is no longer read
  bool cancel = false;      // ugpu_records_free before the end: the pipeline stops at its next chunk
  bool unbounded = false;   // ugpu_records_totals waits for the end: no limit on pieces ahead
  size_t ahead = 4;         // pieces the pipeline may publish ahead of the consumer (UGPU_REC_AHEAD)
  uint64_t chunk = 16ull << 20;  // input bytes per piece (UGPU_REC_CHUNK)
  int rc = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::thread worker;
  int caps = 0;
  uint32_t cap1 = 1;
  uint64_t count = 0, digest = 0, dcap = 0;  // final once done
  // the consumer's piece: pieces[pi - 1] (pi = 0: none yet)
  size_t pi = 0;
  bool sync_d2h = false;  // UGPU_REC_SYNC=1: the pipeline waits for each D2H before the next chunk
  bool zero_copy = false; // UGPU_REC_ZC=1: the pack kernel stores straight into the pinned block
  bool trace = false;     // UGPU_REC_TRACE=1: per-chunk timestamps on stderr
  std::chrono::steady_clock::time_point t0;
  const uint32_t* st = nullptr;
  const uint16_t* ln = nullptr;
  const uint16_t* cp = nullptr;
  const uint8_t* dg = nullptr;  // dense piece: gaps (ln, cp unused)
  const uint8_t* dl = nullptr;  // dense piece: lengths
  uint64_t last = 0;            // dense piece: the end of the last popped record (offset from base)
  const std::pair<uint64_t, uint64_t>* esc = nullptr;
  uint64_t base = 0, n = 0, ri = 0, ei = 0, ne = 0;
};

namespace {

// pinned host blocks, pooled (hipHostMalloc pins pages: milliseconds per MiB
// the first time)
std::mutex g_pin_mu;
std::vector<std::pair<uint8_t*, size_t>> g_pin_pool;
// (the pool keeps at most kPinKeep bytes; blocks beyond that are unpinned)
constexpr size_t kPinKeep = 1ull << 30;
size_t g_pin_kept = 0;

uint8_t* pinned_get(size_t need, size_t& got)
{
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    size_t best = g_pin_pool.size();
    for (size_t i = 0; i < g_pin_pool.size(); ++i)
      if (g_pin_pool[i].second >= need && (best == g_pin_pool.size() || g_pin_pool[i].second < g_pin_pool[best].second))
        best = i;
    if (best < g_pin_pool.size()) {
      uint8_t* p = g_pin_pool[best].first;
      got = g_pin_pool[best].second;
      g_pin_pool.erase(g_pin_pool.begin() + (long)best);
      g_pin_kept -= got;
      return p;
    }
  }
  // (power-of-two blocks from 4 MiB: a piece of a small chunk does not pin
  // 64 MiB, which pushed the pool past kPinKeep and into a pin/unpin per piece)
  size_t c = 4u << 20;
  while (c < need) c *= 2;
  void* p = nullptr;
  // (non-coherent: cached for the host reads that decode the records; every
  // read follows a stream synchronisation)
  if (hipHostMalloc(&p, c, hipHostMallocNonCoherent) != hipSuccess) return nullptr;
  exit_guard_arm();
  got = c;
  return static_cast<uint8_t*>(p);
}


void pinned_put(uint8_t* p, size_t n)
{
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (g_pin_kept + n <= kPinKeep) {
      g_pin_pool.push_back(std::make_pair(p, n));
      g_pin_kept += n;
      return;
    }
  }
  (void)hipHostFree(p);
}

// Per-device workspace of the records path, pooled: copy and D2H streams,
// double-buffered pack / escape buffers and their events.
struct RecWs {
  int dev = -1;
  hipStream_t cst = nullptr, dst = nullptr;
  uint8_t* d_pack[2] = {nullptr, nullptr};
  uint64_t pack_cap[2] = {0, 0};
  uint64_t* d_esc[2] = {nullptr, nullptr};
  uint64_t esc_cap[2] = {0, 0};
  uint32_t* d_nesc = nullptr;  // [2]
  uint32_t* h_nesc = nullptr;  // pinned [2]
  hipEvent_t packed[2] = {nullptr, nullptr}, copied[2] = {nullptr, nullptr};
  bool used[2] = {false, false};

  hipError_t init()
  {
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&cst, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&dst, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&d_nesc, 2 * sizeof(uint32_t))) != hipSuccess ||
        (e = hipHostMalloc(&h_nesc, 2 * sizeof(uint32_t))) != hipSuccess)
      return e;
    for (int i = 0; i < 2; ++i)
      if ((e = hipEventCreateWithFlags(&packed[i], hipEventDisableTiming)) != hipSuccess ||
          (e = hipEventCreateWithFlags(&copied[i], hipEventDisableTiming)) != hipSuccess)
        return e;
    return hipSuccess;
  }
  hipError_t reserve(int b, uint64_t bytes, uint64_t n)
  {
    hipError_t e;
    if (bytes > pack_cap[b]) {
      (void)hipFree(d_pack[b]);
      d_pack[b] = nullptr;
      pack_cap[b] = 0;
      const uint64_t c = bytes + bytes / 4;
      if ((e = hipMalloc(&d_pack[b], c)) != hipSuccess) return e;
      pack_cap[b] = c;
    }
    if (n > esc_cap[b]) {
      (void)hipFree(d_esc[b]);
      d_esc[b] = nullptr;
      esc_cap[b] = 0;
      const uint64_t c = n + n / 4;
      if ((e = hipMalloc(&d_esc[b], c * 16)) != hipSuccess) return e;
      esc_cap[b] = c;
    }
    return hipSuccess;
  }
};

std::mutex g_rec_mu;
std::vector<RecWs*> g_rec_pool;

RecWs* rec_ws_acquire(int dev)
{
  {
    std::lock_guard<std::mutex> lk(g_rec_mu);
    for (size_t i = 0; i < g_rec_pool.size(); ++i)
      if (g_rec_pool[i]->dev == dev) {
        RecWs* w = g_rec_pool[i];
        g_rec_pool.erase(g_rec_pool.begin() + (long)i);
        return w;
      }
  }
  RecWs* w = new (std::nothrow) RecWs;
  if (!w) return nullptr;
  w->dev = dev;
  if (w->init() != hipSuccess) return nullptr;  // (leaks the partial workspace on a broken device)
  exit_guard_arm();
  return w;
}

void rec_ws_release(RecWs* w)
{
  std::lock_guard<std::mutex> lk(g_rec_mu);
  g_rec_pool.push_back(w);
}

// H2D of a host buffer in chunks on its own thread; waiters block until a
// prefix is on the device
struct Uploader {
  ugpu_records* R = nullptr;  // told when the last byte is on the device
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  uint64_t len = 0, chunk = 0;
  hipStream_t st = nullptr;
  int dev = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t done = 0;
  int rc = UGPU_OK;
  std::thread th;

  void run()
  {
    (void)hipSetDevice(dev);
    for (uint64_t o = 0; o < len; o += chunk) {
      bool stop;
      {
        // ugpu_records_free before the end (-m1, -l, -q): copy no more of
        // the input; a scan waiting for it is released and stops too
        std::lock_guard<std::mutex> lk(R->mu);
        stop = R->cancel;
      }
      if (stop) {
        std::lock_guard<std::mutex> lk(mu);
        rc = UGPU_INVAL;  // (no message: nobody reads the result of a cancelled pipeline)
        done = len;
        cv.notify_all();
        break;
      }
      const uint64_t n = len - o < chunk ? len - o : chunk;
      hipError_t e = hipMemcpyAsync(dst + o, src + o, n, hipMemcpyHostToDevice, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      std::lock_guard<std::mutex> lk(mu);
      if (e != hipSuccess) {
        rc = hip_fail(e, "records input copy");
        done = len;
        cv.notify_all();
        break;
      }
      done = o + n;
      cv.notify_all();
    }
    std::lock_guard<std::mutex> lk(R->mu);
    R->input_free = true;
    R->cv.notify_all();
  }
  // the first `upto` bytes are on the device (or the copy failed)
  int wait(uint64_t upto)
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done >= upto || rc != UGPU_OK; });
    return rc;
  }
};

}  // namespace

namespace {

// The records pipeline of ugpu_find_records, on its own thread: publishes
// each chunk's piece as soon as its records are in pinned host memory.
void records_pipeline(ugpu_records* R, const ugpu_dfa* dfa, int dev, const uint8_t* buf, uint64_t len,
                      uint64_t start)
{
  int rc = UGPU_OK;
  uint64_t count = 0, digest = 0, dcap = 0;
  auto trace = [&](const char* what, uint64_t lo) {
    if (R->trace)
      fprintf(stderr, "[records] %9.3f ms  %-10s chunk at %llu\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - R->t0).count(), what,
              (unsigned long long)lo);
  };
  auto publish = [&](ugpu_records::Piece* pc, bool last) {
    std::lock_guard<std::mutex> lk(R->mu);
    if (pc) {
      R->pieces.push_back(std::move(*pc));
      if (rc == UGPU_OK) R->published = R->pieces.size();
    }
    if (last) {
      R->count = count;
      R->digest = digest;
      R->dcap = dcap;
      R->rc = rc;
      R->done = true;
      R->input_free = true;
    }
    R->cv.notify_all();
  };
  if (hipSetDevice(dev) != hipSuccess) {
    rc = fail(UGPU_DEVICE, "hipSetDevice");
    publish(nullptr, true);
    return;
  }
  ugpu_scanner* s = nullptr;
  if ((rc = scanner_acquire(dfa, &s, true)) != UGPU_OK) {
    publish(nullptr, true);
    return;
  }
  FindWs* ws = find_ws_acquire(dev);
  RecWs* rw = ws ? rec_ws_acquire(dev) : nullptr;
  if (!ws || !rw) {
    if (ws) find_ws_release(ws);
    scanner_release(dfa, s);
    rc = fail(UGPU_NOMEM, "records workspace");
    publish(nullptr, true);
    return;
  }
  const uint64_t chunk = R->chunk;
  const uint64_t halo = 1ull << 20;
  const bool host = !is_device_ptr(buf);
  // (the bytes before start are never read but for at_wb / at_bol, 4 back)
  const uint64_t from = host && start > 4 ? start - 4 : 0;
  const uint8_t* dbuf = buf;
  Uploader up;
  hipError_t e = hipSuccess;
  if (host) {
    if ((e = ws->reserve_in(len)) != hipSuccess) {
      rc = hip_fail(e, "records input");
    } else {
      dbuf = ws->d_in;
      up.src = buf + from;
      up.dst = ws->d_in + from;
      up.len = len - from;
      up.chunk = chunk;
      up.st = rw->cst;
      up.dev = dev;
      up.R = R;
      up.th = std::thread([&up] { up.run(); });
    }
  }
  auto ready = [&](uint64_t upto) -> int { return host ? up.wait(upto - from) : UGPU_OK; };
  uint64_t entry = start;
  int b = 0;
  s->stage_once = true;  // single-pass OFFSETS for prefiltered tables
  for (uint64_t lo = start; !rc && lo < len;) {
    {
      // at most R->ahead pieces past the consumer's (their pinned blocks go
      // back to the pool as the consumer moves on); a free() stops the scan
      std::unique_lock<std::mutex> lk(R->mu);
      R->cv.wait(lk, [&] { return R->cancel || R->unbounded || R->pieces.size() < R->pi + R->ahead; });
      if (R->cancel) break;
    }
    const uint64_t hi = len - lo <= chunk + chunk / 4 ? len : lo + chunk;
    uint64_t rend = hi + halo < len ? hi + halo : len;
    ugpu_totals tot{};
    if (entry < hi) {
      for (;;) {
        if ((rc = ready(rend)) != UGPU_OK) break;
        trace("on device", lo);
        rc = ugpu_scan(s, dbuf, entry, hi, rend, rend == len, 0, ws->st);
        if (!rc) rc = ugpu_scan_totals(s, &tot);
        if (rc == UGPU_HALO && rend < len) {
          rend = len;
          continue;
        }
        break;
      }
      if (rc) break;
    } else {
      tot.exit = entry;  // a match of an earlier chunk covers this one
    }
    count += tot.count;
    digest += tot.digest;
    dcap += tot.dcap;
    if (tot.count) {
      ugpu_records::Piece pc;
      pc.base = lo;
      pc.n = tot.count;
      pc.dense = !R->caps && pc.n * 32 >= hi - lo && env_u64("UGPU_REC_DENSE", 1) != 0;
      const uint64_t n = pc.n, bytes = n * (pc.dense ? 2 : R->caps ? 8 : 6);
      if ((e = ws->reserve_out(n)) != hipSuccess) {
        rc = hip_fail(e, "records output");
        break;
      }
      if ((rc = ugpu_scan_offsets(s, ws->d_start, ws->d_len, ws->d_cap, n, ws->st)) != UGPU_OK) break;
      // the pack buffer b was last read by the D2H of two chunks ago
      if (rw->used[b] && (e = hipStreamWaitEvent(ws->st, rw->copied[b], 0)) != hipSuccess) {
        rc = hip_fail(e, "records event");
        break;
      }
      if ((e = rw->reserve(b, bytes, n)) != hipSuccess) {
        rc = hip_fail(e, "records pack buffer");
        break;
      }
      pc.host = pinned_get(bytes, pc.host_bytes);
      if (!pc.host) {
        rc = fail(UGPU_NOMEM, "pinned records");
        break;
      }
      void* hdev = nullptr;
      if (R->zero_copy && hipHostGetDevicePointer(&hdev, pc.host, 0) != hipSuccess) {
        (void)hipGetLastError();
        hdev = nullptr;
      }
      if (hdev) {
        // zero copy: the pack kernel's stores cross PCIe into the pinned block
        // (no device pack buffer, no D2H copy); the block is the consumer's
        // once the kernel has finished
        if ((e = hipMemsetAsync(rw->d_nesc + b, 0, sizeof(uint32_t), ws->st)) != hipSuccess ||
            (e = launch_pack_records(ws->d_start, ws->d_len, ws->d_cap, n, lo, static_cast<uint8_t*>(hdev), R->caps,
                                     pc.dense ? 1 : 0, rw->d_esc[b], rw->d_nesc + b, ws->st)) != hipSuccess ||
            (e = hipMemcpyAsync(rw->h_nesc + b, rw->d_nesc + b, sizeof(uint32_t), hipMemcpyDeviceToHost, ws->st)) !=
                hipSuccess ||
            (e = hipStreamSynchronize(ws->st)) != hipSuccess) {
          rc = hip_fail(e, "records pack");
          publish(&pc, false);
          break;
        }
        trace("packed", lo);
        const uint32_t ne = rw->h_nesc[b];
        if (ne) {
          std::vector<uint64_t> es(2 * (size_t)ne);
          if ((e = hipMemcpy(es.data(), rw->d_esc[b], 16ull * ne, hipMemcpyDeviceToHost)) != hipSuccess) {
            rc = hip_fail(e, "records escapes");
            publish(&pc, false);
            break;
          }
          for (uint32_t k = 0; k < ne; ++k) pc.esc.push_back(std::make_pair(es[2 * k], es[2 * k + 1]));
          std::sort(pc.esc.begin(), pc.esc.end());
        }
        publish(&pc, false);
        entry = tot.exit;
        lo = hi;
        continue;
      }
      if ((e = hipMemsetAsync(rw->d_nesc + b, 0, sizeof(uint32_t), ws->st)) != hipSuccess ||
          (e = launch_pack_records(ws->d_start, ws->d_len, ws->d_cap, n, lo, rw->d_pack[b], R->caps, pc.dense ? 1 : 0,
                                   rw->d_esc[b], rw->d_nesc + b, ws->st)) != hipSuccess ||
          (e = hipMemcpyAsync(rw->h_nesc + b, rw->d_nesc + b, sizeof(uint32_t), hipMemcpyDeviceToHost, ws->st)) !=
              hipSuccess ||
          (e = hipEventRecord(rw->packed[b], ws->st)) != hipSuccess ||
          (e = hipStreamWaitEvent(rw->dst, rw->packed[b], 0)) != hipSuccess ||
          (e = hipMemcpyAsync(pc.host, rw->d_pack[b], bytes, hipMemcpyDeviceToHost, rw->dst)) != hipSuccess ||
          (e = hipEventRecord(rw->copied[b], rw->dst)) != hipSuccess ||
          (e = hipStreamSynchronize(ws->st)) != hipSuccess) {
        rc = hip_fail(e, "records pack");
        publish(&pc, false);  // (not published: handed over so that free() returns its pinned block)
        break;
      }
      rw->used[b] = true;
      trace("packed", lo);
      // escapes (lengths or accept indices >= 0xFFFF, rare)
      const uint32_t ne = rw->h_nesc[b];
      if (ne) {
        std::vector<uint64_t> es(2 * (size_t)ne);
        if ((e = hipMemcpy(es.data(), rw->d_esc[b], 16ull * ne, hipMemcpyDeviceToHost)) != hipSuccess) {
          rc = hip_fail(e, "records escapes");
          publish(&pc, false);
          break;
        }
        for (uint32_t k = 0; k < ne; ++k) pc.esc.push_back(std::make_pair(es[2 * k], es[2 * k + 1]));
        std::sort(pc.esc.begin(), pc.esc.end());
      }
      // the piece is the consumer's once its copy has landed: the consumer
      // waits for that (records_advance), so this chunk's D2H overlaps the
      // next chunk's scans
      if (R->sync_d2h) {
        if ((e = hipEventSynchronize(rw->copied[b])) != hipSuccess) {
          rc = hip_fail(e, "records copy");
          publish(&pc, false);
          break;
        }
        trace("copied", lo);
      } else if ((e = hipEventCreateWithFlags(&pc.landed, hipEventDisableTiming)) != hipSuccess ||
                 (e = hipEventRecord(pc.landed, rw->dst)) != hipSuccess) {
        rc = hip_fail(e, "records copy event");
        publish(&pc, false);
        break;
      }
      publish(&pc, false);
      b ^= 1;
    }
    entry = tot.exit;
    lo = hi;
  }
  if (host && up.th.joinable()) up.th.join();
  (void)hipStreamSynchronize(ws->st);
  (void)hipStreamSynchronize(rw->dst);
  rw->used[0] = rw->used[1] = false;
  rec_ws_release(rw);
  find_ws_release(ws);
  scanner_release(dfa, s);
  if (!rc && host) rc = up.rc;
  publish(nullptr, true);
}

// the consumer's next piece (blocks until the pipeline publishes it); false
// at the end or on a pipeline error (*rc)
bool records_advance(ugpu_records* r, int* rc)
{
  std::unique_lock<std::mutex> lk(r->mu);
  if (r->pi > 0) {
    // the consumer is done with its piece (ugpu_records_next returns copies):
    // its pinned block goes back to the pool, and the pipeline may run ahead
    ugpu_records::Piece& prev = r->pieces[r->pi - 1];
    if (prev.host && !prev.landed) {
      pinned_put(prev.host, prev.host_bytes);
      prev.host = nullptr;
    }
    r->dg = r->dl = nullptr;
    r->st = nullptr;
    r->ln = r->cp = nullptr;
    r->n = r->ri = 0;
    r->cv.notify_all();
  }
  r->cv.wait(lk, [&] { return r->pi < r->published || r->done; });
  if (r->pi >= r->published) {
    *rc = r->rc;
    return false;
  }
  ugpu_records::Piece& p = r->pieces[r->pi++];
  r->cv.notify_all();  // (the pipeline may wait for the consumer to move on: R->ahead)
  if (p.landed) {
    // (the pipeline thread only appends to the deque: p stays put)
    hipEvent_t ev = p.landed;
    lk.unlock();
    const hipError_t e = hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
    lk.lock();
    p.landed = nullptr;
    if (e != hipSuccess) {
      *rc = hip_fail(e, "records copy");
      r->pi = r->published;
      return false;
    }
  }
  if (r->trace)
    fprintf(stderr, "[records] %9.3f ms  consumer   piece %zu\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r->t0).count(), r->pi - 1);
  if (p.dense) {
    r->st = nullptr;
    r->ln = nullptr;
    r->cp = nullptr;
    r->dg = p.host;
    r->dl = p.host + p.n;
    r->last = 0;
  } else {
    r->dg = r->dl = nullptr;
    r->st = reinterpret_cast<const uint32_t*>(p.host);
    r->ln = reinterpret_cast<const uint16_t*>(p.host + 4 * p.n);
    r->cp = r->caps ? reinterpret_cast<const uint16_t*>(p.host + 6 * p.n) : nullptr;
  }
  r->esc = p.esc.data();
  r->ne = p.esc.size();
  r->base = p.base;
  r->n = p.n;
  r->ri = r->ei = 0;
  return true;
}

}  // namespace

int ugpu_warmup(int dev)
{
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  exit_guard_arm();
  if (dev < 0 || dev >= n) return fail(UGPU_INVAL, "no such device");
  HIP_TRY(hipSetDevice(dev));
  // the device context, one scan workspace and one records workspace (their
  // streams: a queue each), a pinned block, and one kernel launch (the
  // library's code object is loaded at the first launch)
  FindWs* w = find_ws_acquire(dev);
  if (!w) return fail(UGPU_DEVICE, "scan workspace");
  RecWs* r = rec_ws_acquire(dev);
  if (!r) {
    find_ws_release(w);
    return fail(UGPU_DEVICE, "records workspace");
  }
  int rc = UGPU_OK;
  uint8_t* d = nullptr;
  hipError_t e = hipMalloc(&d, 64);
  if (e == hipSuccess) e = hipMemsetAsync(d, '\n', 64, w->st);
  if (e == hipSuccess) e = hipStreamSynchronize(w->st);
  if (e != hipSuccess) {
    rc = hip_fail(e, "warm-up");
  } else {
    uint64_t pos = 0;
    rc = ugpu_find_nul(d, 64, &pos, w->st);
  }
  if (d) (void)hipFree(d);
  size_t got = 0;
  if (uint8_t* p = pinned_get(1u << 20, got)) pinned_put(p, got);
  rec_ws_release(r);
  find_ws_release(w);
  return rc;
}

int ugpu_find_records(const ugpu_dfa* dfa, const uint8_t* buf, uint64_t len, uint64_t start, ugpu_records** out)
{
  return ugpu_find_records_ex(dfa, buf, len, start, 0, out);
}

int ugpu_find_records_ex(const ugpu_dfa* dfa, const uint8_t* buf, uint64_t len, uint64_t start, uint32_t flags,
                         ugpu_records** out)
{
  if (!dfa || !out || (!buf && len)) return fail(UGPU_INVAL, "NULL argument");
  if (flags & ~UGPU_REC_BORROW) return fail(UGPU_INVAL, "unknown records flags");
  *out = nullptr;
  if (start > len) start = len;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  int rc = dfa_on(dfa, dev, &dfa);
  if (rc) return rc;
  ugpu_records* R = new (std::nothrow) ugpu_records();
  if (!R) return fail(UGPU_NOMEM, "host allocation");
  R->caps = dfa->t.cap1 == 0 ? 1 : 0;
  R->cap1 = dfa->t.cap1 ? dfa->t.cap1 : 1;
  R->sync_d2h = env_u64("UGPU_REC_SYNC", 0) != 0;
  R->zero_copy = env_u64("UGPU_REC_ZC", 0) != 0;
  R->trace = env_u64("UGPU_REC_TRACE", 0) != 0;
  // chunks of 16 MiB (tools/rec_sweep.py); the pipeline runs
  // at most 256 MiB of input (and at least 4 pieces) ahead of the consumer
  R->chunk = std::max<uint64_t>(env_u64("UGPU_REC_CHUNK", 16ull << 20), 1ull << 20);
  R->ahead = (size_t)std::max<uint64_t>(env_u64("UGPU_REC_AHEAD", std::max<uint64_t>(4, (256ull << 20) / R->chunk)), 1);
  R->t0 = std::chrono::steady_clock::now();
  if (len == start) {
    R->done = R->input_free = true;
  } else {
    try {
      R->worker = std::thread(records_pipeline, R, dfa, dev, buf, len, start);
    } catch (...) {
      delete R;
      return fail(UGPU_NOMEM, "records thread");
    }
    // a host buffer may go away once this returns (ugrep unmaps a file when
    // it stops asking for matches): wait for the last input byte to be on the
    // device; scans and record copies go on behind the consumer.  Borrowed
    // buffers (UGPU_REC_BORROW) stay readable until ugpu_records_free, which
    // joins the pipeline: the consumer starts at the first piece.
    if (!is_device_ptr(buf) && !(flags & UGPU_REC_BORROW)) {
      std::unique_lock<std::mutex> lk(R->mu);
      R->cv.wait(lk, [&] { return R->input_free; });
    }
  }
  *out = R;
  return UGPU_OK;
}

int ugpu_records_next(ugpu_records* r, uint64_t* start, uint32_t* len, uint32_t* cap)
{
  if (!r) return -fail(UGPU_INVAL, "NULL argument");
  while (r->ri >= r->n) {
    int rc = UGPU_OK;
    if (!records_advance(r, &rc)) return rc ? -rc : 0;
  }
  const uint64_t i = r->ri++;
  if (r->dg) {
    uint64_t so;
    uint32_t l = r->dl[i];
    if ((l == 0xFFu || r->dg[i] == 0xFFu) && r->ei < r->ne && r->esc[r->ei].first == i) {
      const uint64_t v = r->esc[r->ei++].second;
      so = (uint32_t)v;
      l = (uint32_t)(v >> 32);
    } else {
      so = r->last + r->dg[i];
    }
    r->last = so + l;
    *start = r->base + so;
    *len = l;
    *cap = r->cap1;
    return 1;
  }
  uint32_t l = r->ln[i], c = r->cp ? r->cp[i] : r->cap1;
  if ((l == 0xFFFFu || c == 0xFFFFu) && r->ei < r->ne && r->esc[r->ei].first == i) {
    const uint64_t v = r->esc[r->ei++].second;
    l = (uint32_t)v;
    if (r->cp) c = (uint32_t)(v >> 32);
  }
  *start = r->base + r->st[i];
  *len = l;
  *cap = c;
  return 1;
}

namespace {

// the count, digest and dcap of one whole piece, from its arrays (what a
// native consumer's inlined loop computes)
struct PieceSums {
  uint64_t k = 0, dg = 0, dc = 0;
};

void decode_piece(const ugpu_records::Piece& p, int caps, uint32_t cap1, PieceSums& out)
{
  const uint64_t pn = p.n, base = p.base;
  const std::pair<uint64_t, uint64_t>* esc = p.esc.data();
  const uint64_t ne = p.esc.size();
  if (p.dense) {
    // a dense piece: start_i = so + sum of gaps up to i + lengths before i,
    // so between escapes the sums of starts are weighted sums of the gaps
    // and lengths (no serial chain; the loop vectorises); an escaped record
    // carries its own start and restarts the sum after it
    const uint8_t* g = p.host;
    const uint8_t* l = p.host + pn;
    uint64_t so = 0, ssum = 0, slen = 0, a = 0;
    auto seg = [&](uint64_t b) {
      // (blocks of 256: the in-block weights j * byte fit 16 bits, so the
      // inner loop vectorises with 16-bit multiplies)
      uint64_t sg = 0, skg = 0, sl = 0, skl = 0;
      for (uint64_t kb = a; kb < b; kb += 256) {
        const uint32_t m = b - kb < 256 ? (uint32_t)(b - kb) : 256u;
        const uint8_t* gp = g + kb;
        const uint8_t* lp = l + kb;
        uint32_t bg = 0, bjg = 0, bl = 0, bjl = 0;
        for (uint32_t j = 0; j < m; ++j) {
          bg += gp[j];
          bjg += (uint16_t)((uint16_t)j * gp[j]);
          bl += lp[j];
          bjl += (uint16_t)((uint16_t)j * lp[j]);
        }
        sg += bg;
        sl += bl;
        skg += kb * bg + bjg;
        skl += kb * bl + bjl;
      }
      ssum += (b - a) * so + (b * sg - skg) + (b ? (b - 1) * sl - skl : 0);
      slen += sl;
      so += sg + sl;
    };
    for (uint64_t j = 0; j < ne; ++j) {
      const uint64_t e = esc[j].first, v = esc[j].second;
      seg(e);
      so = (uint32_t)v;
      ssum += so;
      slen += v >> 32;
      so += v >> 32;
      a = e + 1;
    }
    seg(pn);
    out.dg = 31 * (ssum + pn * base) + slen;
    out.dc = (ssum + pn * (base + 1)) * cap1;
    out.k = pn;
    return;
  }
  const uint32_t* ps = reinterpret_cast<const uint32_t*>(p.host);
  const uint16_t* pl = reinterpret_cast<const uint16_t*>(p.host + 4 * pn);
  const uint16_t* pc = caps ? reinterpret_cast<const uint16_t*>(p.host + 6 * pn) : nullptr;
  uint64_t sdg = 0, sdc = 0, ssum = 0;
  for (uint64_t i = 0; i < pn; ++i) {
    const uint64_t s0 = ps[i];
    ssum += s0;
    sdg += s0 * 31 + pl[i];
    if (pc) sdc += (base + s0 + 1) * pc[i];
  }
  // starts are base + s0; caps are cap1 without a cap array
  out.dg = sdg + pn * base * 31;
  out.dc = pc ? sdc : (ssum + pn * (base + 1)) * cap1;
  for (uint64_t j = 0; j < ne; ++j) {
    // escaped records: replace the 0xFFFF placeholders by the true values
    const uint64_t i = esc[j].first, s0 = base + ps[i];
    const uint32_t l = (uint32_t)esc[j].second, c = pc ? (uint32_t)(esc[j].second >> 32) : cap1;
    out.dg += (uint64_t)l - pl[i];
    if (pc) out.dc += (s0 + 1) * ((uint64_t)c - pc[i]);
  }
  out.k = pn;
}

// the next whole piece for ugpu_records_drain, without releasing the one
// before (its decode may still run); false at the end or on an error (*rc).
// *piece is looked up while r->mu is held: the pipeline thread appends to
// r->pieces under it, and a deque append may rebuild the map that operator[]
// reads (elements themselves never move, so the pointer stays valid after)
bool records_take(ugpu_records* r, size_t* idx, const ugpu_records::Piece** piece, int* rc)
{
  std::unique_lock<std::mutex> lk(r->mu);
  r->cv.wait(lk, [&] { return r->pi < r->published || r->done; });
  if (r->pi >= r->published) {
    *rc = r->rc;
    return false;
  }
  const size_t i = r->pi++;
  r->cv.notify_all();  // (the pipeline may wait for the consumer to move on: R->ahead)
  ugpu_records::Piece& p = r->pieces[i];
  if (p.landed) {
    hipEvent_t ev = p.landed;
    lk.unlock();
    const hipError_t e = hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
    lk.lock();
    p.landed = nullptr;
    if (e != hipSuccess) {
      *rc = hip_fail(e, "records copy");
      r->pi = r->published;
      return false;
    }
  }
  *idx = i;
  *piece = &p;
  return true;
}

void records_release(ugpu_records* r, size_t i)
{
  std::lock_guard<std::mutex> lk(r->mu);
  ugpu_records::Piece& p = r->pieces[i];
  pinned_put(p.host, p.host_bytes);
  p.host = nullptr;
  r->cv.notify_all();
}

}  // namespace

int ugpu_records_drain(ugpu_records* r, uint64_t* n, uint64_t* digest, uint64_t* dcap)
{
  if (!r) return fail(UGPU_INVAL, "NULL argument");
  // the rest of the current piece through ugpu_records_next, then whole
  // pieces straight from their arrays as they are published, decoded on up
  // to UGPU_REC_DRAIN_THREADS threads at once (default 8; a piece's sums
  // need nothing from the pieces before it)
  uint64_t k = 0, dg = 0, dc = 0, st = 0;
  uint32_t ln = 0, cp = 0;
  while (r->ri < r->n && ugpu_records_next(r, &st, &ln, &cp) == 1) {
    ++k;
    dg += st * 31 + ln;
    dc += (st + 1) * cp;
  }
  if (r->pi > 0) {
    // (the current piece is used up: back to the pool)
    std::lock_guard<std::mutex> lk(r->mu);
    ugpu_records::Piece& prev = r->pieces[r->pi - 1];
    if (prev.host && !prev.landed) {
      pinned_put(prev.host, prev.host_bytes);
      prev.host = nullptr;
    }
    r->dg = r->dl = nullptr;
    r->st = nullptr;
    r->ln = r->cp = nullptr;
    r->n = r->ri = 0;
    r->cv.notify_all();
  }
  const size_t threads = (size_t)std::max<uint64_t>(env_u64("UGPU_REC_DRAIN_THREADS", 8), 1);
  std::deque<std::pair<size_t, std::future<PieceSums>>> jobs;
  auto retire = [&]() {
    PieceSums s = jobs.front().second.get();
    records_release(r, jobs.front().first);
    jobs.pop_front();
    k += s.k;
    dg += s.dg;
    dc += s.dc;
  };
  int rc = UGPU_OK;
  size_t idx = 0;
  const ugpu_records::Piece* pp = nullptr;
  while (records_take(r, &idx, &pp, &rc)) {
    const int caps = r->caps;
    const uint32_t cap1 = r->cap1;
    if (threads == 1) {
      jobs.emplace_back(idx, std::async(std::launch::deferred, [pp, caps, cap1] {
        PieceSums o;
        decode_piece(*pp, caps, cap1, o);
        return o;
      }));
    } else {
      try {
        jobs.emplace_back(idx, std::async(std::launch::async, [pp, caps, cap1] {
        PieceSums o;
        decode_piece(*pp, caps, cap1, o);
        return o;
      }));
      } catch (...) {
        jobs.emplace_back(idx, std::async(std::launch::deferred, [pp, caps, cap1] {
        PieceSums o;
        decode_piece(*pp, caps, cap1, o);
        return o;
      }));
      }
    }
    while (jobs.size() >= threads) retire();
  }
  while (!jobs.empty()) retire();
  if (rc) return rc;
  if (n) *n = k;
  if (digest) *digest = dg;
  if (dcap) *dcap = dc;
  return UGPU_OK;
}

int ugpu_records_totals(ugpu_records* r, uint64_t* count, uint64_t* digest, uint64_t* dcap)
{
  if (!r) return fail(UGPU_INVAL, "NULL argument");
  std::unique_lock<std::mutex> lk(r->mu);
  r->unbounded = true;  // (the pipeline must not wait for pops that come after this)
  r->cv.notify_all();
  r->cv.wait(lk, [&] { return r->done; });
  if (r->rc) return r->rc;
  if (count) *count = r->count;
  if (digest) *digest = r->digest;
  if (dcap) *dcap = r->dcap;
  return UGPU_OK;
}

int ugpu_records_free(ugpu_records* r)
{
  if (!r) return UGPU_OK;
  {
    // an early stop (ugrep -m1, -l, -q): the pipeline stops at its next chunk
    // instead of scanning (and pinning records for) the rest of the input
    std::lock_guard<std::mutex> lk(r->mu);
    r->cancel = true;
    r->cv.notify_all();
  }
  if (r->worker.joinable()) r->worker.join();
  if (exiting()) return UGPU_OK;  // (the pinned blocks and events stay)
  for (auto& p : r->pieces) {
    if (p.landed) {  // (never popped: its copy may still be running)
      (void)hipEventSynchronize(p.landed);
      (void)hipEventDestroy(p.landed);
    }
    pinned_put(p.host, p.host_bytes);
  }
  delete r;
  return UGPU_OK;
}

// ---------------------------------------------------------------- multi-device
namespace {

// the table copy of d on device dev (d itself on its own device); the caller
// has made dev current
int dfa_on(const ugpu_dfa* d, int dev, const ugpu_dfa** out)
{
  if (dev == d->device) {
    *out = d;
    return UGPU_OK;
  }
  ugpu_dfa* m = const_cast<ugpu_dfa*>(d);
  std::lock_guard<std::mutex> lk(m->rep_mu);
  if (m->reps.size() <= (size_t)dev) m->reps.resize((size_t)dev + 1, nullptr);
  if (!m->reps[dev]) {
    ugpu_dfa* r = nullptr;
    const int rc = ugpu_dfa_create(m->opc.data(), (uint32_t)m->opc.size(), m->pflags, &r);
    if (rc) return rc;
    m->reps[dev] = r;
  }
  *out = m->reps[dev];
  return UGPU_OK;
}

// One shard of ugpu_find_all_multi: [lo, hi) of the caller's buffer, scanned on
// device dev from its own copy of [lo, rend).
struct Shard {
  int dev = 0;
  uint64_t lo = 0, hi = 0, rend = 0;
  uint64_t org = 0;  // buffer offset of dbuf[0]: lo minus the context prefix (at most 4 bytes: at_wb's code
                     // point before lo, at_bol's byte)
  const ugpu_dfa* tab = nullptr;
  ugpu_scanner* sc = nullptr;
  FindWs* ws = nullptr;
  const uint8_t* dbuf = nullptr;  // the shard's bytes on its device (dbuf[0] = buffer byte org)
  ugpu_totals tot{};
  uint64_t entry = 0, exit = 0;   // global chain entry / exit (entry = lo speculatively)
  uint64_t base = 0;              // first record index (OFFSETS)
  int rc = UGPU_OK;
};

// bytes [org, rend) of the caller's buffer onto the shard's device
int shard_load(Shard& sh, const uint8_t* buf, bool host, int src_dev)
{
  const uint64_t n = sh.rend - sh.org;
  hipError_t e;
  if (!host && src_dev == sh.dev) {
    sh.dbuf = buf + sh.org;
    return UGPU_OK;
  }
  if ((e = sh.ws->reserve_in(n)) != hipSuccess) return hip_fail(e, "shard input");
  if (host)
    e = hipMemcpyAsync(sh.ws->d_in, buf + sh.org, n, hipMemcpyHostToDevice, sh.ws->st);
  else
    e = hipMemcpyPeerAsync(sh.ws->d_in, sh.dev, buf + sh.org, src_dev, n, sh.ws->st);
  if (e != hipSuccess) return hip_fail(e, "shard input copy");
  sh.dbuf = sh.ws->d_in;
  return UGPU_OK;
}

// speculative COUNT scan of the shard from its start (a match that walks past
// the halo: again with the rest of the buffer readable)
void shard_scan(Shard& sh, const uint8_t* buf, uint64_t len, bool host, int src_dev, uint32_t mode)
{
  if ((sh.rc = hipSetDevice(sh.dev)) != hipSuccess) {
    sh.rc = hip_fail((hipError_t)sh.rc, "hipSetDevice");
    return;
  }
  if ((sh.rc = dfa_on(sh.tab, sh.dev, &sh.tab)) != UGPU_OK) return;
  if ((sh.rc = scanner_acquire(sh.tab, &sh.sc)) != UGPU_OK) return;
  if (!(sh.ws = find_ws_acquire(sh.dev))) {
    sh.rc = fail(UGPU_NOMEM, "find workspace");
    return;
  }
  // the shard's line context and the code point before it come with its bytes:
  // dbuf[0] is the buffer's first byte (BOB) or 4 bytes before lo
  ugpu_scanner_context(sh.sc, 1);
  const uint64_t o = sh.org;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if ((sh.rc = shard_load(sh, buf, host, src_dev)) != UGPU_OK) return;
    sh.sc->stage_once = mode == UGPU_MODE_OFFSETS;
    sh.rc = ugpu_scan(sh.sc, sh.dbuf, sh.lo - o, sh.hi - o, sh.rend - o, sh.rend == len, o, sh.ws->st);
    if (!sh.rc) sh.rc = ugpu_scan_totals(sh.sc, &sh.tot);
    if (sh.rc != UGPU_HALO || sh.rend == len) break;
    sh.rend = len;
  }
  if (sh.rc) return;
  sh.entry = sh.lo;
  sh.exit = sh.tot.exit + o;
}

// the shard's records into r at its base (a shard whose chain entry moved
// is scanned again from the true entry first)
void shard_records(Shard& sh, const uint8_t* src_buf, bool src_host, int src_dev, uint64_t len, ugpu_result* r)
{
  if ((sh.rc = hipSetDevice(sh.dev)) != hipSuccess) {
    sh.rc = hip_fail((hipError_t)sh.rc, "hipSetDevice");
    return;
  }
  const uint64_t n = sh.tot.count;
  if (n == 0) return;
  if (sh.entry != sh.lo) {
    ugpu_totals t{};
    for (;;) {
      sh.rc = ugpu_scan(sh.sc, sh.dbuf, sh.entry - sh.org, sh.hi - sh.org, sh.rend - sh.org, sh.rend == len, sh.org,
                        sh.ws->st);
      if (!sh.rc) sh.rc = ugpu_scan_totals(sh.sc, &t);
      // the chain from the true entry may walk farther than the one from lo:
      // again with the rest of the buffer readable
      if (sh.rc != UGPU_HALO || sh.rend == len) break;
      sh.rend = len;
      if ((sh.rc = shard_load(sh, src_buf, src_host, src_dev)) != UGPU_OK) return;
    }
    if (sh.rc) return;
    if (t.count != n) {
      sh.rc = fail(UGPU_DEVICE, "shard re-scan disagrees with the stitched count");
      return;
    }
  }
  hipError_t e;
  if ((e = sh.ws->reserve_out(n)) != hipSuccess) {
    sh.rc = hip_fail(e, "match list");
    return;
  }
  if ((sh.rc = ugpu_scan_offsets(sh.sc, sh.ws->d_start, sh.ws->d_len, sh.ws->d_cap, n, sh.ws->st)) != UGPU_OK) return;
  if ((e = hipMemcpyAsync(r->start + sh.base, sh.ws->d_start, n * 8, hipMemcpyDeviceToHost, sh.ws->st)) != hipSuccess ||
      (e = hipMemcpyAsync(r->len + sh.base, sh.ws->d_len, n * 4, hipMemcpyDeviceToHost, sh.ws->st)) != hipSuccess ||
      (e = hipMemcpyAsync(r->cap + sh.base, sh.ws->d_cap, n * 4, hipMemcpyDeviceToHost, sh.ws->st)) != hipSuccess ||
      (e = hipStreamSynchronize(sh.ws->st)) != hipSuccess)
    sh.rc = hip_fail(e, "hipMemcpy matches");
}

}  // namespace
}  // extern "C"
namespace {
// f(shard) on one host thread per shard
template <class F>
void each_shard(std::vector<Shard>& shards, F f)
{
  std::vector<std::thread> th;
  th.reserve(shards.size());
  for (Shard& sh : shards) th.emplace_back([&sh, &f] { f(sh); });
  for (std::thread& t : th) t.join();
}
}  // namespace
extern "C" {

int ugpu_find_all_multi(const ugpu_dfa* dfa, const uint8_t* buf, uint64_t len, uint64_t start, uint32_t mode,
                        int ndev, ugpu_result** out)
{
  if (!dfa || !out || (!buf && len)) return fail(UGPU_INVAL, "NULL argument");
  if (mode != UGPU_MODE_COUNT && mode != UGPU_MODE_OFFSETS) return fail(UGPU_INVAL, "unknown mode");
  *out = nullptr;
  if (start > len) start = len;
  int devices = 0, cur = 0;
  HIP_TRY(hipGetDeviceCount(&devices));
  HIP_TRY(hipGetDevice(&cur));
  if (devices < 1) return fail(UGPU_DEVICE, "no device");
  if (ndev <= 0) ndev = devices;
  // tiny ranges: one device
  const uint64_t span = len - start;
  if (ndev == 1 || span < (uint64_t)ndev * 4096) return ugpu_find_all(dfa, buf, len, start, mode, out);
  bool host = true;
  int src_dev = cur;
  {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, buf) == hipSuccess && a.type == hipMemoryTypeDevice) {
      host = false;
      src_dev = a.device;
    } else {
      (void)hipGetLastError();
    }
  }
  const uint64_t halo = env_u64("UGPU_MULTI_HALO", 1ull << 20);
  std::vector<Shard> shards((size_t)ndev);
  for (int k = 0; k < ndev; ++k) {
    Shard& sh = shards[(size_t)k];
    sh.dev = k % devices;
    sh.lo = start + span * (uint64_t)k / (uint64_t)ndev;
    sh.hi = start + span * (uint64_t)(k + 1) / (uint64_t)ndev;
    sh.org = sh.lo > 4 ? sh.lo - 4 : 0;
    sh.rend = sh.hi + halo < len ? sh.hi + halo : len;
    sh.tab = dfa;
  }
  int rc = UGPU_OK;
  auto finish = [&](int code) {
    for (Shard& sh : shards) {
      if (sh.ws) {
        (void)hipSetDevice(sh.dev);
        (void)hipStreamSynchronize(sh.ws->st);
        find_ws_release(sh.ws);
      }
      if (sh.sc) scanner_release(sh.tab, sh.sc);
    }
    (void)hipSetDevice(cur);
    return code;
  };
  each_shard(shards, [&](Shard& sh) { shard_scan(sh, buf, len, host, src_dev, mode); });
  for (Shard& sh : shards)
    if (sh.rc) return finish(sh.rc);
  // resolve the chains left to right: shard k's speculative entry (its start)
  // is right iff shard k-1's exit is there; otherwise re-enter it at that exit
  for (size_t k = 1; k < shards.size(); ++k) {
    Shard& sh = shards[k];
    const uint64_t e = shards[k - 1].exit;
    if (e == sh.entry) continue;
    if (e >= sh.hi) {  // the previous shard's last match covers this whole shard
      sh.tot.count = sh.tot.digest = sh.tot.dcap = 0;
      sh.entry = e;
      sh.exit = e;
      continue;
    }
    ugpu_totals d{};
    const hipError_t he = hipSetDevice(sh.dev);
    if (he != hipSuccess) return finish(hip_fail(he, "hipSetDevice"));
    for (;;) {
      rc = ugpu_chain_fix(sh.sc, sh.dbuf, sh.lo - sh.org, sh.hi - sh.org, sh.rend - sh.org, sh.rend == len, sh.org,
                          sh.entry - sh.org, e - sh.org, &d, sh.ws->st);
      // the chain from the true entry may walk past the halo the speculative
      // scan needed: again with the rest of the buffer readable
      if (rc != UGPU_HALO || sh.rend == len) break;
      sh.rend = len;
      if ((rc = shard_load(sh, buf, host, src_dev)) != UGPU_OK) break;
    }
    if (rc) return finish(rc);
    sh.tot.count += d.count;
    sh.tot.digest += d.digest;
    sh.tot.dcap += d.dcap;
    sh.entry = e;
    if (d.exit != ~0ull) sh.exit = d.exit + sh.org;
  }
  ugpu_result* r = result_alloc();
  if (!r) return finish(fail(UGPU_NOMEM, "host allocation"));
  for (Shard& sh : shards) {
    sh.base = r->count;
    r->count += sh.tot.count;
    r->digest += sh.tot.digest;
    r->dcap += sh.tot.dcap;
  }
  if (mode == UGPU_MODE_OFFSETS && r->count > 0) {
    const uint64_t n = r->count;
    r->start = static_cast<uint64_t*>(std::malloc(n * 8));
    r->len = static_cast<uint32_t*>(std::malloc(n * 4));
    r->cap = static_cast<uint32_t*>(std::malloc(n * 4));
    if (!r->start || !r->len || !r->cap) {
      ugpu_result_free(r);
      return finish(fail(UGPU_NOMEM, "match list allocation"));
    }
    each_shard(shards, [&](Shard& sh) { shard_records(sh, buf, host, src_dev, len, r); });
    for (Shard& sh : shards)
      if (sh.rc) {
        ugpu_result_free(r);
        return finish(sh.rc);
      }
  }
  *out = r;
  return finish(UGPU_OK);
}

// ---------------------------------------------------------------- lines
namespace {

// Per-call scratch of ugpu_lines, pooled per device so that repeated calls do
// no hipMalloc/hipFree (hipFree synchronises the device): per-wave counts and
// prefixes, per-wave -c records, quarter counts (sparse mode) and pinned host
// copies of the counts and records.
struct LinesWs {
  int dev = -1;
  uint64_t nw_cap = 0, q_cap = 0;
  uint64_t* d_cnt = nullptr;
  uint64_t* d_pre = nullptr;
  LineRec* d_rec = nullptr;
  uint16_t* d_qc = nullptr;
  uint64_t* h_cnt = nullptr;
  uint64_t* h_pre = nullptr;
  LineRec* h_rec = nullptr;

  void release_wave_arrays()
  {
    (void)hipFree(d_cnt);
    (void)hipFree(d_pre);
    (void)hipFree(d_rec);
    (void)hipHostFree(h_cnt);
    (void)hipHostFree(h_pre);
    (void)hipHostFree(h_rec);
    d_cnt = d_pre = nullptr;
    d_rec = nullptr;
    h_cnt = h_pre = nullptr;
    h_rec = nullptr;
    nw_cap = 0;
  }

  hipError_t reserve(uint64_t nw, uint64_t quarters)
  {
    hipError_t e = hipSuccess;
    if (nw > nw_cap) {
      release_wave_arrays();
      if ((e = hipMalloc(&d_cnt, nw * 8)) != hipSuccess || (e = hipMalloc(&d_pre, nw * 8)) != hipSuccess ||
          (e = hipMalloc(&d_rec, nw * sizeof(LineRec))) != hipSuccess ||
          (e = hipHostMalloc(&h_cnt, nw * 8)) != hipSuccess || (e = hipHostMalloc(&h_pre, nw * 8)) != hipSuccess ||
          (e = hipHostMalloc(&h_rec, nw * sizeof(LineRec))) != hipSuccess) {
        release_wave_arrays();
        return e;
      }
      nw_cap = nw;
    }
    if (quarters > q_cap) {
      (void)hipFree(d_qc);
      d_qc = nullptr;
      q_cap = 0;
      if ((e = hipMalloc(&d_qc, quarters * 2)) != hipSuccess) return e;
      q_cap = quarters;
    }
    return e;
  }
};

std::mutex g_lines_mu;
std::vector<LinesWs*> g_lines_pool;  // idle workspaces (kept for the process lifetime)

LinesWs* lines_ws_acquire(int dev)
{
  std::lock_guard<std::mutex> lk(g_lines_mu);
  for (size_t i = 0; i < g_lines_pool.size(); ++i)
    if (g_lines_pool[i]->dev == dev) {
      LinesWs* w = g_lines_pool[i];
      g_lines_pool.erase(g_lines_pool.begin() + (long)i);
      return w;
    }
  LinesWs* w = new (std::nothrow) LinesWs;
  if (w) w->dev = dev;
  return w;
}

void lines_ws_release(LinesWs* w)
{
  std::lock_guard<std::mutex> lk(g_lines_mu);
  g_lines_pool.push_back(w);
}

}  // namespace

int ugpu_lines(const uint8_t* dbuf, uint64_t len, const uint64_t* d_start, uint64_t n, uint64_t* d_line,
               uint64_t* newlines, uint64_t* matching_lines, void* stream)
{
  if (!dbuf || (n && !d_start)) return fail(UGPU_INVAL, "NULL argument");
  if (reinterpret_cast<uintptr_t>(dbuf) & 15u) return fail(UGPU_INVAL, "buffer must be 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t tile = lines_tile();
  int dev = 0, cus = 256;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // wave ranges: whole tiles, about 16 waves per CU, at most kMaxRec records
  const uint64_t tiles = (len + tile - 1) / tile;
  uint64_t want = (uint64_t)cus * 16;
  if (want > (uint64_t)kMaxRec) want = kMaxRec;
  uint64_t tpw = tiles ? (tiles + want - 1) / want : 1;
  while (tpw * tile > kMaxRecBytes) --tpw;  // (never for sane sizes; 32-bit offsets)
  if (tpw == 0) tpw = 1;
  const uint64_t nw = tiles ? (tiles + tpw - 1) / tpw : 1;
  // sparse assign pass when matches are rarer than one per two quarters
  // (UGPU_LINES_MODE=1/2 forces dense/sparse, for tests)
  const uint64_t quarters = tiles * (tile / kLinesQuarter);
  bool sparse = n > 0 && n * 2 < quarters;
  if (const char* mo = getenv("UGPU_LINES_MODE")) {
    if (mo[0] == '1') sparse = false;
    if (mo[0] == '2') sparse = n > 0;
  }
  LinesWs* ws = lines_ws_acquire(dev);
  if (!ws) return fail(UGPU_NOMEM, "lines workspace");
  hipError_t e = ws->reserve(nw, sparse ? quarters : 0);
  if (e != hipSuccess) {
    lines_ws_release(ws);
    return hip_fail(e, "lines buffers");
  }
  LinesParams L{};
  L.g = dbuf;
  L.len = len;
  L.per = tpw * tile;
  L.nwaves = nw;
  L.starts = d_start;
  L.nmatch = n;
  L.lines = d_line;
  L.counts = ws->d_cnt;
  L.prefix = ws->d_pre;
  L.recs = ws->d_rec;
  L.qcount = sparse ? ws->d_qc : nullptr;
  int rc = UGPU_OK;
  if ((e = launch_nl_count(L, sparse, st)) != hipSuccess ||
      (e = hipMemcpyAsync(ws->h_cnt, ws->d_cnt, nw * 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (e = hipStreamSynchronize(st)) != hipSuccess) {
    rc = hip_fail(e, "newline count");
  } else {
    uint64_t total = 0;
    for (uint64_t i = 0; i < nw; ++i) {
      ws->h_pre[i] = total;
      total += ws->h_cnt[i];
    }
    if (newlines) *newlines = total;
    if (n > 0 || matching_lines) {
      if ((e = hipMemcpyAsync(ws->d_pre, ws->h_pre, nw * 8, hipMemcpyHostToDevice, st)) != hipSuccess ||
          (e = launch_nl_assign(L, sparse, st)) != hipSuccess ||
          (e = hipMemcpyAsync(ws->h_rec, ws->d_rec, nw * sizeof(LineRec), hipMemcpyDeviceToHost, st)) !=
              hipSuccess ||
          (e = hipStreamSynchronize(st)) != hipSuccess) {
        rc = hip_fail(e, "line assignment");
      } else {
        // lines of consecutive matches in different waves may coincide
        uint64_t lines = 0, last = 0;
        bool any = false;
        for (uint64_t i = 0; i < nw; ++i) {
          const LineRec& r = ws->h_rec[i];
          if (!r.nmatch) continue;
          lines += r.trans;
          if (any && r.first_line == last) --lines;
          last = r.last_line;
          any = true;
        }
        if (matching_lines) *matching_lines = lines;
      }
    }
  }
  lines_ws_release(ws);
  return rc;
}

// ---------------------------------------------------------------- binary detection
namespace {

// One device result slot and its pinned host copy, pooled per device.
struct SlotWs {
  int dev = -1;
  uint64_t* d = nullptr;
  uint64_t* h = nullptr;
};
std::mutex g_slot_mu;
std::vector<SlotWs*> g_slot_pool;

SlotWs* slot_acquire(int dev)
{
  {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    for (size_t i = 0; i < g_slot_pool.size(); ++i)
      if (g_slot_pool[i]->dev == dev) {
        SlotWs* w = g_slot_pool[i];
        g_slot_pool.erase(g_slot_pool.begin() + (long)i);
        return w;
      }
  }
  SlotWs* w = new (std::nothrow) SlotWs;
  if (!w) return nullptr;
  w->dev = dev;
  if (hipMalloc(&w->d, 8) != hipSuccess || hipHostMalloc(&w->h, 8) != hipSuccess) {
    (void)hipFree(w->d);
    delete w;
    return nullptr;
  }
  return w;
}

void slot_release(SlotWs* w)
{
  std::lock_guard<std::mutex> lk(g_slot_mu);
  g_slot_pool.push_back(w);
}

// First failing byte of dbuf[0, len) (isutf8, or NUL with nul) or ~0.
int utf8_scan(const uint8_t* dbuf, uint64_t len, bool nul, uint64_t* pos, void* stream)
{
  if (!dbuf && len) return fail(UGPU_INVAL, "NULL buffer");
  if (!pos) return fail(UGPU_INVAL, "NULL result pointer");
  *pos = ~0ull;
  if (len == 0) return UGPU_OK;
  if (!is_device_ptr(dbuf)) return fail(UGPU_INVAL, "buffer must be device memory");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  Utf8Params U = utf8_params(dbuf, len);
  SlotWs* w = slot_acquire(dev);
  if (!w) return fail(UGPU_NOMEM, "result slot");
  U.out = w->d;
  hipError_t e;
  int rc = UGPU_OK;
  if ((e = hipMemsetAsync(w->d, 0xff, 8, st)) != hipSuccess || (e = launch_utf8(U, nul, st)) != hipSuccess ||
      (e = hipMemcpyAsync(w->h, w->d, 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (e = hipStreamSynchronize(st)) != hipSuccess) {
    rc = hip_fail(e, nul ? "NUL scan" : "UTF-8 check");
  } else {
    *pos = *w->h == ~0ull ? ~0ull : *w->h - U.head;
  }
  slot_release(w);
  return rc;
}

}  // namespace

int ugpu_check_utf8(const uint8_t* dbuf, uint64_t len, uint64_t* first_bad, void* stream)
{
  return utf8_scan(dbuf, len, false, first_bad, stream);
}

int ugpu_find_nul(const uint8_t* dbuf, uint64_t len, uint64_t* pos, void* stream)
{
  return utf8_scan(dbuf, len, true, pos, stream);
}

int ugpu_is_binary(const uint8_t* dbuf, uint64_t len, uint32_t flags, int* binary, void* stream)
{
  if (!binary) return fail(UGPU_INVAL, "NULL result pointer");
  *binary = 0;
  if (flags & UGPU_BIN_INIT_WINDOW) {
    // GrepWorker::init_is_binary (src/ugrep.cpp:3998-4015): do not judge a
    // UTF-8 sequence cut off by the window end
    if (len == 0) return UGPU_OK;
    uint8_t tail[4] = {0, 0, 0, 0};
    const uint64_t nt = len < 4 ? len : 4;
    HIP_TRY(hipMemcpy(tail + (4 - nt), dbuf + len - nt, nt, hipMemcpyDeviceToHost));
    const uint8_t* t = tail + 4;  // t[-1] = last byte
    uint64_t avail = len;
    if ((t[-1] & 0x80) == 0x80) {
      uint64_t n = nt;
      while (n > 0 && (t[(int64_t)(--avail) - (int64_t)len] & 0xc0) == 0x80) --n;
      if ((t[(int64_t)avail - (int64_t)len] & 0xc0) != 0xc0) {
        *binary = 1;
        return UGPU_OK;
      }
    }
    len = avail;
  }
  // is_binary (src/ugrep.cpp:699-711)
  if (flags & UGPU_BIN_NULL_DATA) return UGPU_OK;
  uint64_t pos = ~0ull;
  const int rc = utf8_scan(dbuf, len, (flags & UGPU_BIN_NUL_ONLY) != 0, &pos, stream);
  if (rc == UGPU_OK) *binary = pos != ~0ull;
  return rc;
}

// ---------------------------------------------------------------- streaming
// Device buffer holds a context prefix (the up to 4 bytes before the settled
// chain position: at_wb's code point for option W, at_bol's byte for line
// anchors), the unsettled carry and the new chunk; each feed scans [ctx, hi)
// of it with the chain entering at ctx (the previous settled exit), readable
// to the end, and carries [exit - 4, n) into the other buffer.
struct ugpu_stream {
  const ugpu_dfa* dfa = nullptr;
  ugpu_scanner* sc = nullptr;  // pooled (scanner_acquire)
  FindWs* ws = nullptr;        // pooled: private stream, the two buffers, pinned match lists
  uint64_t keep = 0;
  int cur = 0;         // buffer holding the carry
  uint64_t carry = 0;  // bytes at buf[cur][0..carry): the prefix, then the unsettled bytes
  uint64_t ctx = 0;    // prefix bytes (4, or fewer at the stream's start: buf[cur][0] is its first byte)
  uint64_t base = 0;   // absolute offset of buf[cur][ctx] = the settled chain position
  bool done = false;
};

namespace {

// The stream's resources come from the pools ugpu_find_all uses (a scanner of
// the table, a per-device workspace): creating a stream per input costs no
// device allocation once the pools are warm, and no call of a feed touches
// the null stream or frees device memory (hipFree synchronises the device, so
// ugrep's workers would wait on each other; VERDICT r4 item 6's trace)
int stream_grow(ugpu_stream* st, uint64_t need)
{
  FindWs* w = st->ws;
  if (need <= w->sb_cap) return UGPU_OK;
  uint64_t c = w->sb_cap ? w->sb_cap : (1ull << 20);
  while (c < need) c *= 2;
  uint8_t* nb[2] = {nullptr, nullptr};
  for (int i = 0; i < 2; ++i) {
    hipError_t e = hipMalloc(&nb[i], c + 16);
    if (e != hipSuccess) {
      if (nb[0]) (void)hipFree(nb[0]);
      return hip_fail(e, "stream buffer");
    }
  }
  if (st->carry) {
    hipError_t e = hipMemcpyAsync(nb[0], w->d_sb[st->cur], st->carry, hipMemcpyDeviceToDevice, w->st);
    if (e == hipSuccess) e = hipStreamSynchronize(w->st);
    if (e != hipSuccess) {
      (void)hipFree(nb[0]);
      (void)hipFree(nb[1]);
      return hip_fail(e, "stream carry copy");
    }
  }
  for (int i = 0; i < 2; ++i)
    if (w->d_sb[i]) (void)hipFree(w->d_sb[i]);
  w->d_sb[0] = nb[0];
  w->d_sb[1] = nb[1];
  st->cur = 0;
  w->sb_cap = c;
  return UGPU_OK;
}

// a pinned block of the workspace with no live result and room for m records
// (grown here), or null (both lent out: the caller copies into malloc()ed arrays)
PinBlk* stream_pin(FindWs* w, uint64_t m)
{
  for (PinBlk& b : w->pin) {
    if (b.refs.load(std::memory_order_acquire) != 0) continue;
    if (b.cap < m) {
      // (from the pinned pool: non-coherent, so the host's reads of the
      // records are cached)
      if (b.p) pinned_put(b.p, b.bytes);
      b.p = nullptr;
      b.cap = b.cap_n = 0;
      b.bytes = 0;
      size_t got = 0;
      b.p = pinned_get((m + m / 4 + 1024) * 16, got);
      if (!b.p) return nullptr;
      b.bytes = got;
      b.cap = got / 16;
    }
    return &b;
  }
  return nullptr;
}

}  // namespace

int ugpu_stream_create(const ugpu_dfa* dfa, uint64_t keep, ugpu_stream** out)
{
  if (!dfa || !out) return fail(UGPU_INVAL, "NULL argument");
  *out = nullptr;
  ugpu_stream* st = new (std::nothrow) ugpu_stream();
  if (!st) return fail(UGPU_NOMEM, "host allocation");
  int dev = 0;
  int rc = hipGetDevice(&dev) == hipSuccess ? dfa_on(dfa, dev, &dfa) : fail(UGPU_DEVICE, "hipGetDevice");
  if (rc) {
    delete st;
    return rc;
  }
  st->dfa = dfa;
  st->keep = keep ? keep : (64ull << 10);
  // (a records consumer's scanner: the drop-in matcher feeds in OFFSETS mode)
  rc = scanner_acquire(dfa, &st->sc, true);
  if (rc) {
    delete st;
    return rc;
  }
  st->ws = find_ws_acquire(dev);
  if (!st->ws) {
    scanner_release(dfa, st->sc);
    delete st;
    return fail(UGPU_NOMEM, "stream workspace");
  }
  *out = st;
  return UGPU_OK;
}

int ugpu_stream_destroy(ugpu_stream* st)
{
  if (!st || exiting()) return UGPU_OK;
  (void)hipStreamSynchronize(st->ws->st);
  st->sc->bol0 = 1;
  scanner_release(st->dfa, st->sc);
  find_ws_release(st->ws);
  delete st;
  return UGPU_OK;
}

uint64_t ugpu_stream_settled(const ugpu_stream* st) { return st ? st->base : 0; }

int ugpu_stream_reserve(const ugpu_dfa* dfa, int n, uint64_t feed_bytes)
{
  if (!dfa || n < 0) return fail(UGPU_INVAL, "NULL table or negative count");
  if (n > 256) n = 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(UGPU_DEVICE, "hipGetDevice");
  int rc = dfa_on(dfa, dev, &dfa);
  if (rc) return rc;
  // (every item is acquired before any is released, so the pools end up
  // holding n distinct ones)
  const uint64_t need = feed_bytes + (64ull << 10) + 16;  // a feed plus its carry
  uint64_t c = 1ull << 20;
  while (c < need) c *= 2;
  const uint64_t recs = feed_bytes / 8 + 1024;  // (a guess: a list that is longer grows)
  std::vector<ugpu_scanner*> scs;
  std::vector<FindWs*> wss;
  for (int i = 0; i < n && !rc; ++i) {
    ugpu_scanner* s = nullptr;
    rc = scanner_acquire(dfa, &s, true);
    if (rc) break;
    scs.push_back(s);
    if (s->xc && !s->word && env_u64("UGPU_XC_BITMAP", 1) != 0) {
      // (the In bits of a COUNT pass over a whole buffer, as ugpu_scan sizes them)
      const uint64_t nb = ((((c + 16 + 15) & ~uint64_t(15)) + 2048) >> 3) + 64;
      if (nb > s->inbits_cap) {
        (void)hipFree(s->d_inbits);
        s->d_inbits = nullptr;
        s->inbits_cap = 0;
        if (hipMalloc(&s->d_inbits, nb + nb / 8) == hipSuccess)
          s->inbits_cap = nb + nb / 8;
        else
          (void)hipGetLastError();
      }
    }
    FindWs* w = find_ws_acquire(dev);
    if (!w) {
      rc = fail(UGPU_NOMEM, "stream workspace");
      break;
    }
    wss.push_back(w);
    if (w->sb_cap < c) {
      for (int k = 0; k < 2; ++k) {
        (void)hipFree(w->d_sb[k]);
        w->d_sb[k] = nullptr;
      }
      w->sb_cap = 0;
      hipError_t e = hipMalloc(&w->d_sb[0], c + 16);
      if (e == hipSuccess) e = hipMalloc(&w->d_sb[1], c + 16);
      if (e != hipSuccess) {
        rc = hip_fail(e, "stream buffer");
        break;
      }
      w->sb_cap = c;
    }
    hipError_t e = w->reserve_out(recs);
    if (e != hipSuccess) {
      rc = hip_fail(e, "stream match list");
      break;
    }
    if (env_u64("UGPU_RESERVE_PIN", 0) != 0 && !stream_pin(w, recs)) rc = fail(UGPU_NOMEM, "pinned match list");
  }
  for (ugpu_scanner* s : scs) scanner_release(dfa, s);
  for (FindWs* w : wss) find_ws_release(w);
  return rc;
}

int ugpu_stream_feed(ugpu_stream* st, const uint8_t* chunk, uint64_t len, int final, uint32_t mode, ugpu_result** out)
{
  if (!st || !out || (!chunk && len)) return fail(UGPU_INVAL, "NULL argument");
  if (st->done) return fail(UGPU_INVAL, "stream already ended (final chunk fed)");
  if (final != 0 && final != 1 && final != UGPU_FEED_FLUSH) return fail(UGPU_INVAL, "final: 0, 1 or UGPU_FEED_FLUSH");
  const bool flush = final == UGPU_FEED_FLUSH;
  final = final == 1;
  *out = nullptr;
  FindWs* w = st->ws;
  hipStream_t hs = w->st;
  const uint64_t n = st->carry + len;
  int rc = stream_grow(st, n);
  if (rc) return rc;
  uint8_t* b = w->d_sb[st->cur];
  if (len) {
    HIP_TRY(hipMemcpyAsync(b + st->carry, chunk, len, hipMemcpyHostToDevice, hs));
  }
  ugpu_result* r = result_alloc();
  if (!r) return fail(UGPU_NOMEM, "host allocation");
  ugpu_scanner_context(st->sc, 1);  // (buf[cur][0] is the stream's first byte or 4 bytes before lo)
  const uint64_t lo = st->ctx, bias = st->base - lo;
  const bool offsets = mode == UGPU_MODE_OFFSETS;
  // settle the chain up to `keep` bytes before the end (all of it when final);
  // a walk still open at the end of the bytes so far means hi was too close
  uint64_t hi = final ? n : (n > lo + st->keep ? n - st->keep : lo);
  uint64_t exit = lo;
  ugpu_totals tot{};
  if (flush && !final) {
    // settle as far as the bytes decide: the largest hi whose chain has no walk
    // open at the end (the start of the last, still open match) -- step back
    // from the end by 16, 64, 256, ... bytes, then bisect between the last hi
    // that was too close and the first that was not
    auto try_hi = [&](uint64_t h) -> int {
      st->sc->stage_once = offsets;
      int c = ugpu_scan(st->sc, b, lo, h, n, 0, bias, hs);
      if (!c) c = ugpu_scan_totals(st->sc, &tot);
      return c;
    };
    uint64_t good = lo, bad = n + 1, h = n, back = 16, last = ~0ull;
    while (h > lo) {
      rc = try_hi(h);
      last = h;
      if (rc == UGPU_OK) {
        good = h;
        break;
      }
      if (rc != UGPU_HALO) {
        ugpu_result_free(r);
        return rc;
      }
      bad = h;
      h = n > lo + back ? n - back : lo;
      back *= 4;
    }
    while (bad - good > 1) {
      const uint64_t mid = good + (bad - good) / 2;
      rc = try_hi(mid);
      last = mid;
      if (rc == UGPU_OK) {
        good = mid;
      } else if (rc == UGPU_HALO) {
        bad = mid;
      } else {
        ugpu_result_free(r);
        return rc;
      }
    }
    hi = good;
    rc = UGPU_OK;
    if (hi > lo && last != hi) rc = try_hi(hi);  // (the scanner holds the last scan)
    if (rc) {
      ugpu_result_free(r);
      return rc;
    }
    exit = hi > lo ? tot.exit : lo;
  }
  while (hi > lo && !(flush && !final)) {
    st->sc->stage_once = offsets;  // (single-pass OFFSETS for prefiltered tables)
    rc = ugpu_scan(st->sc, b, lo, hi, n, final ? 1 : 0, bias, hs);
    if (!rc) rc = ugpu_scan_totals(st->sc, &tot);
    if (rc == UGPU_HALO && !final) {
      hi = lo + (hi - lo) / 2;
      continue;
    }
    if (rc) {
      ugpu_result_free(r);
      return rc;
    }
    exit = final ? n : tot.exit;
    break;
  }
  if (hi > lo) {
    r->count = tot.count;
    r->digest = tot.digest;
    r->dcap = tot.dcap;
    if (offsets && tot.count > 0) {
      // records into the workspace's device lists, then one copy into a pinned
      // block the result borrows (single-accept tables: no cap array on the
      // device; the block's cap array holds the accept index already)
      const uint64_t m = tot.count;
      const uint32_t cap1 = st->dfa->t.cap1;
      const bool one = cap1 != 0 && !st->dfa->t.anchored;
      hipError_t e = w->reserve_out(m);
      if (e != hipSuccess) rc = hip_fail(e, "stream match list");
      if (!rc) rc = ugpu_scan_offsets(st->sc, w->d_start, w->d_len, one ? nullptr : w->d_cap, m, hs);
      PinBlk* pb = rc ? nullptr : stream_pin(w, m);
      uint64_t* hstart = nullptr;
      uint32_t *hlen = nullptr, *hcap = nullptr;
      if (!rc && pb) {
        hstart = reinterpret_cast<uint64_t*>(pb->p);
        hlen = reinterpret_cast<uint32_t*>(pb->p + pb->cap * 8);
        hcap = reinterpret_cast<uint32_t*>(pb->p + pb->cap * 12);
      } else if (!rc) {
        hstart = static_cast<uint64_t*>(std::malloc(m * 8));
        hlen = static_cast<uint32_t*>(std::malloc(m * 4));
        hcap = static_cast<uint32_t*>(std::malloc(m * 4));
        r->start = hstart;
        r->len = hlen;
        r->cap = hcap;
        if (!hstart || !hlen || !hcap) rc = fail(UGPU_NOMEM, "stream match list");
      }
      if (!rc && ((e = hipMemcpyAsync(hstart, w->d_start, m * 8, hipMemcpyDeviceToHost, hs)) != hipSuccess ||
                  (e = hipMemcpyAsync(hlen, w->d_len, m * 4, hipMemcpyDeviceToHost, hs)) != hipSuccess ||
                  (!one && (e = hipMemcpyAsync(hcap, w->d_cap, m * 4, hipMemcpyDeviceToHost, hs)) != hipSuccess)))
        rc = hip_fail(e, "stream match list copy");
      if (!rc && one) {
        // (while the copies run)
        if (pb && pb->cap_v == cap1 && pb->cap_n >= m) {
        } else {
          std::fill(hcap, hcap + m, cap1);
          if (pb) {
            pb->cap_v = cap1;
            pb->cap_n = m;
          }
        }
      } else if (!rc && pb) {
        pb->cap_n = 0;  // (the cap array now holds copied accept indices)
      }
      if (!rc && (e = hipStreamSynchronize(hs)) != hipSuccess) rc = hip_fail(e, "stream match list copy");
      if (rc) {
        (void)hipStreamSynchronize(hs);
        ugpu_result_free(r);
        return rc;
      }
      if (pb) {
        pb->refs.fetch_add(1, std::memory_order_acq_rel);
        reinterpret_cast<ResBox*>(r)->pin = pb;
        r->start = hstart;
        r->len = hlen;
        r->cap = hcap;
      }
    }
  }
  // carry [exit - ctx', n) to the other buffer, ctx' = the up to 4 bytes before
  // the exit (fewer only when they reach the stream's first byte); the chain
  // resumes at the byte after them
  const uint64_t nctx = exit < 4 ? exit : 4;  // (exit >= lo: buf[cur][0] is the first byte when exit < 4)
  const uint64_t keep_n = n - exit + nctx;
  if (keep_n) {
    hipError_t e = hipMemcpyAsync(w->d_sb[1 - st->cur], b + exit - nctx, keep_n, hipMemcpyDeviceToDevice, hs);
    if (e == hipSuccess) e = hipStreamSynchronize(hs);
    if (e != hipSuccess) {
      ugpu_result_free(r);
      return hip_fail(e, "stream carry copy");
    }
  }
  st->cur = 1 - st->cur;
  st->carry = keep_n;
  st->ctx = nctx;
  st->base += exit - lo;
  if (final) st->done = true;
  *out = r;
  return UGPU_OK;
}

int ugpu_result_free(ugpu_result* r)
{
  if (!r) return UGPU_OK;
  ResBox* b = reinterpret_cast<ResBox*>(r);  // (r is the head of its box: result_alloc)
  if (b->pin) {
    b->pin->refs.fetch_sub(1, std::memory_order_release);
  } else {
    std::free(r->start);
    std::free(r->len);
    std::free(r->cap);
  }
  std::free(b);
  return UGPU_OK;
}

int ugpu_gen(int kind, uint64_t seed, uint64_t off, uint8_t* dbuf, uint64_t len, void* stream)
{
  if (kind < 1 || kind > 4) return fail(UGPU_INVAL, "unknown corpus kind");
  if (!dbuf && len) return fail(UGPU_INVAL, "NULL buffer");
  HIP_TRY(launch_gen(kind, seed, off, dbuf, len, reinterpret_cast<hipStream_t>(stream)));
  return UGPU_OK;
}

}  // extern "C"
