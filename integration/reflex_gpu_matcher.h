// reflex_gpu_matcher.h -- drop-in FIND matcher for ugrep: a reflex::Matcher
// whose FIND is served by the MI355X engine (include/ugpu.h).  This is the
// reference-side binding of INTEGRATION.md; it includes the reference's
// <reflex/matcher.h> and uses only its public and protected interface.
//
// Drop-in: GpuMatcher(pattern, input, opt) has reflex::Matcher's constructor
// (include/reflex/matcher.h, Matcher(const Pattern&, const Input&, const char*)),
// so ugrep's construction site src/ugrep.cpp:8902
//     new reflex::Matcher(Static::reflex_pattern, reflex::Input(), matcher_options.c_str())
// becomes new reflex::GpuMatcher(...) and nothing else changes.  The device
// tables are compiled from the regex the Pattern holds, read through its public
// Pattern::operator[](0) (include/reflex/pattern.h:302) with
// ugpu_compile(..., UGPU_RX_REFLEX): no private Pattern member is touched.
//
// Override point: virtual size_t Matcher::match(Method)
// (include/reflex/matcher.h:1321, called by AbstractMatcher::find
// include/reflex/absmatcher.h:276-280, :1401; ugrep's loop
// `while (matcher->find())` src/ugrep.cpp:10544).
//
// Whole buffers (buffer(), absmatcher.h:542-591: eof_ set, own_ clear): one
// GPU scan from cur_ at the first call, then one (start, len, accept) record
// per call, leaving the matcher in the state lib/matcher.cpp:682-746 leaves
// after a hit:
//   txt_ = buf_ + start, len_ = len, cap_ = accept, cur_ = pos_ = start + len,
//   got_ = buf_[cur_-1] (set_current, absmatcher.h:1571-1580)
// and after exhaustion cap_ = len_ = 0, cur_ = pos_ = end_.
//
// Streamed input (input(): stdin, pipes, decompressed data, files ugrep does
// not mmap, src/ugrep.cpp:3936-3944): the matcher keeps reading into its own
// buffer with the reference's protocol (grow() + get(), absmatcher.h:1417-1593,
// so buffer shifts, line counting and ugrep's flush handler behave as on the
// CPU) and feeds the new bytes to a ugpu_stream in chunks of at least
// UGPU_ADAPTER_CHUNK bytes (default 2 MiB); settled records come back with absolute offsets
// (num_ + buffer position).
//
// Between finds the caller may move cur_ (skip('\n') for -c, --range, context
// modes: src/ugrep.cpp:10583, :3989).  The FIND chain passes through every
// position that is not strictly inside a match, so the remaining records are
// exact whenever the new cur_ is not inside one; otherwise (and for new bytes
// or a rewind) the scan restarts at cur_.
//
// Dispatch (tools/bench_adapter.py):
//   * inputs shorter than UGPU_ADAPTER_MIN_BYTES (default 4 MiB for sparse
//     tables, 64 KiB for dense ones; a stream counts when it ends before its
//     first feed) stay on the CPU matcher: a device round trip costs more than
//     the reference's scan of a small buffer;
//   * patterns with a selective prefilter (sparse_kernel, e.g. foo|bar|baz) go
//     through a per-device queue of UGPU_ADAPTER_SPARSE_MAX (default 2) slots:
//     host buffers cross PCIe at ~55 GB/s per device link, which a few
//     reference AVX2 cores match on such patterns (11 GB/s each), so an input
//     that finds every slot taken is scanned by the CPU matcher meanwhile (with
//     ugrep's workers the GPU and the cores scan at once); dense patterns
//     (C3/C4 class, ~0.2-2 GB/s per core) always take the GPU;
//   * devices: matchers are dealt round-robin over the visible devices
//     (ugpu_select_device before every engine call), and a buffer of at least
//     UGPU_ADAPTER_MULTI_MIN bytes (default 64 MiB) is cut over all of them
//     (ugpu_find_all_multi: one H2D per device link).  UGPU_ADAPTER_STATS=1 prints each
// matcher's GPU scan count to stderr when it is destroyed.
//
// Option N (ugrep -Y, and -x / patterns that start with ^ or end with $, which
// turn it on: src/ugrep.cpp:8381-8386, src/cnf.hpp:201-206) runs on the GPU
// (UGPU_PAT_EMPTY), and so do line anchors when N is on and they are only a
// leading ^ and/or a trailing $ of the whole regex (anchors_outer).  Other
// anchored tables stay on the CPU: there the reference's match predictor
// (lib/pattern.cpp:4342-4430) can skip positions its DFA matches at -- ugrep -c
// 'a$|ab' prints 0 on "xa\nb\nzzzz\n", and '^\w+' without N finds nothing --
// and the GPU walks the DFA (tests/test_anchor.py records both).
//
// SCAN and MATCH (scan(), matches()) on whole buffers come from the same FIND
// records: the longest match at the cursor is the FIND record that starts
// there, if any (MATCH's empty match goes to the CPU matcher).  Everything
// else -- SPLIT, option A, streamed SCAN/MATCH, tables the engine rejects
// (lookahead, W with anchors or N: UGPU_UNSUPPORTED) -- stays on the CPU
// matcher.
#ifndef REFLEX_GPU_MATCHER_H
#define REFLEX_GPU_MATCHER_H

#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <poll.h>

#include <reflex/matcher.h>

#include "ugpu.h"

namespace reflex {

// The engine's device half.  ugrep_gpu links only the host half
// (libugpu_host.so: ugpu_compile, ugpu_dfa_plan_host, ugpu_last_error -- no HIP
// runtime); the device half (libugrep_amd.so, which links libamdhip64) is
// dlopen()ed from the directory the host half was loaded from
// (UGPU_ENGINE_LIB overrides the path) at the first input the policy sends to
// a device.  A run the CPU matcher serves end to end never loads the HIP
// runtime: loading it cost every search ~14 ms on a host without a GPU and
// ~55 ms on the GPU box.  The free functions below are
// NULL-safe and do not load the device half for a NULL handle.
struct GpuEngine {
  bool ok = false;
  decltype(&ugpu_dfa_create) dfa_create = NULL;
  decltype(&ugpu_dfa_destroy) dfa_destroy = NULL;
  decltype(&ugpu_device_count) device_count = NULL;
  decltype(&ugpu_select_device) select_device = NULL;
  decltype(&ugpu_warmup) warmup = NULL;
  decltype(&ugpu_find_all_multi) find_all_multi = NULL;
  decltype(&ugpu_find_records) find_records = NULL;
  decltype(&ugpu_records_next) records_next = NULL;
  decltype(&ugpu_records_free) records_free = NULL;
  decltype(&ugpu_result_free) result_free = NULL;
  decltype(&ugpu_stream_create) stream_create = NULL;
  decltype(&ugpu_stream_destroy) stream_destroy = NULL;
  decltype(&ugpu_stream_feed) stream_feed = NULL;
  decltype(&ugpu_abi_version) abi_version = NULL;
  decltype(&ugpu_stream_reserve) stream_reserve = NULL;

  static GpuEngine& get()
  {
    static GpuEngine e;
    static std::once_flag once;
    std::call_once(once, [] { e.load(); });
    return e;
  }
  // loaded already (without loading it)
  static bool loaded() { return loaded_flag().load(std::memory_order_acquire); }

 private:
  static std::atomic<bool>& loaded_flag()
  {
    static std::atomic<bool> f(false);
    return f;
  }
  template <class F>
  static bool sym(void* h, const char* name, F& f)
  {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != NULL;
  }
  void load()
  {
    std::string path;
    const char* env = std::getenv("UGPU_ENGINE_LIB");
    if (env != NULL && *env)
    {
      path = env;
    }
    else
    {
      Dl_info di;
      if (dladdr(reinterpret_cast<void*>(&ugpu_compile), &di) != 0 && di.dli_fname != NULL)
      {
        path = di.dli_fname;
        const size_t slash = path.rfind('/');
        path = (slash == std::string::npos ? std::string() : path.substr(0, slash + 1)) + "libugrep_amd.so";
      }
      else
      {
        path = "libugrep_amd.so";
      }
    }
    void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (h == NULL)
      return;
    ok = sym(h, "ugpu_dfa_create", dfa_create) && sym(h, "ugpu_dfa_destroy", dfa_destroy) &&
         sym(h, "ugpu_device_count", device_count) && sym(h, "ugpu_select_device", select_device) &&
         sym(h, "ugpu_warmup", warmup) && sym(h, "ugpu_find_all_multi", find_all_multi) &&
         sym(h, "ugpu_find_records", find_records) && sym(h, "ugpu_records_next", records_next) &&
         sym(h, "ugpu_records_free", records_free) && sym(h, "ugpu_result_free", result_free) &&
         sym(h, "ugpu_stream_create", stream_create) && sym(h, "ugpu_stream_destroy", stream_destroy) &&
         sym(h, "ugpu_stream_feed", stream_feed) && sym(h, "ugpu_abi_version", abi_version) &&
         sym(h, "ugpu_stream_reserve", stream_reserve) &&
         abi_version() == UGPU_ABI_VERSION;
    loaded_flag().store(true, std::memory_order_release);
    // (the handle stays open for the process lifetime)
  }
};

// NULL-safe frees that never load the device half for a NULL handle
inline void e_result_free(ugpu_result* r)
{
  if (r != NULL)
    (void)GpuEngine::get().result_free(r);
}
inline void e_stream_destroy(ugpu_stream* s)
{
  if (s != NULL)
    (void)GpuEngine::get().stream_destroy(s);
}
inline void e_records_free(ugpu_records* r)
{
  if (r != NULL)
    (void)GpuEngine::get().records_free(r);
}
inline void e_dfa_destroy(ugpu_dfa* d)
{
  if (d != NULL)
    (void)GpuEngine::get().dfa_destroy(d);
}

class GpuMatcher : public Matcher {
 public:
  /// Drop-in constructor (reflex::Matcher's).  The device tables are compiled
  /// from pattern[0] at the first FIND (and again after pattern() or a reset()
  /// that changes option W).
  GpuMatcher(const Pattern& pattern, const Input& input = Input(), const char* opt = NULL)
      : Matcher(pattern, input, opt)
  {
    init_policy();
    ++live();
  }
  /// Clones (ugrep's worker threads, src/ugrep.cpp:4146, :9006) share the
  /// device tables; per-input state starts empty.
  GpuMatcher(const GpuMatcher& m)
      : Matcher(m), tab_(m.tab_), tab_pat_(m.tab_pat_), tab_w_(m.tab_w_), tab_n_(m.tab_n_),
        tab_anchor_(m.tab_anchor_), tab_ok_(m.tab_ok_), sparse_(m.sparse_),
        min_bytes_(m.min_bytes_), chunk_(m.chunk_), multi_min_(m.multi_min_), sparse_max_(m.sparse_max_),
        warm_async_(m.warm_async_), warm_wait_(m.warm_wait_)
  {
    ++live();
  }
  virtual GpuMatcher* clone() { return new GpuMatcher(*this); }
  virtual ~GpuMatcher()
  {
    const char* st = std::getenv("UGPU_ADAPTER_STATS");
    if (st != NULL && *st == '1')
    {
      // one line per matcher: GPU scans, FIND calls answered from GPU records,
      // FIND calls the CPU matcher answered and why (UGPU_ADAPTER_STATS=1)
      std::string why;
      for (int r = 0; r < kReasons; ++r)
        if (cpu_why_[r] != 0)
          why += std::string(why.empty() ? "" : ",") + reason_name(r) + ":" + std::to_string(cpu_why_[r]);
      std::fprintf(stderr, "[ugpu-adapter] scans=%zu gpu_finds=%zu cpu_finds=%zu table=%s cpu_why=%s read_ms=%.1f feed_ms=%.1f\n",
                   scans_, gpu_finds_, cpu_finds(), tab_pat_ == NULL ? "none" : tab_ok_ ? "gpu" : "unsupported",
                   why.empty() ? "-" : why.c_str(), std::chrono::duration<double, std::milli>(t_read_).count(),
                   std::chrono::duration<double, std::milli>(t_feed_).count());
    }
    src_.clear();
    e_result_free(gres_);
    if (gst_ != NULL)
      on_device();
    e_stream_destroy(gst_);
    release_slot();
    --live();
  }
  /// New input (input() calls this, absmatcher.h:533-540) or options.
  virtual void reset(const char* opt = NULL)
  {
    Matcher::reset(opt);
    drop_records();
    release_slot();
    if (gst_ != NULL)
      on_device();
    e_stream_destroy(gst_);
    gst_ = NULL;
    cpu_stream_ = false;
    sopen_ = false;
    sfit_ = false;
  }

  /// GPU scans (whole-buffer scans and stream feeds) issued so far (tests).
  size_t gpu_scans() const { return scans_; }
  /// FIND calls answered from GPU records, and by the CPU matcher (tests).
  size_t gpu_finds() const { return gpu_finds_; }
  size_t cpu_finds() const
  {
    size_t n = 0;
    for (int r = 0; r < kReasons; ++r)
      n += cpu_why_[r];
    return n;
  }
  /// Whether the engine supports this pattern (builds the device tables if
  /// needed).
  bool gpu_ready() { return tables() != NULL; }
  /// Smallest input sent to the GPU (0: every input).
  void gpu_min_bytes(size_t n) { min_bytes_ = n; }
  /// Prefiltered (sparse) patterns: at most n GPU scans per device at once (the
  /// device queue; an input that finds every slot taken is scanned on the CPU).
  void gpu_sparse_max(int n) { sparse_max_ = n; }

 protected:
  virtual size_t match(Method method)
  {
    // (the hot path of a streamed input: FIND with the cursor where the last
    // record left it and records of the current feed pending -- nothing that
    // the checks below decide can have changed since that record: a new
    // pattern, options or input drop the records)
    if (method == Const::FIND && gres_ != NULL && gi_ < gres_->count && own_ && chr_ == '\0' &&
        num_ + cur_ == gcur_abs_ && tab_pat_ == pat_ && sopen_ && !cpu_stream_)
    {
      const uint64_t s = sbase_ + gres_->start[gi_];
      if (s >= gcur_abs_)
      {
        ++gpu_finds_;
        const size_t r = hit(static_cast<size_t>(s - num_), gres_->len[gi_], gres_->cap[gi_]);
        ++gi_;
        gcur_abs_ = num_ + cur_;
        return r;
      }
    }
    // FIND, and SCAN / MATCH on whole buffers, come from the engine's FIND
    // records; SPLIT stays on the CPU matcher
    if (method == Const::SPLIT)
      return cpu(method, R_METHOD);
    if (opt_.A)
      return cpu(method, R_OPT_A);
    // (decided on the host: a device is initialised at the first input the
    // policy sends to the GPU, never for runs the CPU matcher serves)
    if (!eligible())
      return cpu(method, tab_anchor_ ? R_ANCHOR : R_TABLE);
    if (own_)
    {
      if (method != Const::FIND)
        return cpu(method, R_METHOD);
      if (sfit_ && !device_ready())
        return cpu(method, warm_reason());
      if (sparse_ && sfit_ && !device_slot())
        return cpu(method, R_SPARSE);
      return stream_match();
    }
    if (!eof_)
      return cpu(method, R_PARTIAL);
    if (end_ < min_bytes())
      return cpu(method, R_SMALL);
    if (!device_ready())
      return cpu(method, warm_reason());
    if (sparse_ && !device_slot())
      return cpu(method, R_SPARSE);
    reset_text();
    // buffer() is non-virtual and rewinds cur_ without telling this class
    // (absmatcher.h:542-591), and the caller may hand over new bytes at the
    // same address and size (ugrep re-buffers one std::string per line,
    // src/ugrep.cpp:733-740): any cursor behind the one this class last left
    // means the records may be stale, so scan again
    if (cpu_buf_ == buf_ && cpu_end_ == end_)
      return cpu(method, R_ENGINE);  // (the engine failed on this buffer)
    if (!src_.live() || gbuf_ != buf_ || gend_ != end_ || cur_ < gcur_ || inside_match())
      if (!rescan())
        return engine_failed(method);
    // (records that start before the cursor: the caller skipped past them)
    while (src_.have && src_.start < cur_)
      src_.pop();
    if (src_.err)
      return engine_failed(method);
    if (method != Const::FIND)
    {
      // SCAN and MATCH try the longest match at the cursor only
      // (lib/matcher.cpp:125-546 without adv_, nul = MATCH).  The cursor is a
      // position of the records' FIND chain (it is not inside a record), and
      // a FIND record starting there is the longest non-empty match there;
      // none means there is no non-empty match at the cursor
      const bool here = src_.have && src_.start == cur_ && src_.len > 0;
      if (!here && method == Const::MATCH)
        return cpu(method, R_METHOD);  // (the empty match MATCH accepts: the table's start state decides)
      ++gpu_finds_;
      if (!here)
      {
        // no match: the scan stops at the cursor (:673-679, :694-724)
        set_current(cur_);
        txt_ = buf_ + cur_;
        len_ = 0;
        gcur_ = cur_;
        return cap_ = 0;
      }
    }
    else
    {
      ++gpu_finds_;
    }
    if (!src_.have)
      return exhausted();
    const size_t start = static_cast<size_t>(src_.start), len = src_.len, cap = src_.cap;
    src_.pop();
    return hit(start, len, cap);
  }

 private:
  // why the CPU matcher answered a call (adapter statistics)
  enum Reason { R_METHOD, R_OPT_A, R_ANCHOR, R_TABLE, R_SPARSE, R_PARTIAL, R_SMALL, R_ENGINE, R_WARMUP, R_COLD, kReasons };
  static const char* reason_name(int r)
  {
    static const char* const n[kReasons] = {"method",  "option_A", "anchor_predictor", "table", "sparse_limit",
                                            "partial", "small",    "engine",           "warmup", "cold"};
    return n[r];
  }
  size_t cpu(Method method, int why)
  {
    ++cpu_why_[why];
    return Matcher::match(method);
  }
  // The engine's tables of (pattern, option W, option N), shared with clones:
  // the opcode words and flags, and the device tables uploaded at the first
  // GPU scan (failed: the upload failed, the inputs stay on the CPU matcher)
  struct Tables {
    std::vector<uint32_t> opc;
    uint32_t flags = 0;
    std::mutex mu;
    ugpu_dfa* d = NULL;
    bool failed = false;
    ~Tables() { e_dfa_destroy(d); }
  };
  // whether the engine takes the table (false: unsupported, or anchors left to
  // the reference's predictor, tab_anchor_), and whether it is prefiltered --
  // all on the host (ugpu_dfa_plan_host), no HIP call
  bool eligible()
  {
    if (!tab_pat_ || tab_pat_ != pat_ || tab_w_ != opt_.W || tab_n_ != opt_.N)
    {
      tab_.reset();
      tab_pat_ = pat_;
      tab_w_ = opt_.W;
      tab_n_ = opt_.N;
      tab_anchor_ = false;
      tab_ok_ = false;
      sparse_ = false;
      if (pat_ != NULL && ugpu_abi_version() != UGPU_ABI_VERSION)
      {
        // (a library built against another ugpu.h: its structs may differ)
        tab_err_ = "engine library ABI differs from this ugpu.h";
      }
      else if (pat_ != NULL)
      {
        const std::string rx = (*pat_)[0];
        uint32_t* opc = NULL;
        uint32_t nop = 0;
        if (ugpu_compile(rx.data(), rx.size(), UGPU_RX_REFLEX, &opc, &nop) == UGPU_OK)
        {
          const uint32_t flags = (opt_.W ? UGPU_PAT_WORD : 0u) | (opt_.N ? UGPU_PAT_EMPTY : 0u);
          ugpu_dfa_info info;
          const bool planned = ugpu_dfa_plan_host(opc, nop, flags, &info) == UGPU_OK;
          if (planned && !predictor_exact(rx, info))
          {
            tab_anchor_ = true;
          }
          else if (planned)
          {
            tab_ok_ = true;
            // (a prefiltered table: the reference's own needle search is fast on
            // it; option W without a selective prefilter also runs sparse_kernel,
            // prefilter_ppm 0, but is dense work for the CPU matcher)
            sparse_ = info.kernel == 0 && info.prefilter_ppm != 0;
            tab_ = std::make_shared<Tables>();
            tab_->opc.assign(opc, opc + nop);
            tab_->flags = flags;
          }
          ugpu_opc_free(opc);
        }
        if (tab_anchor_)
          tab_err_ = "meta edges where the reference's match predictor decides (line anchors without option N or "
                     "inside the regex, word boundaries after loops or before more bytes)";
        else if (!tab_ok_)
          tab_err_ = ugpu_last_error();
        const char* dump = std::getenv("UGPU_ADAPTER_DUMP");
        if (dump != NULL && *dump == '1')
          std::fprintf(stderr, "[ugpu-adapter] regex=%s tables=%s%s\n", rx.c_str(), tab_ok_ ? "gpu" : "unsupported: ",
                       tab_ok_ ? "" : tab_err_.c_str());
      }
    }
    return tab_ok_;
  }
  // Device warm-up, once per process.  A fresh process pays ~0.2-0.4 s at its
  // first GPU call (HIP context, queues, pinned memory, code object:
  // ugpu_warmup, tools/probe/startup_probe.cpp); the first input the policy
  // sends to the GPU starts it on a thread of its own, and workers that meet
  // the device warming wait for it (warm_state).  UGPU_ADAPTER_WARM=cpu: the
  // CPU matcher answers meanwhile (reason "warmup"; round 5's default) and
  // inputs move to the GPU at their cursor once the devices are ready, as
  // after a device queue slot frees up.  UGPU_ADAPTER_WARM=0: warm up on the
  // calling thread (the first GPU input waits, the others answer on the CPU;
  // tests that count GPU answers use it).  The thread is joined at exit.
  // Prefiltered tables do not start an asynchronous warm-up (reason "cold"):
  // on host buffers their GPU scans are PCIe-bound, ugrep's workers scan them
  // faster on their cores (tools/bench_ugrep.py: C2 at ~100 GB/s on 16
  // workers), and a run that ends before the warm-up would wait for it at
  // exit; they take the GPU once a dense table has warmed it.
  struct Warm {
    std::mutex mu;
    std::thread th;
    std::atomic<int> state{0};  // 0 not started, 1 warming, 2 ready, 3 failed
    ~Warm()
    {
      if (th.joinable())
        th.join();
    }
  };
  static Warm& warm()
  {
    static Warm w;
    return w;
  }
  // tab: the tables of the matcher that started the warm-up.  With
  // UGPU_ADAPTER_RESERVE, once the devices are up the tables are uploaded and
  // the pooled resources of one stream per live matcher (ugrep: one per
  // worker) are made on each device (ugpu_stream_reserve), so that the
  // workers' first feeds allocate nothing.  Meanwhile the CPU matchers answer
  // (reason "warmup").
  static void run_warm(Warm* w, std::shared_ptr<Tables> tab, size_t feed)
  {
    bool ok = GpuEngine::get().ok;  // (the device half loads here, on the warm-up thread)
    for (int d = 0; ok && d < devices(); ++d)
      ok = GpuEngine::get().warmup(d) == UGPU_OK;
    // UGPU_ADAPTER_RESERVE: 1 = reserve before the devices count as ready,
    // 2 = after (the workers' first feeds overlap it), unset/0 = no reserve.
    // Off by default: on ugrep -J16 over 16 files the serial reserve lengthens
    // the warm-up by about as much as it saves the workers (C3 3.26x with it,
    // 3.41x without, means of 4 and 2 runs; profiles/r05_ugrep_e2e.json).
    // A long-running process with many inputs per worker is where it pays.
    const char* re = std::getenv("UGPU_ADAPTER_RESERVE");
    const bool late = re != NULL && *re == '2';
    ugpu_dfa* t = NULL;
    if (ok && tab && re != NULL && (*re == '1' || *re == '2'))
    {
      std::lock_guard<std::mutex> lk(tab->mu);
      if (tab->d == NULL && !tab->failed)
      {
        (void)GpuEngine::get().select_device(0);
        if (GpuEngine::get().dfa_create(tab->opc.data(), static_cast<uint32_t>(tab->opc.size()), tab->flags,
                                        &tab->d) != UGPU_OK)
        {
          tab->d = NULL;
          tab->failed = true;
        }
      }
      t = tab->d;  // (tab keeps it alive)
    }
    if (late)
      w->state.store(ok ? 2 : 3, std::memory_order_release);
    const int per = (live().load() + devices() - 1) / devices();
    for (int d = 0; t != NULL && d < devices(); ++d)
      if (GpuEngine::get().select_device(d) == UGPU_OK)
        (void)GpuEngine::get().stream_reserve(t, per, feed);
    if (!late)
      w->state.store(ok ? 2 : 3, std::memory_order_release);
  }
  bool device_ready()
  {
    Warm& w = warm();
    int st = w.state.load(std::memory_order_acquire);
    if (st == 0 && !(sparse_ && warm_async_))
    {
      std::lock_guard<std::mutex> lk(w.mu);
      if (w.state.load(std::memory_order_acquire) == 0)
      {
        w.state.store(1, std::memory_order_release);
        bool async = warm_async_;
        if (async)
        {
          try
          {
            w.th = std::thread(run_warm, &w, tab_, 2 * chunk_);
          }
          catch (...)
          {
            async = false;
          }
        }
        if (!async)
          run_warm(&w, tab_, 2 * chunk_);
      }
      st = w.state.load(std::memory_order_acquire);
    }
    if (st == 1)
      st = warm_state();
    return st == 2;
  }
  // the warm-up state; under UGPU_ADAPTER_WARM=wait a warming device is
  // waited for (polled every 200 us: it is ready within ~0.3 s)
  int warm_state() const
  {
    int st = warm().state.load(std::memory_order_acquire);
    while (warm_wait_ && st == 1)
    {
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      st = warm().state.load(std::memory_order_acquire);
    }
    return st;
  }
  static int warm_reason()
  {
    const int st = warm().state.load(std::memory_order_acquire);
    return st == 3 ? R_ENGINE : st == 0 ? R_COLD : R_WARMUP;
  }
  // the device tables (uploaded on this matcher's device at the first call;
  // the engine copies them to other devices itself); NULL: not eligible, or
  // the upload failed
  const ugpu_dfa* tables()
  {
    if (!eligible())
      return NULL;
    std::lock_guard<std::mutex> lk(tab_->mu);
    if (tab_->d == NULL && !tab_->failed)
    {
      on_device();
      if (!GpuEngine::get().ok ||
          GpuEngine::get().dfa_create(tab_->opc.data(), static_cast<uint32_t>(tab_->opc.size()), tab_->flags,
                                      &tab_->d) != UGPU_OK)
      {
        tab_->d = NULL;
        tab_->failed = true;
        tab_err_ = ugpu_last_error();
      }
    }
    return tab_->d;
  }
  // Tables with meta edges (line anchors, word boundaries) whose FIND results
  // the reference's match predictor shares: ugrep runs FIND between candidate
  // positions its Pattern predicts (lib/matcher.cpp:52-86, :797-954), and for
  // meta edges the prediction can reject positions the DFA matches at -- the
  // engine implements the DFA (the reference with its predictor off).
  //  - line anchors: option N on and only a leading ^ / trailing $
  //    (tests/test_anchor.py: "a$|ab", "^\w+" without N differ);
  //  - word boundaries: a finite language whose boundary-dependent accepts
  //    end the walk (\bfoo\b, \<(foo|bar)\>, \b\w\w\b); loops before the
  //    assertion ("\w+\b" prints nothing in the reference CLI) and accepts
  //    that go on with bytes ("x\b|xy") stay on the CPU matcher
  //    (tests/test_wordb.py, a fuzz over tools/fuzz_wordb.py agrees).
  bool predictor_exact(const std::string& rx, const ugpu_dfa_info& info) const
  {
    if (info.contexts == 1)
      return true;
    if (has_line_anchor(rx) && !(opt_.N && anchors_outer(rx)))
      return false;
    if (info.contexts == 64 && !((info.shape & UGPU_SHAPE_FINITE) && !(info.shape & UGPU_SHAPE_WORD_COND)))
      return false;
    return true;
  }
  // a ^ or $ that is a line anchor (not in a bracket expression, escaped or
  // inside \Q...\E)
  static bool has_line_anchor(const std::string& rx)
  {
    size_t i = 0;
    const size_t n = rx.size();
    while (i < n)
    {
      const char c = rx[i];
      if (c == '\\')
      {
        if (i + 1 < n && rx[i + 1] == 'Q')
        {
          const size_t e = rx.find("\\E", i + 2);
          i = e == std::string::npos ? n : e + 2;
        }
        else
          i += 2;
        continue;
      }
      if (c == '[')
      {
        size_t j = i + 1;
        if (j < n && rx[j] == '^')
          ++j;
        if (j < n && rx[j] == ']')
          ++j;
        while (j < n && rx[j] != ']')
          j += rx[j] == '\\' ? 2 : 1;
        i = j + 1;
        continue;
      }
      if (c == '^' || c == '$')
        return true;
      ++i;
    }
    return false;
  }
  // the regex's line anchors are at most a leading ^ (after the (?m...) prefix
  // ugrep puts first, src/ugrep.cpp:8586-8604) and a trailing $: ^ and $ in
  // bracket expressions, escaped or inside \Q...\E are literals
  static bool anchors_outer(const std::string& rx)
  {
    size_t i = 0;
    const size_t n = rx.size();
    while (i + 1 < n && rx[i] == '(' && rx[i + 1] == '?')
    {
      size_t q = i + 2;
      while (q < n && std::strchr("imsx-", rx[q]) != NULL)
        ++q;
      if (q >= n || rx[q] != ')')
        break;
      i = q + 1;
    }
    const size_t first = i;
    while (i < n)
    {
      const char c = rx[i];
      if (c == '\\')
      {
        if (i + 1 < n && rx[i + 1] == 'Q')
        {
          const size_t e = rx.find("\\E", i + 2);
          i = e == std::string::npos ? n : e + 2;
        }
        else
          i += 2;
        continue;
      }
      if (c == '[')
      {
        size_t j = i + 1;
        if (j < n && rx[j] == '^')
          ++j;
        if (j < n && rx[j] == ']')
          ++j;
        while (j < n && rx[j] != ']')
          j += rx[j] == '\\' ? 2 : 1;
        i = j + 1;
        continue;
      }
      if ((c == '^' && i != first) || (c == '$' && i + 1 != n))
        return false;
      ++i;
    }
    return true;
  }
  // smallest input for the GPU: measured crossover against one reference
  // matcher on a host buffer (profiles/r02_adapter_latency.jsonl): 4 MiB for
  // C2-like sparse tables, 64 KiB for dense ones (profiles/r02b_adapter_latency.jsonl)
  size_t min_bytes() const
  {
    return min_bytes_ != ~static_cast<size_t>(0) ? min_bytes_ : (sparse_ ? (4u << 20) : (64u << 10));
  }
  // live GpuMatchers of the process (ugrep: one per worker thread)
  static std::atomic<int>& live()
  {
    static std::atomic<int> n(0);
    return n;
  }
  // The device queue for prefiltered tables.  Their GPU scans of host buffers
  // are bound by the PCIe link (~55 GB/s per device), which a few reference
  // AVX2 cores match, so each device runs at most sparse_max_ of them at once
  // and an input that finds no free slot is scanned by the CPU matcher: with
  // ugrep's 16 workers on one device, 2 workers feed the GPU and the others
  // scan on their cores, all at once.  A slot is held from the scan of an
  // input to its last record (or a reset / new input).  Dense tables gain
  // 100-200x per matcher and always take the GPU.
  struct DevQueue {
    std::mutex mu;
    int busy = 0;
  };
  static DevQueue& queue(int dev)
  {
    static DevQueue q[64];
    return q[dev & 63];
  }
  bool device_slot()
  {
    if (slot_)
      return true;
    // the decision holds for the rest of the input (a cursor that moves back
    // means new bytes: decide again)
    if (!own_ && slot_buf_ == buf_ && slot_end_ == end_ && cur_ >= slot_cur_)
    {
      slot_cur_ = cur_;
      return false;
    }
    slot_buf_ = buf_;
    slot_end_ = end_;
    slot_cur_ = cur_;
    DevQueue& q = queue(dev());
    std::lock_guard<std::mutex> lk(q.mu);
    if (q.busy >= sparse_max_)
      return false;
    ++q.busy;
    slot_ = true;
    return true;
  }
  void release_slot()
  {
    if (!slot_)
      return;
    DevQueue& q = queue(dev());
    std::lock_guard<std::mutex> lk(q.mu);
    --q.busy;
    slot_ = false;
    slot_buf_ = NULL;
  }
  // visible devices (at least 1), and the next matcher's device
  static int devices()
  {
    static const int n = [] {
      int k = 0;
      return GpuEngine::get().ok && GpuEngine::get().device_count(&k) == UGPU_OK && k > 0 ? k : 1;
    }();
    return n;
  }
  static int next_device()
  {
    static std::atomic<int> k(0);
    return k++ % devices();
  }
  // this matcher's device, assigned round-robin at its first GPU input (the
  // first HIP call of the process is there)
  int dev()
  {
    if (dev_ < 0)
      dev_ = next_device();
    return dev_;
  }
  // this matcher's device current on the calling thread (ugrep calls a matcher
  // from the worker thread that owns it, but clones are made elsewhere)
  void on_device()
  {
    if (GpuEngine::get().ok)
      (void)GpuEngine::get().select_device(dev());
  }
  void drop_records()
  {
    e_result_free(gres_);
    gres_ = NULL;
    gi_ = 0;
    src_.clear();
  }
  size_t hit(size_t start, size_t len, size_t cap)
  {
    txt_ = buf_ + start;
    len_ = len;
    cap_ = cap;
    // an empty match (option N) leaves the cursor one past it, as
    // lib/matcher.cpp:715-719 does ("advance one char ... when we return")
    set_current(start + len + (len == 0 && start < end_ ? 1 : 0));
    gcur_ = cur_;
    return cap_;
  }
  size_t exhausted()
  {
    release_slot();  // (the input's records are all popped)
    set_current(end_);
    txt_ = buf_ + end_;
    len_ = 0;
    gcur_ = cur_;
    return cap_ = 0;
  }
  void init_policy()
  {
    const char* e = std::getenv("UGPU_ADAPTER_MIN_BYTES");
    min_bytes_ = e && *e ? static_cast<size_t>(std::strtoull(e, NULL, 0)) : ~static_cast<size_t>(0);  // ~0: per table
    e = std::getenv("UGPU_ADAPTER_SPARSE_MAX");
    sparse_max_ = e && *e ? std::atoi(e) : 2;  // device queue slots for prefiltered tables
    e = std::getenv("UGPU_ADAPTER_MULTI_MIN");
    multi_min_ = e && *e ? static_cast<size_t>(std::strtoull(e, NULL, 0)) : (64u << 20);
    e = std::getenv("UGPU_ADAPTER_WARM");
    warm_async_ = !(e && *e == '0');
    // By default (since round 6) a worker that meets the device warming waits
    // for it instead of letting the CPU matcher answer (reason "warmup"):
    // ugrep -co -J16 over 16 x 256 MiB, C3 0.602 against 0.663 s and C4 0.723
    // against 0.873 s, with no FIND call answered by the CPU
    // (profiles/r06_ugrep_e2e_wait.jsonl).  UGPU_ADAPTER_WARM=cpu restores the
    // CPU answers, =0 warms up on the first GPU input's thread (the others
    // answer on the CPU meanwhile).
    warm_wait_ = !(e && (*e == '0' || std::strcmp(e, "cpu") == 0));
    e = std::getenv("UGPU_ADAPTER_CHUNK");
    // (2 MiB: a feed's bytes and records stay in the worker's caches between
    // the read, the H2D staging and the pops -- ugrep C3 3.2-3.5x against
    // 2.4-2.6x with 8 MiB feeds, profiles/r05_ugrep_e2e.json)
    chunk_ = e && *e ? static_cast<size_t>(std::strtoull(e, NULL, 0)) : (2u << 20);
    if (chunk_ == 0)
      chunk_ = 1;
  }
  // cur_ (at or after the cursor this class left) lies strictly inside a
  // pending record; the records before it are dropped on the way, the caller
  // skipped past them
  bool inside_match()
  {
    while (src_.have && src_.start < cur_ && src_.start + src_.len <= cur_)
      src_.pop();
    return src_.have && src_.start < cur_;
  }
  // the engine failed on this buffer (also midway through its records: the
  // CPU matcher goes on from the cursor, where the FIND chains agree)
  size_t engine_failed(Method method)
  {
    drop_records();
    cpu_buf_ = buf_;
    cpu_end_ = end_;
    return cpu(method, R_ENGINE);
  }
  bool rescan()
  {
    drop_records();
    on_device();
    const ugpu_dfa* t = tables();
    if (t == NULL)
      return false;
    const uint8_t* b = reinterpret_cast<const uint8_t*>(buf_);
    int rc;
    if (devices() > 1 && end_ - cur_ >= multi_min_) {
      rc = GpuEngine::get().find_all_multi(t, b, end_, cur_, UGPU_MODE_OFFSETS, 0, &gres_);
      if (rc == UGPU_OK)
        src_.set(gres_);
    } else {
      // the pipelined host path: records popped from pinned memory as find()
      // asks for them (ugpu_find_records)
      ugpu_records* r = NULL;
      rc = GpuEngine::get().find_records(t, b, end_, cur_, &r);
      if (rc == UGPU_OK)
        src_.set(r);
    }
    if (rc != UGPU_OK)
      return false;  // (this input stays on the CPU matcher)
    ++scans_;
    gbuf_ = buf_;
    gend_ = end_;
    gcur_ = cur_;
    return true;
  }

  // ---- streamed input
  // Records of the current feed are absolute (sbase_ + record start); the
  // stream was started at absolute offset sbase_ and has been fed up to sfed_.
  size_t stream_match()
  {
    if (cpu_stream_)
      return cpu(Const::FIND, cpu_stream_why_);
    reset_text();
    txt_ = buf_ + cur_;  // bytes before the cursor may be shifted out (as lib/matcher.cpp:51)
    const uint64_t at = static_cast<uint64_t>(num_ + cur_);
    if (!sopen_ || at < gcur_abs_ || at > sfed_ || stream_inside(at))
      stream_restart(at);
    ++gpu_finds_;
    for (;;)
    {
      while (gres_ != NULL && gi_ < gres_->count && sbase_ + gres_->start[gi_] < at)
        ++gi_;
      if (gres_ != NULL && gi_ < gres_->count)
      {
        const size_t start = static_cast<size_t>(sbase_ + gres_->start[gi_] - num_);
        const size_t len = gres_->len[gi_], cap = gres_->cap[gi_];
        ++gi_;
        const size_t r = hit(start, len, cap);
        gcur_abs_ = num_ + cur_;
        return r;
      }
      if (sdone_)
      {
        const size_t r = exhausted();
        gcur_abs_ = num_ + cur_;
        return r;
      }
      // read until chunk_ unfed bytes are buffered or the input ends, then
      // feed.  A short read with nothing more ready (a slow pipe or a TTY that
      // ugrep set non-blocking, src/ugrep.cpp:3956-3966; Input::get returns what
      // has arrived, include/reflex/input.h:716-731) feeds at once: the next
      // get() would block, and the reference matcher reports the matches in the
      // bytes it already has before it blocks.
      if (gst_ == NULL && !stream_may_feed())
      {
        // no device for this stream yet (cold, warming, failed, or the device
        // queue is full): the CPU matcher answers from the cursor on its own
        // reads -- reading chunk_ bytes ahead here first would cost the CPU
        // path ~20 % (larger buffer shifts; tools/bench_ugrep.py C2)
        --gpu_finds_;
        return cpu(Const::FIND, gst_why_);
      }
      bool flush = false;
      const auto t_read = std::chrono::steady_clock::now();
      while (!eof_ && num_ + end_ - sfed_ < chunk_)
      {
        if (end_ + blk_ + 1 >= max_)
          (void)grow(chunk_ > Const::BLOCK ? chunk_ : Const::BLOCK);
        const size_t want = blk_ > 0 ? blk_ : max_ - end_ - 1;
        const size_t n = get(buf_ + end_, want);
        if (n == 0)
        {
          eof_ = !wrap();
        }
        else
        {
          end_ += n;
          if (n < want && !input_ready())
          {
            flush = true;
            break;
          }
        }
      }
      t_read_ += std::chrono::steady_clock::now() - t_read;
      if (eof_ && scans_at_restart_ == scans_ && num_ + end_ - sbase_ < min_bytes())
      {
        // a small input, all of it read before any feed: the CPU matcher is faster
        cpu_stream_ = true;
        cpu_stream_why_ = R_SMALL;
        if (gst_ != NULL)
          on_device();
        e_stream_destroy(gst_);
        gst_ = NULL;
        --gpu_finds_;
        return cpu(Const::FIND, R_SMALL);
      }
      if (gst_ == NULL)
      {
        // the first feed of this stream: a prefiltered table takes a device
        // queue slot first (none free: the CPU matcher goes on from the
        // cursor, and the stream restarts there once a slot frees up), then
        // the device tables and the stream
        sfit_ = true;
        if (!device_ready())
        {
          --gpu_finds_;
          return cpu(Const::FIND, warm_reason());
        }
        if (sparse_ && !device_slot())
        {
          --gpu_finds_;
          return cpu(Const::FIND, R_SPARSE);
        }
        on_device();
        const ugpu_dfa* t = tables();
        if (t == NULL || GpuEngine::get().stream_create(t, 0, &gst_) != UGPU_OK)
        {
          gst_ = NULL;
          cpu_stream_ = true;
          cpu_stream_why_ = R_ENGINE;
          --gpu_finds_;
          return cpu(Const::FIND, R_ENGINE);
        }
      }
      const size_t from = static_cast<size_t>(sfed_ - num_);
      drop_records();
      on_device();
      const auto t_feed = std::chrono::steady_clock::now();
      const int frc = GpuEngine::get().stream_feed(gst_, reinterpret_cast<const uint8_t*>(buf_ + from), end_ - from,
                                                   eof_ ? 1 : flush ? UGPU_FEED_FLUSH : 0, UGPU_MODE_OFFSETS, &gres_);
      t_feed_ += std::chrono::steady_clock::now() - t_feed;
      if (frc != UGPU_OK)
      {
        // engine unavailable for this input: the CPU matcher takes over at the cursor
        cpu_stream_ = true;
        cpu_stream_why_ = R_ENGINE;
        e_stream_destroy(gst_);
        gst_ = NULL;
        --gpu_finds_;
        return cpu(Const::FIND, R_ENGINE);
      }
      ++scans_;
      sfed_ = num_ + end_;
      sdone_ = eof_;
    }
  }
  // whether a first feed could go to a device now, decided without reading
  // ahead and without side effects (gst_why_: the reason when not).  A device
  // still cold for a dense table is not decided here: the read-ahead's
  // small-input test comes first, so a small input never starts the warm-up.
  bool stream_may_feed()
  {
    const int st = warm_state();
    if (st == 1 || st == 3 || (st == 0 && sparse_ && warm_async_))
    {
      gst_why_ = warm_reason();
      return false;
    }
    if (st == 2 && sparse_ && !slot_)
    {
      DevQueue& q = queue(dev());
      std::lock_guard<std::mutex> lk(q.mu);
      if (q.busy >= sparse_max_)
      {
        gst_why_ = R_SPARSE;
        return false;
      }
    }
    return true;
  }
  // more input can be read without blocking (memory and std::istream sources
  // never block; for a FILE*, poll its descriptor)
  bool input_ready()
  {
    FILE* f = in.file();
    if (f == NULL)
      return true;
    struct pollfd p;
    p.fd = fileno(f);
    p.events = POLLIN;
    p.revents = 0;
    return ::poll(&p, 1, 0) > 0;  // data, EOF or an error: get() returns at once
  }
  bool stream_inside(uint64_t at)
  {
    // the cursor moved strictly inside a pending match
    if (gres_ == NULL)
      return false;
    for (size_t i = gi_ > 0 ? gi_ - 1 : 0; i < gres_->count; ++i)
    {
      const uint64_t s = sbase_ + gres_->start[i];
      if (s >= at)
        return false;
      if (s + gres_->len[i] > at)
        return true;
    }
    return false;
  }
  // a new stream from absolute offset at (created at its first feed)
  void stream_restart(uint64_t at)
  {
    drop_records();
    if (gst_ != NULL)
      on_device();
    e_stream_destroy(gst_);
    gst_ = NULL;
    sopen_ = true;
    sbase_ = at;
    sfed_ = at;
    sdone_ = false;
    gcur_abs_ = at;
    scans_at_restart_ = scans_;
  }

  // the records of a whole-buffer scan, popped in chain order: a
  // ugpu_find_records cursor, or a ugpu_result (multi-device scans)
  struct Source {
    ugpu_records* rec = NULL;
    const ugpu_result* res = NULL;
    size_t i = 0;
    bool have = false, err = false;
    uint64_t start = 0;
    uint32_t len = 0, cap = 0;
    bool live() const { return rec != NULL || res != NULL; }
    void clear()
    {
      e_records_free(rec);
      rec = NULL;
      res = NULL;  // (owned by gres_)
      have = err = false;
    }
    void set(ugpu_records* r)
    {
      clear();
      rec = r;
      pop();
    }
    void set(const ugpu_result* r)
    {
      clear();
      res = r;
      i = 0;
      pop();
    }
    void pop()
    {
      if (rec != NULL)
      {
        const int rc = GpuEngine::get().records_next(rec, &start, &len, &cap);
        have = rc == 1;
        err = rc < 0;
      }
      else if (res != NULL && i < res->count)
      {
        start = res->start[i];
        len = res->len[i];
        cap = res->cap[i];
        ++i;
        have = true;
      }
      else
        have = false;
    }
  };
  Source src_;
  std::shared_ptr<Tables> tab_;
  const Pattern* tab_pat_ = NULL;
  bool tab_w_ = false, tab_n_ = false;
  bool tab_anchor_ = false;  // anchored table left to the CPU matcher (see anchors_outer)
  bool tab_ok_ = false;      // the engine takes the table (eligible())
  bool sparse_ = false;  // the table has a selective prefilter (sparse_kernel)
  ugpu_result* gres_ = NULL;
  const char* gbuf_ = NULL;
  const char* cpu_buf_ = NULL;  // a buffer the engine failed on (with cpu_end_)
  size_t cpu_end_ = 0;
  // gcur_: the cursor this class left behind (after the scan or the last hit)
  size_t gend_ = 0, gcur_ = 0, gi_ = 0, scans_ = 0, scans_at_restart_ = 0;
  size_t min_bytes_ = 0, chunk_ = 0, multi_min_ = 0;
  int dev_ = -1;  // this matcher's device (dev(): assigned at the first GPU input)
  int sparse_max_ = 4;
  bool warm_async_ = true;  // device warm-up on its own thread (UGPU_ADAPTER_WARM)
  bool warm_wait_ = true;   // workers wait for a warming device (UGPU_ADAPTER_WARM)
  ugpu_stream* gst_ = NULL;
  uint64_t sbase_ = 0, sfed_ = 0, gcur_abs_ = 0;
  bool sdone_ = false, cpu_stream_ = false;
  int gst_why_ = R_COLD;  // (stream_may_feed)
  // time in the stream's reads and feeds (UGPU_ADAPTER_STATS)
  std::chrono::steady_clock::duration t_read_{}, t_feed_{};
  bool sopen_ = false;  // a stream was started for this input (its ugpu_stream at the first feed)
  bool sfit_ = false;   // this input passed the small-input test (device queue decisions from here)
  int cpu_stream_why_ = R_ENGINE;
  bool slot_ = false;  // this matcher holds a device queue slot (prefiltered tables)
  const char* slot_buf_ = NULL;  // the input the last slot decision was for
  size_t slot_end_ = 0, slot_cur_ = 0;
  std::string tab_err_;  // why the engine rejected the table (ugpu_last_error)
  size_t gpu_finds_ = 0;
  size_t cpu_why_[kReasons] = {};
};

}  // namespace reflex

#endif
