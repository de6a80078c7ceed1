// plan.hpp -- the host half of the engine (libugpu_host.so), shared with the
// device half (engine.hip in libugrep_amd.so).
//
// The host half holds everything a caller needs to decide, without a device,
// whether and how a pattern runs on the GPU: the table builder (tables.cpp),
// the regex compiler (regex_compile.cpp), the plan below, the host-only C ABI
// (ugpu_compile, ugpu_dfa_plan_host, ugpu_tables_*_host) and the error string
// of both halves (ugpu_last_error).  It does not link the HIP runtime, so the
// drop-in matcher links only it and loads the device half at the first input
// its policy sends to a GPU (integration/reflex_gpu_matcher.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "tables.hpp"

// Unicode Word ranges as flat [lo, hi] pairs (regex_compile.cpp, the table of \w)
void ugpu_word_ranges(std::vector<uint32_t>& out);

namespace ugpu {

// What ugpu_dfa_create uploads for a table under pattern flags, and so which
// kernels its scans run: decided on the host alone (ugpu_dfa_plan_host answers
// it without touching a device)
constexpr int kLbNeedles = 16;

struct DfaPlan {
  bool ok = true;  // false: option W with line anchors or empty matches (UGPU_UNSUPPORTED)
  bool nul = false, amode = false;
  bool wtab = false, wplus = false, xcw = false;
  bool xtrans = false, xid = false, xu = false, xg = false;
  // loop-needle table (C+ N for a finite set N of strings over C,
  // host_api.cpp loop_needle): the sparse kernel's prefilter looks for the
  // strings of N and its candidates walk back to their C-run's start
  bool lb = false;
  // option W on a byte table without a selective prefilter: the sparse
  // kernel's W walks from the first-byte candidates that follow no ASCII
  // letter (ScanParams::wstart) instead of wfind_kernel (UGPU_WSPARSE)
  bool wsparse = false;
  uint32_t lb_cls[8] = {};
  std::vector<std::string> lb_needles;  // (N, at most kLbNeedles strings of 2-32 bytes)
  uint8_t lb_ft[20] = {};               // the prefilter over N (tables.cpp needle_filter)
  double lb_density = 0;                // its estimated candidate fraction
};

// lb: loop-needle lookback 1 / 0, or -1 for the UGPU_LB default (on)
DfaPlan dfa_plan(const DfaTables& t, uint32_t flags, int lb = -1);
// ugpu_dfa_info from the tables and the plan (ugpu_dfa_plan_host, ugpu_dfa_info_get)
void dfa_info_fill(const DfaTables& t, const DfaPlan& p, void* info /* ugpu_dfa_info* */);
// \w+ as ugpu_compile builds it
bool is_word_plus(const DfaTables& t);
// sets the calling thread's error string (ugpu_last_error) and returns code
int host_fail(int code, const std::string& msg);

}  // namespace ugpu
