// host_api.cpp -- the host half of the C ABI (libugpu_host.so, no HIP runtime):
// table planning, the host-only table entry points and the error string.  See
// plan.hpp.  The device half (engine.hip) calls dfa_plan / dfa_info_fill and
// reports its errors through host_fail, so ugpu_last_error answers for both.
#include <array>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../../include/ugpu.h"
#include "plan.hpp"
#include "tables.hpp"

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg)
{
  g_err = msg;
  return code;
}
}  // namespace

namespace ugpu {

int host_fail(int code, const std::string& msg) { return fail(code, msg); }

// \w+ as ugpu_compile builds it (language-equivalent to the reference's table,
// tests/test_compile.py), compiled once
bool is_word_plus(const DfaTables& t)
{
  static DfaTables wp;
  static bool ok = [] {
    uint32_t* opc = nullptr;
    uint32_t nop = 0;
    if (ugpu_compile("\\w+", 3, 0, &opc, &nop) != UGPU_OK) return false;
    std::string err;
    const bool built = build_tables(opc, nop, wp, err) == 0;
    ugpu_opc_free(opc);
    return built;
  }();
  return ok && tables_equivalent(t, wp);
}

// Loop-needle tables: the language is C+ N for a byte set C and a finite set
// N of strings of >= 2 bytes of C (e.g. [a-z]+ing, [a-z]+(ing|ed)).  Then
// every FIND match is a whole C-run prefix: it starts at a C-run's first byte
// (or at the scan start, inside a run) and ends at the end of the run's last
// string of N -- after which no position of the run starts a match -- so the
// chain enters every run at its start, and a run holds a match iff a string of
// N occurs in it after its first byte.  The sparse kernel's prefilter then
// looks for the strings of N (3 bytes deep) instead of the first bytes (here,
// common ones), and each candidate walks back over C to its run's start (the
// reference's lookback, lib/matcher.cpp:636-656 lbk_ / cbk_, restated for the
// FIND chain).  Recognised on the DFA:
//  - C = the start state's live bytes; s1 = the state after one byte c0 of C.
//    If the language is C+ N, s1's language is M = C* N, and the shortest
//    basis of N is the set of w in M with not (w[0] in C and w[1:] in M).
//  - Those w are the paths of the product (state after w, state after w[1:])
//    from (s1, none) to the nodes that accept in the first component only;
//    the part of the product that reaches such a node must be acyclic (N
//    finite) with at most kLbNeedles paths.
//  - Then the table must equal the Aho-Corasick automaton of C+ N on every
//    byte from the start (a product walk): dead exactly where the automaton
//    leaves C, accepting exactly where a string of N has just ended.
bool loop_needle(const DfaTables& t, uint32_t cls[8], std::vector<std::string>& needles)
{
  needles.clear();
  if (t.format != FMT_BYTE || t.anchored || t.redo || t.cap1 == 0 || t.start >= t.accb || t.row != 256) return false;
  const uint32_t R = t.row, S = t.states;
  if (S > 128) return false;
  for (int i = 0; i < 8; ++i) cls[i] = 0;
  uint32_t c0 = 256;
  for (uint32_t b = 0; b < 256; ++b)
    if (t.trans[t.start + b]) {
      cls[b >> 5] |= 1u << (b & 31);
      if (c0 == 256) c0 = b;
    }
  if (c0 == 256) return false;
  auto inC = [&](uint32_t b) { return (cls[b >> 5] >> (b & 31)) & 1u; };
  const uint32_t e1 = t.trans[t.start + c0];
  if (e1 >= t.accb) return false;  // (a one-byte match)
  const uint32_t s1 = e1 / R;
  // product nodes a * (S + 1) + b, b == S: none (w empty)
  const uint32_t NB = S + 1;
  auto node = [&](uint32_t a, uint32_t bb) { return a * NB + bb; };
  std::vector<int32_t> idx((size_t)S * NB, -1);
  std::vector<uint32_t> nodes{node(s1, S)};
  std::vector<uint8_t> end{0};
  idx[nodes[0]] = 0;
  // (successor of node i on byte x of C)
  auto succ = [&](uint32_t i, uint32_t x) {
    const uint32_t a = nodes[i] / NB, bb = nodes[i] % NB;
    const uint32_t ea = t.trans[(size_t)a * R + x];
    const uint32_t eb = bb == S ? e1 : t.trans[(size_t)bb * R + x];
    return std::make_pair(ea, eb);
  };
  std::vector<std::vector<uint32_t>> in(1);  // predecessors
  for (size_t i = 0; i < nodes.size(); ++i) {
    for (uint32_t x = 0; x < 256; ++x) {
      if (!inC(x)) continue;
      const auto [ea, eb] = succ((uint32_t)i, x);
      if (!ea || !eb) return false;  // (C* N stays alive on C)
      const uint32_t n2 = node(ea / R, eb / R);
      if (idx[n2] < 0) {
        idx[n2] = (int32_t)nodes.size();
        nodes.push_back(n2);
        end.push_back(ea >= t.accb && eb < t.accb);
        in.emplace_back();
      }
      in[idx[n2]].push_back((uint32_t)i);
    }
  }
  // the nodes that reach an end node (or are one)
  const size_t V = nodes.size();
  std::vector<uint8_t> co(V, 0);
  std::vector<uint32_t> st;
  for (size_t i = 0; i < V; ++i)
    if (end[i]) co[i] = 1, st.push_back((uint32_t)i);
  while (!st.empty()) {
    const uint32_t j = st.back();
    st.pop_back();
    for (uint32_t i : in[j])
      if (!co[i]) co[i] = 1, st.push_back(i);
  }
  if (!co[0]) return false;
  // the words: paths from the root through co-reachable nodes to end nodes;
  // a cycle among those nodes means N is infinite (DFS with a path stack)
  std::vector<uint8_t> onpath(V, 0);
  std::string w;
  bool bad = false;
  std::function<void(uint32_t)> walk = [&](uint32_t i) {
    if (bad) return;
    if (end[i] && i != 0) {
      if (needles.size() >= (size_t)kLbNeedles || w.size() < 2 || w.size() > 32) {
        bad = true;
        return;
      }
      needles.push_back(w);
    }
    onpath[i] = 1;
    for (uint32_t x = 0; x < 256; ++x) {
      if (!inC(x)) continue;
      const auto [ea, eb] = succ(i, x);
      const uint32_t j = (uint32_t)idx[node(ea / R, eb / R)];
      if (!co[j]) continue;
      if (onpath[j] || w.size() >= 32) {
        bad = true;
        return;
      }
      w.push_back((char)x);
      walk(j);
      w.pop_back();
      if (bad) return;
    }
    onpath[i] = 0;
  };
  walk(0);
  if (bad || needles.empty()) {
    needles.clear();
    return false;
  }
  // Aho-Corasick automaton of N: trie nodes, full goto over bytes, outputs
  std::vector<std::array<int32_t, 256>> go(1);
  go[0].fill(-1);
  std::vector<uint8_t> outp(1, 0);
  for (const std::string& n : needles) {
    int32_t k = 0;
    for (unsigned char x : n) {
      if (go[k][x] < 0) {
        go[k][x] = (int32_t)go.size();
        go.emplace_back();
        go.back().fill(-1);
        outp.push_back(0);
      }
      k = go[k][x];
    }
    outp[k] = 1;
  }
  const uint32_t T = (uint32_t)go.size();
  std::vector<int32_t> fl(T, 0);
  std::vector<uint32_t> q;
  for (uint32_t x = 0; x < 256; ++x) {
    if (go[0][x] < 0) {
      go[0][x] = 0;
    } else {
      fl[go[0][x]] = 0;
      q.push_back((uint32_t)go[0][x]);
    }
  }
  for (size_t qi = 0; qi < q.size(); ++qi) {
    const uint32_t k = q[qi];
    outp[k] |= outp[fl[k]];
    for (uint32_t x = 0; x < 256; ++x) {
      if (go[k][x] < 0) {
        go[k][x] = go[fl[k]][x];
      } else {
        fl[go[k][x]] = go[fl[k]][x];
        q.push_back((uint32_t)go[k][x]);
      }
    }
  }
  // product walk: (table entry, automaton node), node T = before the first byte
  // (which C+ consumes: no string of N starts there)
  std::vector<uint8_t> seen((size_t)S * (T + 1), 0);
  std::vector<std::pair<uint32_t, uint32_t>> ps{{t.start, T}};
  seen[(size_t)(t.start / R) * (T + 1) + T] = 1;
  while (!ps.empty()) {
    const auto [e, k] = ps.back();
    ps.pop_back();
    for (uint32_t b = 0; b < 256; ++b) {
      const uint32_t e2 = t.trans[e + b];
      const bool alive = inC(b) != 0;
      if (!e2 != !alive) {  // one side dead, the other not
        needles.clear();
        return false;
      }
      if (!e2) continue;
      const uint32_t k2 = k == T ? 0u : (uint32_t)go[k][b];
      if ((e2 >= t.accb) != (outp[k2] != 0)) {
        needles.clear();
        return false;
      }
      uint8_t& v = seen[(size_t)(e2 / R) * (T + 1) + k2];
      if (!v) {
        v = 1;
        ps.push_back({e2, k2});
      }
    }
  }
  return true;
}

DfaPlan dfa_plan(const DfaTables& t, uint32_t flags, int lb)
{
  DfaPlan p;
  p.nul = (flags & UGPU_PAT_EMPTY) != 0;
  p.amode = t.anchored || (p.nul && t.start_acc);
  if (t.lookahead) {
    // lookahead tables: the lookahead walk on wfind_kernel (tables.hpp look),
    // with option W since round 6 (at_wb at the walk start, at_we on TAKE
    // only: lib/matcher.cpp:107, :142, :208); option N with empty matches is
    // not modelled with lookahead (the CPU matcher keeps those)
    p.ok = !p.amode;
    p.wtab = (flags & UGPU_PAT_WORD) != 0;
    return p;
  }
  if (t.redo && p.amode) {
    // (negative patterns with empty matches under option N: the reference
    // reports an empty REDO match; not modelled -- the CPU matcher keeps
    // those.  Under option W a REDO accept skips at_we: walk<FMT, kWalkWord>)
    p.ok = false;
    return p;
  }
  if (p.amode) {
    p.ok = !(flags & UGPU_PAT_WORD);
    return p;
  }
  // loop-needle tables run the sparse kernel, with or without a first-byte
  // prefilter; under option W the run bytes must be word bytes (then no match
  // starts inside a run: at_wb fails there)
  const char* lenv = std::getenv("UGPU_LB");
  if (lb < 0) lb = !(lenv && lenv[0] == '0');
  if (lb && t.format == FMT_BYTE && loop_needle(t, p.lb_cls, p.lb_needles)) {
    p.lb = true;
    p.lb_density = needle_filter(p.lb_needles, p.lb_ft);
    if (flags & UGPU_PAT_WORD)
      for (uint32_t b = 0; b < 256 && p.lb; ++b)
        if ((p.lb_cls[b >> 5] >> (b & 31)) & 1u)
          p.lb = (b >= '0' && b <= '9') || (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == '_';
  }
  if (flags & UGPU_PAT_WORD) {
    p.wtab = true;
    const bool wf = !(std::getenv("UGPU_WFAST") && std::getenv("UGPU_WFAST")[0] == '0');
    p.wplus = wf && t.gap && !t.filter && !p.lb && t.cap1 != 0 && is_word_plus(t);
    p.xcw = wf && t.xc && (t.xc_w || t.xc_wsub) && !t.filter && !p.lb && t.cap1 != 0;
    // option W without a selective prefilter: the sparse kernel when every
    // first byte is an ASCII word byte (then the word-start filter leaves about
    // the word starts: C2 -w '[A-Za-z]+' 229.7 -> 89.0 ms against
    // wfind_kernel; profiles/r05_wsparse_ab.json).  UGPU_WSPARSE=0: wfind_kernel.
    const char* wsenv = std::getenv("UGPU_WSPARSE");
    p.wsparse = !(wsenv && wsenv[0] == '0') && !t.filter && !p.lb && !p.wplus && !p.xcw && t.format == FMT_BYTE &&
                t.row == 256 && t.first_bytes > 0 && !t.start_acc;
    for (uint32_t b = 0; b < 256 && p.wsparse; ++b)
      if (t.trans[t.start + b])
        p.wsparse = (b >= '0' && b <= '9') || (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == '_';
    if (!p.wplus && !p.xcw) return p;  // option W runs wfind_kernel only: no transducer tables
  }
  const bool tx = !t.filter && !p.lb && t.cap1 != 0;
  p.xtrans = t.restart_local && tx;
  p.xid = t.immediate && tx;
  p.xu = t.xu && tx;
  p.xg = t.gap && tx;
  return p;
}

void dfa_info_fill(const DfaTables& t, const DfaPlan& p, void* out)
{
  ugpu_dfa_info* info = static_cast<ugpu_dfa_info*>(out);
  info->states = t.states;
  info->classes = t.classes;
  info->row = t.row;
  info->format = t.format;
  info->table_bytes = (uint32_t)(t.trans.size() * 2 + t.trans32.size() * 4 + (t.format != FMT_BYTE ? 256 : 0));
  // (loop-needle tables: the estimate of the prefilter over their strings)
  info->prefilter_ppm = p.lb ? (uint32_t)(p.lb_density * 1e6) + 1 : t.filter ? (uint32_t)(t.fdensity * 1e6) + 1 : 0u;
  info->first_bytes = t.first_bytes;
  info->accepting = t.accepting;
  info->contexts = t.ctx_word ? 64u : t.anchored ? 4u : 1u;
  info->shape = (t.finite ? UGPU_SHAPE_FINITE : 0u) | (t.word_cond_edges ? UGPU_SHAPE_WORD_COND : 0u) |
                (t.cap1 != 0 && !t.anchored ? UGPU_SHAPE_ONE_ACCEPT : 0u) | (p.lb ? UGPU_SHAPE_LOOP_NEEDLE : 0u) |
                (t.lookahead ? UGPU_SHAPE_LOOKAHEAD : 0u);
  const char* xenv = std::getenv("UGPU_XI");
  const char* genv = std::getenv("UGPU_XG");
  const char* cenv = std::getenv("UGPU_XC");
  const char* uenv = std::getenv("UGPU_XU");
  const char* senv = std::getenv("UGPU_SPARSE");
  const bool byte_filter = (t.filter || p.lb || p.wsparse) && t.format == FMT_BYTE && !(senv && senv[0] == '0');
  // (dfa_xc and dfa_xu, from the plan instead of the uploaded tables)
  const bool xc = t.xc && !t.filter && !p.lb && t.cap1 != 0 && (!p.wtab || p.xcw) && !(cenv && cenv[0] == '0');
  const bool xu = p.xu && (!p.wtab || p.wplus) && !(uenv && uenv[0] == '0');
  // (context accepts on a prefiltered table: sparse_kernel's context walks)
  info->kernel = (p.amode && !byte_filter) || t.format == FMT_WIDE || t.lookahead ||
                         (p.wtab && !p.wplus && !p.xcw && !byte_filter)
                     ? 4u
                 : byte_filter                                                                  ? 0u
                 : xc                                                                           ? 5u
                 : xu                                                                           ? 6u
                 : (p.xid && !(xenv && xenv[0] == '0'))                                          ? 2u
                 : (p.xg && !(genv && genv[0] == '0'))                                           ? 3u
                                                                                                  : 1u;
}

}  // namespace ugpu

using namespace ugpu;

extern "C" {

const char* ugpu_last_error(void) { return g_err.c_str(); }

const char* ugpu_version(void) { return "ugrep_amd 0.1 (gfx950)"; }
int ugpu_abi_version(void) { return UGPU_ABI_VERSION; }

int ugpu_dfa_plan_host(const uint32_t* opc, uint32_t nop, uint32_t pattern_flags, ugpu_dfa_info* info)
{
  if (!info) return fail(UGPU_INVAL, "info is NULL");
  if (pattern_flags & ~(UGPU_PAT_WORD | UGPU_PAT_EMPTY)) return fail(UGPU_INVAL, "unknown pattern flags");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  const DfaPlan pl = dfa_plan(t, pattern_flags);
  if (!pl.ok) return fail(UGPU_UNSUPPORTED, "option W with line anchors, empty matches, negative patterns or lookahead");
  dfa_info_fill(t, pl, info);
  return UGPU_OK;
}

int ugpu_tables_build_host(const uint32_t* opc, uint32_t nop, ugpu_dfa_info* info, uint16_t* trans,
                           uint32_t trans_cap, uint8_t* cls, uint32_t* caps, uint32_t caps_cap, uint32_t* start,
                           uint32_t* accb)
{
  if (!info) return fail(UGPU_INVAL, "info is NULL");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  info->states = t.states;
  info->classes = t.classes;
  info->row = t.row;
  info->format = t.format;
  info->table_bytes = (uint32_t)(t.trans.size() * 2 + t.trans32.size() * 4 + (t.format != FMT_BYTE ? 256 : 0));
  info->prefilter_ppm = t.filter ? (uint32_t)(t.fdensity * 1e6) + 1 : 0;
  info->first_bytes = t.first_bytes;
  info->accepting = t.accepting;
  info->contexts = t.ctx_word ? 64u : t.anchored ? 4u : 1u;
  info->shape = (t.finite ? UGPU_SHAPE_FINITE : 0u) | (t.word_cond_edges ? UGPU_SHAPE_WORD_COND : 0u) |
                (t.cap1 != 0 && !t.anchored ? UGPU_SHAPE_ONE_ACCEPT : 0u);
  info->kernel = (t.filter && t.format == FMT_BYTE) ? 0u
                 : t.format == FMT_WIDE              ? 4u
                 : (t.xc && t.cap1 != 0)             ? 5u
                 : (t.xu && t.cap1 != 0)             ? 6u
                 : (t.immediate && t.cap1 != 0)      ? 2u
                 : (t.gap && t.cap1 != 0)            ? 3u
                                                     : 1u;
  if (start) *start = t.start;
  if (accb) *accb = t.accb;
  if (trans) {
    if (t.format == FMT_WIDE) return fail(UGPU_UNSUPPORTED, "wide table (u32 entries): no u16 host form");
    if (trans_cap < t.trans.size()) return fail(UGPU_CAPACITY, "trans capacity");
    std::copy(t.trans.begin(), t.trans.end(), trans);
  }
  if (cls) std::copy(t.cls.begin(), t.cls.end(), cls);
  if (caps) {
    if (caps_cap < t.caps.size()) return fail(UGPU_CAPACITY, "caps capacity");
    std::copy(t.caps.begin(), t.caps.end(), caps);
  }
  return UGPU_OK;
}

int ugpu_tables_prefilter_host(const uint32_t* opc, uint32_t nop, uint8_t* ft, int* enabled)
{
  if (!ft || !enabled) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  std::copy(t.ft, t.ft + 20, ft);
  *enabled = t.filter ? 1 : 0;
  return UGPU_OK;
}

int ugpu_tables_transducer_host(const uint32_t* opc, uint32_t nop, uint16_t* xtrans, uint32_t xtrans_cap, int* local)
{
  if (!local) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *local = t.restart_local ? 1 : 0;
  if (!t.restart_local) return UGPU_OK;
  if (!xtrans || xtrans_cap < t.xtrans.size()) return fail(UGPU_INVAL, "xtrans capacity too small");
  std::copy(t.xtrans.begin(), t.xtrans.end(), xtrans);
  return UGPU_OK;
}

int ugpu_tables_immediate_host(const uint32_t* opc, uint32_t nop, uint8_t* xid, uint32_t xid_cap, uint32_t* rows,
                               uint8_t* sync_byte, int* immediate)
{
  if (!immediate || !rows) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *immediate = t.immediate ? 1 : 0;
  *rows = t.xid_rows;
  if (sync_byte) *sync_byte = t.sync_byte;
  if (!t.immediate || !xid) return UGPU_OK;
  if (xid_cap < t.xid.size()) return fail(UGPU_INVAL, "xid capacity too small");
  std::copy(t.xid.begin(), t.xid.end(), xid);
  return UGPU_OK;
}

int ugpu_tables_gap_host(const uint32_t* opc, uint32_t nop, uint16_t* xg, uint32_t xg_cap, uint8_t* sync, int* gap)
{
  if (!gap) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *gap = t.gap ? 1 : 0;
  if (!t.gap) return UGPU_OK;
  if (!xg || xg_cap < t.xg.size()) return fail(UGPU_INVAL, "xg capacity too small");
  std::copy(t.xg.begin(), t.xg.end(), xg);
  if (sync) std::copy(t.xg_sync.begin(), t.xg_sync.end(), sync);
  return UGPU_OK;
}

int ugpu_tables_xc_host(const uint32_t* opc, uint32_t nop, uint8_t* cls, int* ok)
{
  if (!ok) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *ok = t.xc ? 1 : 0;
  if (cls && t.xc) std::copy(t.xc_tab.begin(), t.xc_tab.end(), cls);
  return UGPU_OK;
}

int ugpu_tables_xu_host(const uint32_t* opc, uint32_t nop, uint8_t* tab, uint32_t* bm3, int* ok)
{
  if (!ok) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *ok = t.xu ? 1 : 0;
  if (tab && t.xu) std::copy(t.xu_tab.begin(), t.xu_tab.end(), tab);
  if (bm3 && t.xu) std::copy(t.xu_bm3.begin(), t.xu_bm3.end(), bm3);
  return UGPU_OK;
}

int ugpu_tables_dom_host(const uint32_t* opc, uint32_t nop, uint32_t* dom, uint32_t dom_cap, uint32_t* n, int* all)
{
  if (!n) return fail(UGPU_INVAL, "NULL argument");
  DfaTables t;
  std::string err;
  const int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *n = (uint32_t)t.dom.size();
  if (all) *all = t.dom_all ? 1 : 0;
  if (dom && dom_cap < t.dom.size()) return fail(UGPU_INVAL, "dom too small");
  if (dom) std::copy(t.dom.begin(), t.dom.end(), dom);
  return UGPU_OK;
}

int ugpu_tables_context_host(const uint32_t* opc, uint32_t nop, uint32_t* acap, uint32_t acap_cap, int* anchored,
                             int* start_acc)
{
  DfaTables t;
  std::string err;
  const int rc = build_tables(opc, nop, t, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  if (acap && acap_cap < t.acap.size()) return fail(UGPU_INVAL, "acap too small");
  if (acap) std::copy(t.acap.begin(), t.acap.end(), acap);
  if (anchored) *anchored = t.anchored ? 1 : 0;
  if (start_acc) *start_acc = t.start_acc ? 1 : 0;
  return UGPU_OK;
}

int ugpu_tables_equivalent_host(const uint32_t* opc_a, uint32_t nop_a, const uint32_t* opc_b, uint32_t nop_b, int* eq)
{
  if (!eq) return fail(UGPU_INVAL, "NULL argument");
  DfaTables a, b;
  std::string err;
  int rc = build_tables(opc_a, nop_a, a, err);
  if (rc == 0) rc = build_tables(opc_b, nop_b, b, err);
  if (rc != 0) return fail(rc == 1 ? UGPU_UNSUPPORTED : UGPU_INVAL, err);
  *eq = tables_equivalent(a, b) ? 1 : 0;
  return UGPU_OK;
}

}  // extern "C"
