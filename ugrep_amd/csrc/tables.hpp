// tables.hpp -- dense DFA tables built from RE/flex opcode words (host side).
//
// Replaces the reference's table consumer: the opcode interpreter of
// Matcher::match (lib/matcher.cpp:125-546) reads Pattern::opc_ word by word and
// scans each state's descending [lo,hi] goto list per input byte (:467-502).
// The GPU walk instead needs one dependent lookup per byte, so the words are
// flattened once per pattern into
//
//   trans[state*R + col]  (u16) = row offset (sid*R) of the target, 0 = dead
//   cls[byte]             (u8)  = column (byte class) when R < 256
//   caps[sid]             (u32) = accept index of TAKE states (cap_)
//
// with state ids renumbered so that dead = 0 and accepting states occupy the
// top range: "entry >= accb" is the accept test and "entry == 0" the dead test.
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include "ctx_bits.hpp"

namespace ugpu {

// FMT_WIDE: states x row > 64 Ki (e.g. two Unicode classes in a row): u32
// row offsets in trans32, no transducer forms; served by the exact-walk
// kernels (wfind_kernel, fix, forest) reading the table from global memory
enum TableFormat : uint32_t { FMT_BYTE = 0, FMT_CLASS = 1, FMT_WIDE = 2 };

struct DfaTables {
  uint32_t format = FMT_BYTE;
  uint32_t states = 0;   // including dead state 0
  uint32_t classes = 0;  // distinct byte columns
  uint32_t row = 256;    // R: 256 (FMT_BYTE) or pow2 >= classes (FMT_CLASS)
  uint32_t log_row = 8;
  uint32_t start = 0;    // start entry = start_sid * R
  uint32_t accb = 0;     // first accepting entry (A * R)
  uint32_t accepting = 0;
  uint32_t cap1 = 0;     // the accept index when every accepting state has the same one, else 0
  bool redo = false;     // some state accepts with REDO (caps = kCapRedo, ctx_bits.hpp); cap1 is then 0
  // Candidate prefilter (replaces the reference's needle/pin prefilters,
  // lib/matcher_avx2.cpp:303-799): the first bytes of the pattern are split
  // into two groups g; a position p can start a match only if for some g
  //   B[p] in B_g  and  B[p+1] in C_g  and  B[p+2] in D_g
  // (B_g = the group's first bytes, C_g / D_g = the bytes that may follow;
  // all bytes once a prefix accepts).  All six sets are tested at once by
  // three byte-table lookups on the 3-bit fields of a byte (v_perm_b32 on the
  // GPU): R(b) = T0[b & 7] & T1[(b >> 3) & 7] & T2[b >> 6], with B_g = bit g,
  // C_g = bit 2+g, D_g = bit 4+g (bits 6, 7 stay 0).  Each set's
  // approximation is a superset of it (safe: it only adds candidates).
  bool filter = false;       // false: dense pattern, no prefilter
  uint8_t ft[20] = {};       // T0[8], T1[8], T2[4]
  double fdensity = 1.0;     // estimated candidate fraction on printable ASCII
  uint32_t first_bytes = 0;
  std::vector<uint16_t> trans;  // states * row (FMT_BYTE, FMT_CLASS)
  std::vector<uint32_t> trans32;  // states * row (FMT_WIDE)
  std::vector<uint8_t> cls;     // 256
  std::vector<uint32_t> caps;   // states
  // FIND transducer (dense_kernel.hip lockstep path), valid when the table is
  // restart-local: whenever a walk dies at byte q, every walk the FIND chain
  // would start between the end of the emitted match (or p+1) and q dies by q
  // without accepting, so the chain never has to re-read bytes before q.  Then
  //   xtrans[s*R + col] = trans[..]                                   (alive)
  //                     = r | XT_DEAD | (trans[start][col] ? XT_LIVE : 0)  (dead)
  // with r = the row of trans[start][col] (the start row when that is dead):
  // one lookup per byte both continues the walk and restarts it at the dying
  // byte.  Flags sit below the row offset (R >= 4), so "entry >= accb" still
  // tests acceptance.
  bool restart_local = false;
  std::vector<uint16_t> xtrans;  // states * row (empty unless restart_local)
  // Immediate FIND transducer (xi_kernel.hip), for restart-local tables whose
  // walks accept on every byte (every live state other than start accepts,
  // nothing re-enters start): a match is then exactly one walk, it starts at
  // the byte that leaves the start state and ends where the walk dies.  Byte
  // ids (u8) carry the walk state and the events of the byte just read:
  //   id = sigma << 3 | Y << 2 | IN << 1 | ST
  //   ST  a match starts at this byte      IN  this byte lies inside a match
  //   Y   this is a sync byte: it kills every walk and starts none, so every
  //       FIND chain is in the start state after it
  // and xid[id * 256 + byte] = next id (rows of ids sharing sigma are equal).
  // Needs sigma < 32 and at least one sync byte.
  bool immediate = false;
  uint32_t xid_rows = 0;        // ids (table rows)
  uint8_t sync_byte = 0;        // smallest sync byte
  std::vector<uint8_t> xid;     // xid_rows * 256
  bool gap = false;             // xg table valid
  std::vector<uint16_t> xg;     // states * row
  std::vector<uint8_t> xg_sync; // 256
  // Device form of the gap transducer (xg_kernel.hip): product states
  // p = (DFA state, "the walk has accepted"), so an entry carries the events
  // of its byte outright (see XG2_* below); stored class-major, column c at
  // entry c * xg2_pad, xg2_pad = 2 (mod 4) so that lanes reading one column in
  // different states, or one state in different columns, hit different LDS
  // banks.  Product state 0 = (start, not accepted).
  std::vector<uint16_t> xg2;    // xg2_cols * xg2_pad
  std::vector<uint8_t> xg2_cls; // 256: column of each byte
  uint32_t xg2_pad = 0, xg2_cols = 0, xg2_states = 0;
  // Two-state tables (xc_kernel.hip): start --G--> A, A --X--> A with A
  // accepting, G a subset of X, every other edge dead.  The FIND chain is then
  // a carry chain (In_i = G_i | X_i & In_{i-1}); xc_tab[byte] = G << 7 | X << 6
  // are the kernel's byte classes.  xc_w: X is exactly the ASCII word bytes
  // [0-9A-Za-z_] (option W on xc_kernel).
  bool xc = false, xc_w = false;
  // xc_wsub: X is a proper subset of the ASCII word bytes ([A-Za-z]+ ...):
  // option W on xc_kernel too (ScanParams::xc_w = 2), the ASCII word bytes
  // outside X coded apart (xc_tab bit 5) so that at_wb / at_we see them
  bool xc_wsub = false;
  std::vector<uint8_t> xc_tab;
  // Code-point runs (xc_kernel U mode): the language is S+ for a prefix-free
  // set S of tokens (one UTF-8 code point each: an ASCII byte, or a lead byte
  // >= 0xC0 followed by 1-3 continuation bytes 80-BF, and no token starts with
  // a continuation byte).  Tokens then never overlap, so the FIND matches are
  // exactly the maximal runs of bytes that lie inside some token, and "byte i
  // lies inside a token" (M_i) is a local property of bytes i-3 .. i+3.  The
  // code of byte x (next byte y) is (see XU_* below)
  //   xu_tab[x]                            x < 0x80 (y is irrelevant)
  //   xu_tab[kXuCls + y]                   x a continuation byte: y's class
  //   xu_tab[256 + (x & 63) * 256 + y]     lead bytes x >= 0xC0
  // xu_bm3: for 3-byte tokens whose third byte z decides beyond the classes
  // (XU_MIX), bit ((x & 15) << 12 | (y & 63) << 6 | (z & 63)).
  // xu_null: a byte that starts no token and is no continuation byte; the
  // kernel reads it in place of bytes outside [lo, readable end).
  bool xu = false;
  uint8_t xu_null = 0;
  std::vector<uint8_t> xu_tab;    // kXuTab bytes
  std::vector<uint32_t> xu_bm3;   // kXuBm3 dwords
  // Line anchors (META_BOL `^`, META_EOL `$`, include/reflex/pattern.h:942-943)
  // and option N (empty matches).  The reference tests meta edges when it has
  // fetched the byte after the current position (lib/matcher.cpp:294-316): a
  // META_BOL edge holds when the walk started at the begin of a line (`bol`,
  // fixed at the walk start, :93), a META_EOL edge when that byte is '\n', EOF,
  // or '\r' before '\n'; the first edge that holds is followed (to at most 5
  // chained meta targets), and a TAKE met on the way is the accept at the
  // current position.  So acceptance is a function of (state, bol, eol):
  //   acap[sid * 4 + bol * 2 + eol] = accept index, 0 = none
  // (also for tables without meta edges: the state's TAKE in all four).
  // anchored: the table has meta edges, so its acceptance is conditional and
  // only the context walk (device_common.hpp walk mode 2) may scan it.
  // start_acc: the start state accepts in some context (empty matches).
  // Word boundaries (META_WBB .. META_EWE, pattern.h:933-940; ctx_word): the
  // context grows to 64 (CTX_* below) -- acap[sid * 64 + ctx] -- with the
  // match begin's at_wb / at_bw (fixed at the walk start like bol) and the
  // position's at_ew / at_we (include/reflex/matcher.h:1194-1319).  Meta
  // targets must be accept-only states (a meta edge into byte edges makes the
  // interpreter backtrack, lib/matcher.cpp:405-460: UGPU_UNSUPPORTED).
  bool anchored = false, start_acc = false, ctx_word = false;
  // ctx_word: the distinct 64-context rows of acap (row 0 all zero) and each
  // state's row -- the device form (tables fit LDS: most states share a row)
  std::vector<uint32_t> acap_rows, acap_map;
  // shape: the language is finite (acyclic DFA); a state whose accept depends
  // on the word context also has byte edges
  bool finite = false, word_cond_edges = false;
  // Dominated restarts (device_common.hpp chain_step): bit s (state id) is set
  // when L(start) is a subset of L(s), i.e. every string a walk from the start
  // state accepts is accepted from s too.  A walk from p that fails (no
  // accept) and is in such a state at q shows that the walk from q fails as
  // well, so the FIND chain may skip q: a needle-free run is crossed with one
  // walk instead of one walk per position.  Empty: not computed (anchored or
  // word-context tables, or more states than the budget allows).
  std::vector<uint32_t> dom;
  // every non-accepting state reachable from the start dominates it: a failed
  // walk (it never accepts) then lets the chain skip every position it
  // crossed, up to the byte it died on (sparse_kernel's long walks)
  bool dom_all = false;
  // Lookahead (X(?=Y), lib/pattern.cpp:2953-2964): per state, TAIL la in bit
  // la and HEAD la in bit 8 + la (la < 4).  A walk runs each state's block on
  // entry as the reference does (lib/matcher.cpp:139-175): TAKE, TAILs (the
  // match end moves back to HEAD la's recorded position), HEADs (record).
  // Empty unless some state has one; such tables take the lookahead walk only.
  std::vector<uint32_t> look;
  bool lookahead = false;
  std::vector<uint32_t> acap;  // states * 4, or states * 64 (ctx_word)
};

// (context bits CTX_*: ctx_bits.hpp)

// xu codes.  Bits 0-3: a thermometer of the token's bytes (bit k: the token
// covers byte x + k; 0x0F = a 4-byte token may start here, XU_SLOW: the kernel
// flags the range and the host scans it with another kernel).  A 3-byte lead
// (x, y) has bit 7 (XU_L3) and in bits 4-6 the continuation-byte classes z
// that complete a token; a continuation byte's code carries the one-hot class
// of the byte after it in bits 4-6 (0 when that is no continuation byte).  So
// the token at x exists iff code(x) & code(x + 1) & 0x70, one AND per dword
// for every byte.  XU_L3 with no class bits (XU_MIX): z decides through xu_bm3.
// The 64 continuation bytes fall into at most 3 classes, chosen so that the
// common mixed blocks (General Punctuation, Currency Symbols first) are unions.
constexpr uint8_t XU_SLOW = 0x0F, XU_L3 = 0x80, XU_MIX = 0x80, XU_CLS = 0x70;
constexpr uint32_t kXuCls = 256 + 64 * 256;               // continuation classes, 256 bytes
constexpr uint32_t kXuTab = kXuCls + 256, kXuBm3 = 2048;

// True when the two tables accept the same strings with the same accept
// indices (so the FIND chains agree on every input).
bool tables_equivalent(const DfaTables& a, const DfaTables& b);

constexpr uint8_t XI_ST = 1, XI_IN = 2, XI_Y = 4;

// Gap transducer (xg_kernel.hip), for restart-local tables in which the
// number of bytes a walk has read since its start or its last accept (its
// "gap") is a function of the DFA state (true for UTF-8 word patterns such as
// \w+, \S+, where states sit at fixed depths of a UTF-8 sequence).  Then every
// accept adds gap + 1 bytes to the current match and the first accept of a
// walk starts a match at q + 1 - (gap + 1), so a walk needs no (p, last)
// registers: only one bit "this walk has accepted" per lane.  Entries are the
// xtrans entries (row | XT_DEAD | XT_LIVE) plus
//   XG_A   the new state accepts (after a death: the restart state does)
//   L      bits 3-5: gap + 1 of that accept (0 when XG_A is clear)
// which needs row >= 64.  xg_sync[byte] = 1 for sync bytes (kill every walk,
// start none).
constexpr uint16_t XG_A = 4;
constexpr uint32_t XG_LSHIFT = 3;

// xg2 entries (u16): bits 0-2 L (gap + 1 of an accept on this byte, 0 = no
// accept), bit 3 F (the first accept of a walk: a match starts at
// q + 1 - L), bit 4 D (the walk died on this byte; the entry is the restart),
// bits 5-15 = 2 * the target product state (its byte offset within a column).
constexpr uint32_t XG2_L = 7, XG2_F = 8, XG2_D = 16, XG2_ROWSHIFT = 5;
constexpr uint32_t kXg2MaxStates = 1024;

constexpr uint16_t XT_DEAD = 1;  // the walk died on this byte; the row is the restart state
constexpr uint16_t XT_LIVE = 2;  // the restart at this byte is alive (a walk begins here)

// Returns 0 (UGPU_OK), 1 (UNSUPPORTED) or 2 (INVAL); err gets a message.
int build_tables(const uint32_t* opc, uint32_t nop, DfaTables& out, std::string& err);
// the prefilter tables (ft) of a loop-needle table's strings; returns the estimated candidate density
double needle_filter(const std::vector<std::string>& needles, uint8_t (&ft)[20]);

}  // namespace ugpu
