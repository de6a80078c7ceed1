// scan_kernels.hpp -- device side of the MI355X FIND engine.
//
// One chain = the sequence of search positions the reference's FIND loop visits
// (lib/matcher.cpp:42-750): at position p walk the DFA,
// remember the last accepting state, emit the longest non-empty match and jump
// to its end, else move to p+1.  The chain is sequential; the GPU cuts the
// input into pieces (lane segments, wave ranges, GPU shards), runs every
// piece's chain speculatively from the piece start, and stitches the true chain
// back together:
//
//   * the true chain enters piece k at the exit x of piece k-1 (x >= start);
//   * if x differs from the speculative entry, both chains are re-walked in
//     lock step, subtracting the speculative matches and adding the true ones,
//     until they meet (then everything after is identical) or both leave the
//     piece (then the exit changed and the next piece repeats this).
//
// Lanes of a wave resolve this with DPP rounds inside the scan kernels
// (dense_kernel.hip; sparse_kernel.hip has no lane pieces: its candidates are
// resolved in order), waves are stitched by fix_kernel, GPU shards by
// chain_fix_kernel (ugrep_amd/dist.py).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ugpu {

constexpr int kMaxRec = 8192;          // chain records stitched by one fix_kernel block
constexpr int kFixThreads = 1024;
constexpr int kWaveTile = 4096;        // sparse kernel: bytes per wave per iteration
constexpr int kSpWaves = 4;            // sparse kernel: waves per workgroup
// Dense kernel geometry (overridable for variant builds, ugrep_amd/Makefile):
// lane segment bytes (S/4 odd) and waves per workgroup.  One staged table per
// workgroup: the big class tables share theirs among more waves.  Measured
// (16 GiB C3 / 8 GiB C4): byte S = 60/92/124/188/252 -> 29.2/22.1/20.7/18.7/
// 20.7 ms; class S = 28/44/60/92 (16/12/8/8 waves) -> 20.7/17.8/18.9/14.8 ms:
// per-segment costs (walk tails, fix-ups) favour long segments until the
// LDS buffers cut occupancy.
#ifndef UGPU_DSEG_BYTE
#define UGPU_DSEG_BYTE 188
#endif
#ifndef UGPU_DSEG_CLASS
#define UGPU_DSEG_CLASS 92
#endif
#ifndef UGPU_DWAVES_BYTE
#define UGPU_DWAVES_BYTE 4
#endif
#ifndef UGPU_DWAVES_CLASS
#define UGPU_DWAVES_CLASS 8
#endif
constexpr int kDSegByte = UGPU_DSEG_BYTE;    // 256-column tables
constexpr int kDSegClass = UGPU_DSEG_CLASS;  // class tables
constexpr int kDWavesByte = UGPU_DWAVES_BYTE;
constexpr int kDWavesClass = UGPU_DWAVES_CLASS;
constexpr int dense_waves(uint32_t format) { return format == 0 ? kDWavesByte : kDWavesClass; }
constexpr uint64_t kMaxRecBytes = 1ull << 30;  // bytes per chain record (32-bit wave-relative offsets)

struct BlockRec {
  uint64_t entry, exit, cnt, dg, dc, pad0, pad1, pad2;
};
// sparse_kernel COUNT records also describe the first match their speculative
// chain keeps, for fix_kernel's shortcuts (pad0 = its start c1, pad1 = its end
// e1: 0 = the chain keeps no match, kOpenEnd = the open walk below; pad2 =
// accept entry | kRecOpen | kRecFirst)
constexpr uint64_t kOpenEnd = ~0ull;
constexpr uint64_t kRecOpen = 1ull << 32;   // the wave ends in an open walk (OpenRec)
constexpr uint64_t kRecFirst = 1ull << 33;  // pad0 / pad1 are valid

// Open walk of a sparse_kernel wave (walk truncation, P.open): the walk of a
// kept candidate was still alive at the wave's walk limit `lim` (its range
// end).  The wave counts no match for it and keeps nothing after it
// (optimistically: the walk's match covers the rest of its range).  fix_kernel
// resolves it from the next waves' records (convergence with their first
// walks) and stores the walk's true end; the WRITE pass reads that back.
struct OpenRec {
  uint64_t c;      // walk start
  uint64_t last;   // last accept position before lim (== c: none)
  uint64_t lim;    // where the walk stands: kOpenSlack past the wave's range end (or less at rend)
  uint32_t s, le;  // DFA entry at lim, entry of the last accepting state
  // fix_kernel resolution
  uint64_t q;      // R1: position where the walk converged with / died
  uint64_t lastw;  // R1: last accept of the walk at or after lim (0: none)
  uint32_t lew;    // R1: its accepting entry
  uint32_t type;   // R1: kOpenDead / kOpenConv / kOpenUnres
  uint64_t e;      // R2: the walk's last accept overall (== c: it never accepts)
  uint32_t le_e;   // R2: its accepting entry
  uint32_t sq;     // R1: the walk's DFA entry at q (R1b goes on from there)
};
constexpr uint32_t kOpenDead = 1, kOpenConv = 2, kOpenUnres = 3;

// A sparse_kernel wave suspended at a walk longer than its 32-byte window: its
// chain state and the walked batch, for the resume launch (sparse_kernel.hip)
struct PendSlot {
  uint64_t c;
  uint32_t s, le, packed;  // qr | lr << 8 | st << 16 | todo << 24
  uint32_t pad;
};
struct SuspRec {
  uint64_t x, widx, cnt, dg, dc, c1, e1, rs, sgn;
  uint64_t lbr, lbs;  // loop-needle tables: the lookback carry (sparse_kernel.hip lb_batch)
  uint32_t wover, ovf, first, open, le1, sgover, tile, dn;
  PendSlot lanes[64];
};
constexpr uint64_t kOpenConvBudget = 4096;  // bytes R1 may walk looking for convergence
constexpr uint64_t kOpenSlack = 256;        // bytes a walk goes on past its wave's range end before it is open

struct DevTotals {
  uint64_t count, digest, dcap, entry, exit;
  uint32_t flags, rounds;
};

#define UGPU_FLAG_HALO 1u
#define UGPU_FLAG_CAPACITY 2u
// a stitch (fix_kernel rounds or one merge walk) ran past its work budget: the
// FIND chains of this table do not resynchronise on this input (e.g. \D\D over
// text without digits); the totals are invalid and the host resolves the
// range with the forest FIND (forest.hip)
#define UGPU_FLAG_BUDGET 4u
// option W on xc_kernel met a byte >= 0x80 (the W rules then need the UTF-8
// decode): the host redoes the range with wfind_kernel
#define UGPU_FLAG_WSLOW 32u
// stage_copy_kernel left waves whose staged records were not the true chain's
#define UGPU_FLAG_NEEDWRITE 64u
// xc_kernel's U mode met a lead byte of a 4-byte token (tables.hpp XU_SLOW):
// the host redoes the range with the table's next kernel
#define UGPU_FLAG_USLOW 128u
// xc_kernel U mode (fast kernel): a code with bit 3 (an XU_MIX or XU_SLOW lead)
// was met; the host redoes the range with the exact U kernel (P.xu_exact)
#define UGPU_FLAG_UMIX 256u
// sparse_kernel: a wave's walk was truncated at its range end (OpenRec); fix_kernel resolves it
#define UGPU_FLAG_OPEN 512u
constexpr uint32_t kStageOver = 0xffffffffu;
constexpr uint32_t kStageDone = 0xfffffffeu;
constexpr uint32_t kStagePer = 1024;  // staged records per wave (16 B each: 128 MiB for 8192 waves)

struct ScanParams {
  const uint8_t* g;   // 16-byte aligned base of the scanned bytes
  uint64_t lo, hi;    // chain positions [lo, hi) (base coordinates)
  uint64_t rend;      // walks may read bytes < rend
  int64_t delta;      // reported start = position + delta
  uint32_t at_eof;    // rend is the end of the stream
  uint32_t ablate;    // benchmarking only (UGPU_ABLATE; sparse kernel: 1 loads, 2 + prefilter, 3 no walks;
                      // dense: 4 no fix-up, 5 no tails; xi: 6 loads only)
  uint32_t zero;      // always 0 (keeps prefetch loads alive in xi_kernel)
  uint64_t t0, t1, tpb;  // tiles [t0, t1), tiles per record
  uint32_t unit;         // bytes per tile (kWaveTile, or dense_unit())
  uint32_t nrec;         // chain records (blocks or waves)
  uint32_t nstates;
  const uint16_t* trans;
  const uint16_t* xtrans;  // FIND transducer table or NULL (dense kernel, tables.hpp)
  const uint8_t* xid;      // immediate transducer byte ids (xi_kernel, tables.hpp) or NULL
  uint32_t xid_rows;
  const uint16_t* xg;      // gap transducer, device form (xg_kernel, tables.hpp xg2) or NULL
  const uint8_t* xg_sync;  // its sync-byte flags
  const uint8_t* xg_cls;   // its byte columns
  uint32_t xg_stride;      // bytes per column
  uint32_t xg_entries;     // u16 entries (multiple of 8)
  const uint8_t* cls;
  const uint32_t* trans32;  // wide tables (format 2): u32 row offsets, states * row
  const uint32_t* caps;
  uint32_t ntrans_pad;   // u16 entries, multiple of 8
  uint32_t start, accb, log_row;
  uint32_t ft[5];        // prefilter lookup tables T0 (lo, hi), T1 (lo, hi), T2 (tables.hpp)
  uint32_t cap1;         // the accept index when all accepting states share it, else 0
  uint32_t grid;
  BlockRec* recs;
  const uint64_t* entries;   // OFFSETS pass: exact block entries
  const uint64_t* out_base;  // OFFSETS pass: first output index per block
  uint64_t* out_start;
  uint32_t* out_len;
  uint32_t* out_cap;
  uint64_t out_capacity;
  uint64_t* out_fix;         // xc_kernel OFFSETS: per wave, a record whose len holds its raw end (~0: none)
  uint32_t* flags;
  DevTotals* totals;
  uint64_t* entries_out;     // fix_kernel: exact block entries
  uint64_t* out_base_out;    // fix_kernel: exclusive scan of block counts
  // option W (ugrep -w): Unicode Word ranges ([lo, hi] pairs) or NULL, and the
  // base coordinate of the buffer's first byte (at_wb is true there: BOB)
  const uint32_t* wtab;
  uint32_t nwtab;
  uint64_t bob;
  // stitch budgets (UGPU_FLAG_BUDGET): fix_kernel rounds, and chain bytes one
  // merge may cross before giving up (fix_kernel, chain_fix_kernel)
  uint32_t max_rounds;
  uint64_t merge_budget;
  // two-state tables (xc_kernel.hip)
  const uint8_t* xc_cls;  // byte classes G << 7 | X << 6 (256 B)
  // single-pass OFFSETS (sparse_kernel): a COUNT pass with st_n set also stages
  // each wave's records (st_per per wave); st_n[wave] = records staged, or
  // kStageOver; stage_copy_kernel moves them and marks the wave kStageDone
  uint64_t* st_start;
  uint32_t* st_len;
  uint32_t* st_cap;
  uint32_t* st_n;
  uint32_t st_per;
  uint32_t xc_w;          // option W on xc_kernel: 1 = X is the ASCII word bytes, 2 = a proper subset of them
  uint32_t xu_w;          // option W on xc_kernel's U mode (tables equivalent to \w+): run edges checked
  uint32_t xu_exact;      // xc_kernel U mode: the exact main loop (XU_MIX / XU_SLOW checked per chunk)
  // code-point run tables (xc_kernel U mode, tables.hpp xu_*) or NULL
  const uint8_t* xu_tab;  // kXuTab bytes (4-byte aligned)
  const uint32_t* xu_bm3; // kXuBm3 dwords
  uint32_t xu_null;       // the fill byte
  // xc_kernel COUNT (U mode or carry chain, no option W): also write the In
  // bit of every byte (bit p % 16 of inbits[p / 16], base coordinates), which
  // xc_expand_kernel turns into the match records (OFFSETS without a second
  // walk); NULL: not written
  uint16_t* inbits;
  // line anchors / option N (tables.hpp acap): per-context accept indices
  // (sid * 4 + bol * 2 + eol; ctx_word: sid * 64 + CTX_* bits, with wtab
  // set) or NULL; bol0: the position bob starts a line (the byte before the
  // buffer is '\n', or the buffer begins the input); nul: option N, empty
  // matches are reported
  const uint32_t* acap;
  // sparse_kernel: no match starts after a word character (option W's at_wb
  // at the match begin, lib/matcher.cpp:107; or a table whose every accept
  // needs CTX_WB), so candidates right after an ASCII letter are dropped
  uint32_t wstart;
  // sparse_kernel, loop-needle tables (engine.hip loop_needle): the prefilter
  // (ft) finds the needle N; each candidate walks back over the bytes of C
  // (256-bit mask) to its run's start.  NULL: ft finds first bytes.
  const uint32_t* lb_cls;
  // plain walks: the states that dominate the start state (tables.hpp dom;
  // bit = state id), or NULL: a failed walk skips the positions it crossed in
  // such states (device_common.hpp chain_step)
  const uint32_t* dom;
  // lookahead tables (tables.hpp look): per state TAIL / HEAD masks, or NULL;
  // every walk of such a table is the lookahead walk (device_common.hpp kWalkLook)
  const uint32_t* look;
  // sparse_kernel: every non-accepting state dominates the start (tables.hpp
  // dom_all): a failed long walk moves the chain past the byte it died on
  uint32_t dom_all;
  uint32_t bol0;
  uint32_t nul;
  uint32_t ctx_word;
  // the number of acap entries (4 * states, or ctx_word: 64 * distinct rows)
  // and, ctx_word, each state's row (tables.hpp acap_rows / acap_map)
  uint32_t acap_n;
  const uint32_t* amap;
  // sparse_kernel: acap and amap are staged in LDS (small context tables)
  uint32_t acap_lds;
  // sparse_kernel walk truncation: per wave, the open walk (COUNT pass writes,
  // fix_kernel resolves, the WRITE pass reads); NULL: walks run to rend
  OpenRec* open;
  // sparse_kernel long walks: per wave, suspended (1) or not (0), and the
  // suspended state; NULL: walks complete in their lanes (option W)
  uint32_t* susp;
  SuspRec* srec;
};

// Forest FIND (forest.hip): exact for every table, no resynchronisation
// assumed; runs when a speculative stitch exceeds its budget.
struct ForestArgs {
  uint64_t c_lo, c_hi;  // chunk of chain positions (base coordinates)
  uint32_t nblk;        // blocks of forest_block() positions in the chunk
  uint32_t* ex;         // per chunk position: its block exit - block end
  uint64_t* entry;      // device: chain entry of the chunk (in) / its exit (out)
  uint64_t* run;        // device: count, digest, dcap of the chunks so far
  uint64_t* bentry;     // per block: exact chain entry
  uint64_t* bsum;       // per block: count, digest, dcap
  uint64_t* bbase;      // per block: first output index
};
constexpr uint64_t kFChunk = 64ull << 20;  // positions per forest chunk (4 B of exits each)
hipError_t launch_forest(const ScanParams& P, uint32_t format, const ForestArgs& A, uint64_t entry, bool write,
                         DevTotals* tot, hipStream_t stream);
uint64_t forest_block();

// launchers (scan_kernels.hip, gen.hip)
hipError_t launch_fix(const ScanParams& P, uint32_t format, hipStream_t stream);
hipError_t launch_pack_records(const uint64_t* start, const uint32_t* len, const uint32_t* cap, uint64_t n,
                               uint64_t base, uint8_t* out, int caps, int dense, uint64_t* esc, uint32_t* nesc,
                               hipStream_t stream);
hipError_t launch_chain_fix(const ScanParams& P, uint32_t format, uint64_t old_entry, uint64_t new_entry,
                            hipStream_t stream);
hipError_t launch_gen(int kind, uint64_t seed, uint64_t off, uint8_t* dbuf, uint64_t len, hipStream_t stream);
// sparse (prefiltered) wave-persistent kernel, sparse_kernel.hip
hipError_t launch_sparse(const ScanParams& P, bool write, size_t smem, hipStream_t stream);
hipError_t launch_stage_copy(const ScanParams& P, hipStream_t stream);
hipError_t sparse_occupancy(const ScanParams& P, size_t smem, int* blocks_per_cu);
size_t sparse_smem_bytes(uint32_t ntrans_pad, uint32_t nstates, uint32_t nlds_acap = 0);
// context tables whose acap (+ amap) entries sparse_kernel stages in LDS
constexpr uint32_t kSpAcapLds = 2048;
// line-level consumers, lines.hip
struct LineRec {
  uint64_t first_line, last_line;  // lines of the wave's first / last match start (0: none)
  uint64_t trans;                  // matches whose line differs from the previous match's (first included)
  uint64_t nmatch;
};
struct LinesParams {
  const uint8_t* g;         // 16-byte aligned buffer
  uint64_t len;             // bytes
  uint64_t per;             // bytes per wave range (multiple of 4 KiB)
  uint64_t nwaves;
  const uint64_t* starts;   // sorted match starts (offsets into g)
  uint64_t nmatch;
  uint64_t* counts;         // out (count pass): newlines per wave range
  const uint64_t* prefix;   // in (assign pass): newlines before each wave range
  uint64_t* lines;          // out: line of each match start (1-based), may be NULL
  LineRec* recs;            // out: per-wave line transitions
  uint16_t* qcount;         // sparse mode: newlines per 1 KiB quarter (count pass out, assign pass in)
};
// sparse = the assign pass loads only the 1 KiB quarters holding match starts
// (the count pass also writes qcount); dense = it reloads the whole buffer
hipError_t launch_nl_count(const LinesParams& L, bool sparse, hipStream_t stream);
hipError_t launch_nl_assign(const LinesParams& L, bool sparse, hipStream_t stream);
uint32_t lines_tile();
constexpr uint32_t kLinesQuarter = 1024;
// binary-file detection, utf8.hip: first byte failing reflex::isutf8 (or, with
// nul, the first 0x00) of the data bytes [head, head + len) of the 16-byte
// aligned span g[0, span), atomically min'ed into *out (preset to ~0)
struct Utf8Params {
  const uint8_t* g;  // 16-byte aligned
  uint64_t head;     // data start within the span (< 16)
  uint64_t len;      // data bytes
  uint64_t span;     // head + len rounded up to 16
  uint64_t per;      // bytes per wave range (multiple of the 4 KiB tile)
  uint64_t nwaves;
  uint64_t* out;     // span offset of the first failing byte (head + len: truncated sequence)
};
hipError_t launch_utf8(const Utf8Params& U, bool nul, hipStream_t stream);
uint32_t utf8_tile();
// option W (-w) FIND, wfind.hip: one chain record per wave (64 lane segments
// stitched in the wave), exact W walks (device_common.hpp), records stitched
// by fix_kernel; COUNT and OFFSETS passes
hipError_t launch_wfind(const ScanParams& P, uint32_t format, bool write, hipStream_t stream);
uint32_t wfind_unit();
uint32_t wfind_waves();
size_t wfind_smem_bytes(uint32_t ntrans_pad, uint32_t nstates, uint32_t nwtab, uint32_t nacap, uint32_t nmap);
// immediate-transducer kernel, xi_kernel.hip (COUNT mode only)
hipError_t launch_xi(const ScanParams& P, size_t smem, hipStream_t stream);
hipError_t xi_occupancy(size_t smem, int* blocks_per_cu);
uint32_t xi_unit();
uint32_t xi_waves();
// gap-transducer kernel, xg_kernel.hip (COUNT mode only)
hipError_t launch_xg(const ScanParams& P, hipStream_t stream);
hipError_t xg_occupancy(uint32_t entries, int* blocks_per_cu);  // 0 blocks: the table does not fit
size_t xg_smem_bytes(uint32_t entries);
uint32_t xg_unit();
uint32_t xg_waves();
// two-state carry-chain kernel, xc_kernel.hip (COUNT, or WRITE into P.out_*
// at the output bases of the COUNT pass's records; out_capacity = the count)
hipError_t launch_xc(const ScanParams& P, bool write, hipStream_t stream, uint64_t count = 0);
hipError_t xc_occupancy(bool u, int* blocks_per_cu);  // u: the U-mode COUNT kernel
uint32_t xc_unit(bool u);  // wave-tile bytes (u: U mode)
// OFFSETS from the In bits of an xc_kernel COUNT pass (P.inbits): one
// workgroup per COUNT wave record writes that wave's records; then the fix of
// the one record per wave whose start an earlier wave wrote
hipError_t launch_xc_expand(const ScanParams& P, hipStream_t stream, uint64_t count);
uint32_t xc_waves();
// dense wave-persistent kernel, dense_kernel.hip
hipError_t launch_dense(const ScanParams& P, uint32_t format, bool write, size_t smem, hipStream_t stream);
hipError_t dense_occupancy(uint32_t format, bool cap1, bool xt, size_t smem, int* blocks_per_cu);
size_t dense_smem_bytes(uint32_t format, uint32_t ntrans_pad, uint32_t nstates);
uint32_t dense_unit(uint32_t format);

}  // namespace ugpu
