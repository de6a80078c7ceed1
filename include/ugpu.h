/*
 * ugpu.h -- C ABI of the MI355X DFA buffer-scan engine (ugrep_amd).
 *
 * This is the drop-in boundary for ugrep's hot path: the FIND loop of
 * reflex::Matcher::match(Const::FIND) (reference lib/matcher.cpp:42-750), i.e.
 * the adv_ prefilters (lib/matcher.cpp:797-954, lib/matcher_avx2.cpp:78-799,
 * lib/matcher_avx512bw.cpp:50-463) plus the DFA opcode walk (lib/matcher.cpp:
 * 125-546), driven by `while (matcher->find())` (src/ugrep.cpp:10544, :10869).
 *
 * Input artifact: the reference's compiled pattern, Pattern::opc_[0..nop_)
 * (include/reflex/pattern.h:1302-1304; word format :1155-1247; produced by
 * Pattern::encode_dfa, lib/pattern.cpp:2823-3063).  The same words are what the
 * reference's precompiled-table constructor Pattern(const Opcode*, ...) takes
 * (include/reflex/pattern.h:151-159), so a caller passes pattern.opc_ as is.
 *
 * Semantics: identical match records (start, length, accept index) to
 * Matcher::find() on a fully buffered input (AbstractMatcher::buffer(),
 * include/reflex/absmatcher.h:542-591): leftmost-longest, non-overlapping,
 * empty matches rejected unless option N (UGPU_PAT_EMPTY), option A off;
 * option W by UGPU_PAT_WORD.  Line anchors (META_BOL/META_EOL) and word
 * boundaries (META_WBB/WBE/WEB/WEE/NWB/NWE/BWB/EWB) at the start or end of a
 * match become per-context accepts.  Tables with
 * lookahead HEAD/TAIL words, buffer anchors (META_BOB/EOB), assertions between
 * consumed characters, or REDO words return UGPU_UNSUPPORTED; the caller keeps
 * its CPU matcher for those (include/reflex/pattern.h:1194-1217).
 *
 * All functions return an int status; no exceptions cross this ABI (reference
 * errors: regex_error lib/pattern.cpp:162-169, std::bad_alloc absmatcher.h:401).
 * Handles are opaque.  A ugpu_dfa is immutable after creation and may be shared
 * by threads (the reference shares one Pattern across GrepWorker clones,
 * src/ugrep.cpp:4146-4149, :4206); a ugpu_scanner is per thread/stream.
 */
#ifndef UGPU_H
#define UGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define UGPU_OK 0
#define UGPU_UNSUPPORTED 1 /* table needs lookahead/REDO/inner assertions: use the CPU matcher */
#define UGPU_INVAL 2       /* bad argument or malformed opcode table */
#define UGPU_NOMEM 3       /* host or device allocation failed */
#define UGPU_DEVICE 4      /* HIP runtime error (see ugpu_last_error) */
#define UGPU_HALO 5        /* a match walked past readable bytes of a non-final shard */
#define UGPU_CAPACITY 6    /* more matches than the caller's output capacity */

/* scan modes */
#define UGPU_MODE_COUNT 0   /* count + digests only */
#define UGPU_MODE_OFFSETS 1 /* also materialize (start, len, cap) records */

/* ABI version of this header: bumped whenever a struct below changes layout
   or an entry point is added (ugpu_dfa_info gained contexts/shape in ABI 2;
   ugpu_stream_reserve came in ABI 3).  A caller compiled against
   one header checks ugpu_abi_version() == UGPU_ABI_VERSION before passing a
   struct to the library (integration/reflex_gpu_matcher.h does; on a mismatch
   it keeps the CPU matcher). */
#define UGPU_ABI_VERSION 3

typedef struct ugpu_dfa ugpu_dfa;
typedef struct ugpu_scanner ugpu_scanner;

typedef struct ugpu_dfa_info
{
  uint32_t states;      /* DFA states including the dead state */
  uint32_t classes;     /* byte equivalence classes */
  uint32_t row;         /* table row width (256 = byte-indexed, else class-indexed, pow2) */
  uint32_t format;      /* 0 = next[state][byte], 1 = cls[byte] + next[state][class] */
  uint32_t table_bytes; /* bytes of the transition table staged in LDS */
  uint32_t prefilter_ppm; /* prefiltered (sparse) scan: est. candidate positions per million + 1; 0 = dense scan */
  uint32_t first_bytes; /* number of bytes that can start a match (|fst_|) */
  uint32_t accepting;   /* accepting states */
  uint32_t kernel;      /* kernel of a COUNT scan: 0 sparse (prefiltered), 1 dense, 2 xi (immediate
                           transducer; UGPU_XI=0 selects dense), 3 xg (gap transducer; UGPU_XG=0),
                           4 wfind (option W, UGPU_PAT_WORD), 5 xc (two-state carry chain; UGPU_XC=0),
                           6 xc U mode (code-point runs without a gap transducer; UGPU_XU=1 prefers it,
                           UGPU_XU=0 never) */
  uint32_t contexts;    /* accept contexts per state of the per-context accepts (ugpu_tables_context_host):
                           1 = none (no meta edges), 4 = line anchors (bol * 2 + eol), 64 = word boundaries
                           (ugrep_amd/csrc/ctx_bits.hpp) */
  uint32_t shape;       /* UGPU_SHAPE_* bits (the drop-in matcher's test of where the reference's
                           match predictor is exact for word-boundary patterns) */
} ugpu_dfa_info;

#define UGPU_SHAPE_FINITE 1u     /* the language is finite (no cycle in the DFA) */
#define UGPU_SHAPE_WORD_COND 2u  /* a state whose accept depends on a word boundary also has byte edges */
#define UGPU_SHAPE_ONE_ACCEPT 4u /* every match has the same accept index: 12-byte records (ugpu_scan_offsets d_cap NULL) */
#define UGPU_SHAPE_LOOKAHEAD 16u /* lookahead (X(?=Y): TAIL/HEAD words): the lookahead walk on wfind_kernel */
#define UGPU_SHAPE_LOOP_NEEDLE 8u /* C+ N on the sparse kernel: the prefilter looks for the needle N and walks back
                                     (UGPU_LB=0 disables) */

/* Totals of one scan.  digest = sum(start*31 + len), dcap = sum((start+1)*cap),
   both mod 2^64, start = byte offset + bias. */
typedef struct ugpu_totals
{
  uint64_t count;
  uint64_t digest;
  uint64_t dcap;
  uint64_t entry;  /* chain position entering the range (== lo for a fresh scan) */
  uint64_t exit;   /* first chain position >= hi: where the search resumes after the range */
  uint32_t flags;  /* bit0: a walk hit the readable end of a non-final shard (UGPU_HALO);
                      bit3 (UGPU_TOT_FOREST): the speculative stitch did not converge (FIND chains
                      that never resynchronise, e.g. \D\D over text without digits) and the range
                      was resolved exactly by the forest FIND (ugrep_amd/csrc/forest.hip);
                      bit4 (UGPU_TOT_WFAST): option W on a \w+ table ran the non-W kernels
                      (the scanned bytes are valid UTF-8, so W removes nothing) */
  uint32_t fix_rounds;
} ugpu_totals;

#define UGPU_TOT_FOREST 8u
#define UGPU_TOT_WFAST 16u

/* Library-owned match list for ugpu_find_all. */
typedef struct ugpu_result
{
  uint64_t count;
  uint64_t digest;
  uint64_t dcap;
  uint64_t *start; /* count entries, byte offsets relative to buf */
  uint32_t *len;
  uint32_t *cap;   /* accept index (Matcher::accept(), absmatcher.h:605-609) */
} ugpu_result;

/* --- pattern tables (replaces the Pattern -> Matcher table consumer) --- */

/* Build the dense device tables from opcode words and upload them once to the
   current device.  pattern_flags: 0, or UGPU_PAT_WORD for Matcher option W
   (ugrep -w: matches bounded by word boundaries, src/ugrep.cpp:8616-8618,
   lib/matcher.cpp:107, :142, :208, include/reflex/matcher.h:1194-1237); at_wb
   at a walk start reads the code point before it, so dbuf[0] counts as the
   begin of the input and a scan that starts inside the input passes the bytes
   before lo in dbuf (4 suffice; ugpu_find_all_multi and the stream API do).
   UGPU_PAT_EMPTY: Matcher option N (ugrep -Y, and -x:
   src/ugrep.cpp:8381-8386, :8612-8613), empty matches are reported
   (lib/matcher.cpp:682-728; never at the end of the input).  Tables with line
   anchors (META_BOL ^, META_EOL $ edges, include/reflex/pattern.h:942-943, as
   ugrep -x makes, src/cnf.hpp:167-185) are accepted; other meta edges (word
   boundaries, \A, \Z, indent) return UGPU_UNSUPPORTED.  Anchored tables, and
   tables that match the empty string under option N, scan on the exact context
   walk (wfind_kernel; its W rules replaced by the anchor rules): bol at a walk
   start is "the byte before is '\n' or the position is the buffer begin"
   (see ugpu_scanner_context for buffers that do not begin the input), eol is
   "the next byte is '\n', EOF, or '\r' before '\n'".  W together with anchors
   or empty matches returns UGPU_UNSUPPORTED. */
#define UGPU_PAT_WORD 1u
#define UGPU_PAT_EMPTY 2u
int ugpu_dfa_create(const uint32_t *opc, uint32_t nop, uint32_t pattern_flags, ugpu_dfa **out);
/* Releases made once the process is exiting (exit() or a return from main:
   static destructors, atexit handlers that run after the engine's own) free
   nothing and return UGPU_OK -- the HIP runtime may already be torn down --
   for ugpu_dfa_destroy, ugpu_scanner_destroy, ugpu_stream_destroy and
   ugpu_records_free; ugpu_select_device makes no HIP call then. */
int ugpu_dfa_destroy(ugpu_dfa *dfa);
int ugpu_dfa_info_get(const ugpu_dfa *dfa, ugpu_dfa_info *info);

/* Host-only: what ugpu_dfa_create(opc, nop, pattern_flags) would return
   (UGPU_OK, UGPU_UNSUPPORTED, UGPU_INVAL) and, on UGPU_OK, the info it would
   report (the kernel a COUNT scan runs) -- without touching a device, so a
   caller can decide whether a device is worth initialising (the drop-in
   matcher decides CPU or GPU per input before any HIP call). */
int ugpu_dfa_plan_host(const uint32_t *opc, uint32_t nop, uint32_t pattern_flags, ugpu_dfa_info *info);

/* Host-only: build the dense tables without touching a device (inspection and
   CPU tests).  trans gets states*row u16 entries (entry = target_state*row,
   0 = dead), cls 256 bytes, caps `states` accept indices; *start is the start
   entry, *accb the first accepting entry.  Pass NULL arrays to query sizes
   through info first. */
int ugpu_tables_build_host(const uint32_t *opc, uint32_t nop, ugpu_dfa_info *info, uint16_t *trans,
                           uint32_t trans_cap, uint8_t *cls, uint32_t *caps, uint32_t caps_cap, uint32_t *start,
                           uint32_t *accb);

/* Host-only: the prefilter lookup tables (T0[8], T1[8], T2[4] bucket bytes, see
   ugrep_amd/csrc/tables.hpp) into ft[20]; returns UGPU_OK and sets *enabled to 1
   when the sparse (prefiltered) kernel is used for this table. */
int ugpu_tables_prefilter_host(const uint32_t *opc, uint32_t nop, uint8_t *ft, int *enabled);

/* Host-only: the FIND transducer table of a restart-local DFA (see
   ugrep_amd/csrc/tables.hpp: entries = row | XT_DEAD(1) | XT_LIVE(2)), same
   shape as trans.  *local = 0 (and nothing written) when the table is not
   restart-local; then the dense kernel uses its general walk. */
int ugpu_tables_transducer_host(const uint32_t *opc, uint32_t nop, uint16_t *xtrans, uint32_t xtrans_cap,
                                int *local);

/* Host-only: the immediate FIND transducer of xi_kernel (ugrep_amd/csrc/
   tables.hpp): for restart-local tables whose walks accept on every byte,
   u8 ids (walk state << 3 | SYNC 4 | IN 2 | START 1), rows*256 bytes of
   next ids.  *immediate = 0 (nothing written) when the table does not qualify;
   pass xid = NULL to query *rows first. */
int ugpu_tables_immediate_host(const uint32_t *opc, uint32_t nop, uint8_t *xid, uint32_t xid_cap, uint32_t *rows,
                               uint8_t *sync_byte, int *immediate);

/* Host-only: the gap transducer of xg_kernel (ugrep_amd/csrc/tables.hpp):
   xtrans entries plus XG_A (4, the new state accepts) and the accept's
   gap + 1 in bits 3-5, same shape as trans; sync[256] = sync-byte flags.
   *gap = 0 (nothing written) when the table does not qualify. */
int ugpu_tables_gap_host(const uint32_t *opc, uint32_t nop, uint16_t *xg, uint32_t xg_cap, uint8_t *sync, int *gap);

/* Host-only: the byte classes of xc_kernel (two-state tables: start --G--> A
   --X--> A, ugrep_amd/csrc/tables.hpp): cls[256] = G << 7 | X << 6 (may be
   NULL).  *ok = 0 when the table does not qualify.  (Replaces, for these
   tables, the per-byte opcode scan of lib/matcher.cpp:460-545.) */
int ugpu_tables_xc_host(const uint32_t *opc, uint32_t nop, uint8_t *cls, int *ok);

/* Host-only: the code-point run tables of a table whose language is S+ for a
   set S of single-code-point tokens (\w+, \S+, [[:alpha:]]+ over UTF-8;
   ugrep_amd/csrc/tables.hpp xu_*): tab[256 + 64 * 256 + 256] token codes and
   bm3[2048] third-byte bits (either may be NULL).  *ok = 0 when the table does
   not qualify.  (Replaces, for these tables, the per-byte opcode scan of
   lib/matcher.cpp:460-545.) */
int ugpu_tables_xu_host(const uint32_t *opc, uint32_t nop, uint8_t *tab, uint32_t *bm3, int *ok);

/* Host-only: the dominated-restart bits of the dense tables (bit s of
   dom[s / 32], state numbering as ugpu_tables_build_host): L(start) is a
   subset of L(s), so a failed FIND walk that crosses position q in state s
   shows that no match starts at q (the chain skips it; ugrep_amd/csrc/
   tables.hpp dom).  *n = the number of u32 words (0: not computed, no skips);
   *all (may be NULL) = 1 when every non-accepting state reachable from the
   start has its bit (then a failed walk skips up to the byte it died on).
   (Replaces the reference's position-by-position restart after a failed
   match, lib/matcher.cpp:692-713, for the stitching re-walks.) */
int ugpu_tables_dom_host(const uint32_t *opc, uint32_t nop, uint32_t *dom, uint32_t dom_cap, uint32_t *n, int *all);

/* Host-only: the per-context accept indices of the dense tables (states * 4
   u32: acap[state * 4 + bol * 2 + eol], state numbering as
   ugpu_tables_build_host), whether the table has line anchors, and whether its
   start state accepts in some context (empty matches). */
int ugpu_tables_context_host(const uint32_t *opc, uint32_t nop, uint32_t *acap, uint32_t acap_cap, int *anchored,
                             int *start_acc);

/* Host-only: *eq = 1 when two opcode tables accept the same strings with the
   same accept indices (so their FIND chains agree on every input).  The
   engine uses it to recognise \w+ under option W. */
int ugpu_tables_equivalent_host(const uint32_t *opc_a, uint32_t nop_a, const uint32_t *opc_b, uint32_t nop_b, int *eq);

/* --- whole-buffer FIND (Matcher::buffer(); while (find()) ...) --- */

/* buf may be host or device memory, len bytes, search starts at `start`
   (the matcher's cur_).  Synchronous.  mode: UGPU_MODE_COUNT or _OFFSETS. */
int ugpu_find_all(const ugpu_dfa *dfa, const uint8_t *buf, uint64_t len, uint64_t start, uint32_t mode,
                  ugpu_result **out);
int ugpu_result_free(ugpu_result *res);

/* Records for a consumer that pops them one at a time (the drop-in matcher's
   find() loop, lib/matcher.cpp:42-750 returning one match per call), at the
   rate PCIe moves the input: a host buffer goes H2D in chunks
   (UGPU_REC_CHUNK, default 64 MiB) on a copy thread, each chunk is scanned
   from the true chain entry as soon as it (and a 1 MiB halo) is resident, its
   records are packed to 6 B (8 B when the table has several accept indices)
   and copied asynchronously into pinned host memory, so input copy, scans and
   record copy overlap.  ugpu_find_records returns once the last input byte is
   on the device (a host buffer may then go away); scans and record copies go
   on behind the consumer on a pipeline thread.  ugpu_records_next pops the
   records in chain order, waiting for the pipeline where needed (1 = a record,
   0 = none left, -code on a pipeline error, after which the consumer may go on
   from the last record's end on the CPU: FIND chains agree there; start, len
   and cap must not be NULL); ugpu_records_totals waits for the end and equals
   ugpu_find_all's totals.  A device buffer must stay valid until
   ugpu_records_free, which waits for the pipeline. */
typedef struct ugpu_records ugpu_records;
int ugpu_find_records(const ugpu_dfa *dfa, const uint8_t *buf, uint64_t len, uint64_t start, ugpu_records **out);
/* ugpu_find_records with flags.  UGPU_REC_BORROW: the caller keeps buf
   readable until ugpu_records_free returns (which stops and joins the
   pipeline), so the call returns at once and the first records can be popped
   while the rest of the input is still crossing PCIe.  Plain
   ugpu_find_records returns only once the last input byte is on the device
   (ugrep may unmap a file as soon as it stops asking for matches). */
#define UGPU_REC_BORROW 1u
int ugpu_find_records_ex(const ugpu_dfa *dfa, const uint8_t *buf, uint64_t len, uint64_t start, uint32_t flags,
                         ugpu_records **out);
int ugpu_records_next(ugpu_records *r, uint64_t *start, uint32_t *len, uint32_t *cap);
int ugpu_records_totals(ugpu_records *r, uint64_t *count, uint64_t *digest, uint64_t *dcap);
/* Pop every remaining record, returning their number and digests (what a
   native consumer's loop costs; tests and benchmarks). */
int ugpu_records_drain(ugpu_records *r, uint64_t *n, uint64_t *digest, uint64_t *dcap);
int ugpu_records_free(ugpu_records *r);

/* Multi-device FIND (the reference has no counterpart: one
   buffer is always scanned by one thread, src/ugrep.cpp:4118-4480).  One
   process drives the devices: [start, len) is cut into `ndev` contiguous
   shards at arbitrary byte offsets; shard k runs on device k mod
   hipGetDeviceCount() (so ndev may exceed the devices: virtual shards share a
   card), each with its own table copy, its own input copy (host buffers: H2D
   over that device's PCIe link; a device buffer: a peer copy over xGMI for
   the shards on other devices) plus a 1 MiB halo, and its own stream.  The
   shards' FIND chains are then resolved left to right on the host
   (ugpu_chain_fix on the owning device when a chain enters a shard elsewhere
   than at its start), and OFFSETS records are copied straight from each
   device into their slice of the result.  Same result as ugpu_find_all.
   Each shard's copy starts 4 bytes before it (the code point at_wb reads for
   option W, the byte at_bol reads for line anchors).  ndev <= 0: one shard per
   device. */
int ugpu_find_all_multi(const ugpu_dfa *dfa, const uint8_t *buf, uint64_t len, uint64_t start, uint32_t mode,
                        int ndev, ugpu_result **out);

/* --- device-resident scanning (benchmarks, multi-GPU shards) --- */

/* Workspace for scans of device buffers on the current device. */
int ugpu_scanner_create(const ugpu_dfa *dfa, ugpu_scanner **out);
/* UGPU_SCANNER_RECORDS: the scans will be followed by ugpu_scan_offsets --
   prefer kernels with their own record-writing pass (code-point run tables
   take xc_kernel's U mode instead of xg_kernel, whose OFFSETS are rebuilt on
   dense_kernel).  Results never depend on it. */
#define UGPU_SCANNER_RECORDS 1u
int ugpu_scanner_create_ex(const ugpu_dfa *dfa, uint32_t flags, ugpu_scanner **out);
int ugpu_scanner_destroy(ugpu_scanner *sc);

/* Enqueue a COUNT scan of dbuf[lo..hi) on `stream` (hipStream_t, NULL = default).
   Walks may read up to read_end; at_eof says read_end is the end of the whole
   stream.  Reported starts are offset by `bias` (global shard offset).
   Asynchronous: results are read with ugpu_scan_totals. */
int ugpu_scan(ugpu_scanner *sc, const uint8_t *dbuf, uint64_t lo, uint64_t hi, uint64_t read_end, int at_eof,
              uint64_t bias, void *stream);
/* Context of the scanner's next scans: bol0 != 0 when dbuf[0] begins a line
   (it is the first byte of the input, or the byte before it is '\n'); the
   default is 1.  Only line-anchored tables read it, for a walk at dbuf[0];
   walks after dbuf[0] read the byte before them (the library's own shards and
   streams keep 4 bytes before their range in dbuf instead). */
int ugpu_scanner_context(ugpu_scanner *sc, int bol0);
/* Synchronize the scanner's stream and return the totals of the last scan. */
int ugpu_scan_totals(ugpu_scanner *sc, ugpu_totals *out);
/* After ugpu_scan + ugpu_scan_totals: write the match records of the last scan
   into device arrays (capacity entries each) on `stream`.  d_cap may be NULL
   for a table with one accept index (ugpu_dfa_info.accepting states all take
   the same index; the records are then 12 bytes: start, len) -- the accept
   index of every record is that index; UGPU_INVAL for other tables. */
int ugpu_scan_offsets(ugpu_scanner *sc, uint64_t *d_start, uint32_t *d_len, uint32_t *d_cap, uint64_t capacity,
                      void *stream);
/* Shard-boundary stitch: the scan of [lo,hi) assumed the chain entered at
   old_entry; the true chain enters at new_entry.  Returns the correction to add
   to the totals and the (possibly changed) exit.  Synchronous. */
int ugpu_chain_fix(ugpu_scanner *sc, const uint8_t *dbuf, uint64_t lo, uint64_t hi, uint64_t read_end, int at_eof,
                   uint64_t bias, uint64_t old_entry, uint64_t new_entry, ugpu_totals *delta, void *stream);
/* Single-pass OFFSETS: with on != 0, COUNT scans of prefiltered tables also
   stage each wave's records, and ugpu_scan_offsets copies them to the output
   (plus a WRITE pass over the waves whose speculative chain was not the true
   one) instead of re-running the scan.  ugpu_find_all in OFFSETS mode does
   this by itself.  Costs 16 B of staging per record (128 MiB per scanner). */
int ugpu_scanner_stage(ugpu_scanner *sc, int on);
/* Time (ms) of the scan kernel of the last ugpu_scan, measured with HIP events
   recorded on the scan stream around that launch. */
int ugpu_scan_kernel_ms(ugpu_scanner *sc, float *ms);

/* --- streaming FIND ---
   Input fed in chunks (what AbstractMatcher::input() + grow()/peek_more()
   provide to Matcher::match, absmatcher.h:1417-1536, :1582-1593; ugrep streams
   stdin, decompressed data and files it does not mmap, src/ugrep.cpp:3936-3944).
   Each ugpu_stream_feed() scans the unsettled tail of the previous chunks plus
   the new chunk on the device and returns the matches that are final: the
   FIND chain is settled up to a point `keep` bytes before the end (or the end
   when `final`), the rest is carried to the next call.  Offsets are absolute
   (from the first byte ever fed); a match may span any number of chunks.  The
   concatenation of all results equals ugpu_find_all over the whole input
   (also for option W and line anchors: the carry keeps the 4 bytes before the
   settled position, the code point at_wb and the byte at_bol read). */
typedef struct ugpu_stream ugpu_stream;

/* keep: bytes held back from each non-final scan (a match that is still open
   that close to the end is re-scanned with the next chunk; 0 = 64 KiB). */
int ugpu_stream_create(const ugpu_dfa *dfa, uint64_t keep, ugpu_stream **out);
int ugpu_stream_destroy(ugpu_stream *st);

/* Feed host bytes; *out (free with ugpu_result_free) gets the newly final
   matches (records in OFFSETS mode) and their count/digest/dcap.
   final: 1 = the input ends with this chunk; UGPU_FEED_FLUSH = more input may
   follow, but settle every match the bytes so far decide (the input would
   block: a slow pipe or a TTY, whose reference matcher reports those matches
   before it waits, include/reflex/input.h:716-731); 0 = hold back `keep`. */
#define UGPU_FEED_FLUSH 2
int ugpu_stream_feed(ugpu_stream *st, const uint8_t *chunk, uint64_t len, int final, uint32_t mode,
                     ugpu_result **out);

/* Absolute offset up to which the FIND chain is settled (bytes before it will
   not be scanned again). */
uint64_t ugpu_stream_settled(const ugpu_stream *st);

/* Pre-create, on the calling thread's device, the pooled resources of `n`
   streams on this table whose feeds hold up to feed_bytes (scanners, device
   buffers and match lists, a private queue and a pinned block each), so that
   the streams created later allocate nothing (ugrep's workers otherwise make
   these device allocations all at once, and they serialise).  Optional: a
   stream without reserved resources creates them itself. */
int ugpu_stream_reserve(const ugpu_dfa *dfa, int n, uint64_t feed_bytes);

/* --- line-level consumers ---
   For a device-resident buffer (16-byte aligned; the kernels load whole
   16-byte granules, so the last granule is read up to its end and the bytes
   past len are ignored) and its sorted match starts
   (e.g. from ugpu_scan_offsets): *newlines = number of '\n' bytes in [0, len)
   (simd nlcount, lib/simd.cpp:62-166), d_line[i] = 1-based line of
   d_start[i] (AbstractMatcher::lineno(), absmatcher.h:695-766; d_line may be
   NULL), *matching_lines = number of distinct lines holding a match start
   (ugrep -c with skip('\n') after each hit, src/ugrep.cpp:10567-10586; equal
   to ugrep -c whenever matches cannot contain '\n').  Synchronous. */
int ugpu_lines(const uint8_t *dbuf, uint64_t len, const uint64_t *d_start, uint64_t n, uint64_t *d_line,
               uint64_t *newlines, uint64_t *matching_lines, void *stream);

/* --- binary-file detection ---
   Device buffers of any alignment (the kernel reads the enclosing 16-byte
   granules).  Synchronous. */

/* reflex::isutf8(s, s + len) (lib/simd.cpp:169-421): *first_bad = UINT64_MAX
   when the bytes are valid UTF-8 without NUL (as the reference defines it:
   surrogates and 3/4-byte overlongs pass), else the offset of the first byte
   that fails (len for a sequence cut off by the end). */
int ugpu_check_utf8(const uint8_t *dbuf, uint64_t len, uint64_t *first_bad, void *stream);

/* memchr(s, '\0', len): *pos = offset of the first NUL or UINT64_MAX. */
int ugpu_find_nul(const uint8_t *dbuf, uint64_t len, uint64_t *pos, void *stream);

/* ugrep's is_binary(s, n) (src/ugrep.cpp:699-711) and, with
   UGPU_BIN_INIT_WINDOW, GrepWorker::init_is_binary() (:3998-4015) over a
   window of len bytes (a trailing UTF-8 sequence is not judged).
   flags: UGPU_BIN_NULL_DATA = --null-data (never binary by content);
   UGPU_BIN_NUL_ONLY = -a/-U without -W (binary iff it holds a NUL);
   otherwise binary iff not isutf8. */
#define UGPU_BIN_NULL_DATA 1u
#define UGPU_BIN_NUL_ONLY 2u
#define UGPU_BIN_INIT_WINDOW 4u
int ugpu_is_binary(const uint8_t *dbuf, uint64_t len, uint32_t flags, int *binary, void *stream);

/* --- synthetic corpora, generated on device --- */
#define UGPU_GEN_WORDS 1
#define UGPU_GEN_PLANTED 2
#define UGPU_GEN_CODE 3
#define UGPU_GEN_UTF8 4
/* Write bytes [off, off+len) of corpus `kind` with `seed` into dbuf. */
int ugpu_gen(int kind, uint64_t seed, uint64_t off, uint8_t *dbuf, uint64_t len, void *stream);

/* --- regex -> opcode words (replaces Matcher::convert + Pattern(conv, "r"),
   lib/convert.cpp and lib/pattern.cpp:171-3063, for FIND tables) ---

   Compiles `regex` (len bytes, ugrep's default ERE syntax in Unicode mode with
   notnewline, src/ugrep.cpp:8574-8578) into opcode words in the reference's
   format (include/reflex/pattern.h:1155-1247), language-equivalent per accept
   index to the reference's Pattern; feed them to ugpu_dfa_create().  *opc is
   malloc'd, free it with ugpu_opc_free().  Returns UGPU_INVAL on a syntax error
   (the reference throws regex_error, lib/pattern.cpp:162-169) and
   UGPU_UNSUPPORTED for constructs the GPU tables do not cover (anchors, word
   boundaries, lazy quantifiers, lookaround, rare \p{..} scripts, \p{Lu} under -i); the
   message is in ugpu_compile_error(). */
#define UGPU_RX_FIXED 1u /* -F: the pattern is a literal string (src/cnf.hpp:147-165) */
#define UGPU_RX_ICASE 2u /* -i: ASCII letters and the reference's Unicode case pairs */
/* The regex a reflex::Pattern holds (its public Pattern::operator[](0),
   include/reflex/pattern.h:302): RE/flex syntax over bytes as produced by
   Matcher::convert (lib/convert.cpp) -- Unicode classes, '.' and -i over
   non-ASCII letters already expanded into byte sequences; inline (?i) (?s) (?m)
   modifiers and (?i:...) scopes; \Q...\E.  The drop-in adapter builds its tables
   from this, so it needs no access to Pattern's private opcode words. */
#define UGPU_RX_REFLEX 4u
int ugpu_compile(const char *regex, size_t len, uint32_t flags, uint32_t **opc, uint32_t *nop);
void ugpu_opc_free(uint32_t *opc);
const char *ugpu_compile_error(void);

const char *ugpu_last_error(void);
const char *ugpu_version(void);
/* Provenance of the device library: "src:<hash of ugrep_amd/csrc and this
   header (tools/srchash.py)> git:<commit it was built at>".  The Python
   binding warns when the hash differs from the sources beside the library. */
const char *ugpu_build_id(void);
/* UGPU_ABI_VERSION of the header the library was built with */
int ugpu_abi_version(void);

/* Devices (no reference counterpart: its matchers are CPU threads).
   ugpu_select_device makes `dev` the calling thread's device (hipSetDevice):
   ugpu_find_all, ugpu_stream_create and scanners created afterwards on this
   thread run there, with the table copy a ugpu_dfa keeps per device (uploaded
   at the first use).  The drop-in adapter spreads ugrep's worker matchers over
   the devices this way. */
int ugpu_device_count(int *n);
int ugpu_select_device(int dev);
/* Initialise device dev for this process ahead of its first scan: the HIP
   context, a scan and a records workspace (streams), a pinned block, the
   kernels' code object -- the ~0.2-0.4 s a fresh process pays at its first
   GPU call (tools/probe/startup_probe.cpp).  The drop-in matcher runs it on a
   thread of its own while the CPU matcher serves the first inputs. */
int ugpu_warmup(int dev);

#ifdef __cplusplus
}
#endif

#endif /* UGPU_H */
