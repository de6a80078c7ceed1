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

namespace ugpu {

enum TableFormat : uint32_t { FMT_BYTE = 0, FMT_CLASS = 1 };

struct DfaTables {
  uint32_t format = FMT_BYTE;
  uint32_t states = 0;   // including dead state 0
  uint32_t classes = 0;  // distinct byte columns
  uint32_t row = 256;    // R: 256 (FMT_BYTE) or pow2 >= classes (FMT_CLASS)
  uint32_t log_row = 8;
  uint32_t start = 0;    // start entry = start_sid * R
  uint32_t accb = 0;     // first accepting entry (A * R)
  uint32_t accepting = 0;
  // Candidate prefilter (replaces the reference's needle/pin prefilters,
  // lib/matcher_avx2.cpp:303-799): a position p can start a match only if
  //   B[p] in A  (1-byte match possible)  or  B[p] in B and B[p+1] in C.
  // Each set is an exact cover by (mask, value) terms: b matches a term iff
  // (b & mask) == value.  filter == false: no prefilter (dense patterns).
  bool filter = false;
  uint32_t nA = 0, nB = 0, nC = 0;  // nC == 0: no second-byte test
  uint8_t tm[12] = {}, tv[12] = {};  // terms: A at [0,nA), B at [4,4+nB), C at [8,8+nC)
  uint32_t first_bytes = 0;
  std::vector<uint16_t> trans;  // states * row
  std::vector<uint8_t> cls;     // 256
  std::vector<uint32_t> caps;   // states
};

// Returns 0 (UGPU_OK), 1 (UNSUPPORTED) or 2 (INVAL); err gets a message.
int build_tables(const uint32_t* opc, uint32_t nop, DfaTables& out, std::string& err);

}  // namespace ugpu
