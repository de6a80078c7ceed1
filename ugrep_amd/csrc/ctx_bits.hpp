// ctx_bits.hpp -- context bits of the per-context accept tables of
// word-boundary patterns (tables.hpp acap, device_common.hpp ctx_accept).
// Of the position q: eol (the byte at q is '\n', EOF, or '\r' before '\n'),
// ew (at_ew: the character before q is a word character), we (at_we as the
// meta edges call it, pos_ one past the byte at q); of the walk start p: bol,
// wb (at_wb: no word character before p), bw (at_bw: a word character at p)
// -- include/reflex/matcher.h:1194-1319.
#pragma once
#include <cstdint>

namespace ugpu {
enum : uint32_t { CTX_EOL = 1, CTX_EW = 2, CTX_WE = 4, CTX_BOL = 8, CTX_WB = 16, CTX_BW = 32 };

// The accept index (tables.hpp caps) of a REDO state: a negative pattern's
// accept (ugrep -N makes '(?^...)', src/ugrep.cpp:6487; lib/pattern.cpp:
// 2945-2947 emits REDO for it).  Walks take it like a TAKE (the last accept
// wins, lib/matcher.cpp:151-156, :218-225); a match ending in it is not
// reported and the FIND chain resumes at its end (:732-738).  No TAKE index
// has more than 24 bits, so it never collides.
constexpr uint32_t kCapRedo = 0xFFFFFFFFu;
}
