"""ugrep_amd -- MI355X-native engine for ugrep's RE/flex DFA buffer-scan hot path.

The C ABI (include/ugpu.h, libugrep_amd.so) is the product boundary; this
package mirrors the reference's Pattern/Matcher FIND interface on top of it and
holds the multi-GPU shard stitching (dist.py).
"""
from ._lib import (GEN_CODE, GEN_PLANTED, GEN_UTF8, GEN_WORDS, MODE_COUNT, MODE_OFFSETS, UgpuError,  # noqa: F401
                   Unsupported, lib)
from .matcher import (compile_regex, Matcher, Pattern, Records, Scanner, Stream, check_utf8, find_all, find_all_multi, find_nul, gen,  # noqa: F401
                      host_plan, host_prefilter, host_tables, host_transducer, is_binary, isutf8, lines)

__all__ = ["compile_regex", "Pattern", "Matcher", "Records", "Scanner", "Stream", "find_all", "find_all_multi", "gen", "host_tables", "host_plan", "host_prefilter", "Unsupported",
           "UgpuError", "lines", "isutf8", "check_utf8", "find_nul", "is_binary"]
