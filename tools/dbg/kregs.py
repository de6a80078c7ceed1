"""Per-kernel VGPR count and scratch bytes from a hipcc -S file (amdhsa metadata)."""
import re, sys
txt = open(sys.argv[1]).read()
for blk in re.split(r"\n\s+- \.agpr_count", txt)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    pr = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
    vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
    sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
    if name:
        print("%-60s vgpr %s scratch %s spill %s" % (name.group(1)[:60], vg and vg.group(1), pr and pr.group(1), sp and sp.group(1)))
