"""Basic blocks of one kernel in a hipcc -S file: per block the counts of VALU,
SALU, LDS, global/buffer loads; loops marked by backward branches.
usage: asm_blocks.py FILE.s KERNEL_SUBSTRING [min_valu]"""
import re, sys
src = open(sys.argv[1]).read().splitlines()
name = sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
start = next(i for i, l in enumerate(src) if l.startswith("_Z") and name in l and l.split(";")[0].strip().endswith(":"))
end = next(i for i in range(start, len(src)) if src[i].strip().startswith("s_endpgm") or ".Lfunc_end" in src[i])
blocks, cur, label = [], [], "entry"
for l in src[start + 1:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        blocks.append((label, cur)); cur, label = [], m.group(1); continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur.append(s.split()[0])
blocks.append((label, cur))
pos = {b[0]: i for i, b in enumerate(blocks)}
for i, (lab, ins) in enumerate(blocks):
    c = dict(valu=sum(x.startswith("v_") for x in ins), salu=sum(x.startswith("s_") for x in ins),
             lds=sum(x.startswith("ds_") for x in ins), vmem=sum(x.startswith(("buffer_", "global_")) for x in ins))
    back = [x for x in ins if x.startswith("s_cbranch") or x == "s_branch"]
    if c["valu"] >= mn:
        ops = {}
        for x in ins:
            if x.startswith("v_"): ops[x] = ops.get(x, 0) + 1
        top = sorted(ops.items(), key=lambda t: -t[1])[:14]
        print(i, lab, c, " ".join("%s:%d" % t for t in top))
