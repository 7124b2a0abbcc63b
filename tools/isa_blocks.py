"""Per-basic-block instruction mix of one kernel in a hipcc -S listing, with
the loop back-edges: python tools/isa_blocks.py file.s <kernel-substring>.
VALU = v_* (minus v_readlane/v_writelane which are counted apart), SALU = s_*
(minus branches/waits), LDS = ds_*, VMEM = global_/buffer_/flat_."""
import re
import sys

path, key = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + key + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or
           re.match(r"^\.Lfunc_end", lines[i]))
blocks, cur = [], None
for i in range(start, end):
    l = lines[i]
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m or cur is None:
        cur = {"name": m.group(1) if m else "entry", "line": i + 1, "ins": []}
        blocks.append(cur)
        if m:
            continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    cur["ins"].append(t.split()[0])
pos = {b["name"]: k for k, b in enumerate(blocks)}
for k, b in enumerate(blocks):
    ins = b["ins"]
    valu = sum(1 for x in ins if x.startswith("v_") and not x.startswith(("v_readlane", "v_writelane", "v_readfirstlane")))
    rl = sum(1 for x in ins if x.startswith(("v_readlane", "v_readfirstlane", "v_writelane")))
    salu = sum(1 for x in ins if x.startswith("s_") and not x.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop")))
    lds = sum(1 for x in ins if x.startswith("ds_"))
    vmem = sum(1 for x in ins if x.startswith(("global_", "buffer_", "flat_")))
    wait = sum(1 for x in ins if x.startswith("s_waitcnt"))
    back = []
    for i in range(b["line"], b["line"] + 100000):
        pass
    print(f"{b['name']:>14} L{b['line']:<6} n={len(ins):4d} valu={valu:4d} rl={rl:3d} salu={salu:3d} lds={lds:3d} vmem={vmem:3d} wait={wait:3d}")
# back-edges
for k, b in enumerate(blocks):
    for i in range(b["line"], (blocks[k + 1]["line"] if k + 1 < len(blocks) else end)):
        m = re.search(r"s_c?branch\S*\s+(\.LBB\d+_\d+)", lines[i])
        if m and m.group(1) in pos and pos[m.group(1)] <= k:
            print(f"loop: {blocks[pos[m.group(1)]]['name']} .. {b['name']}")
