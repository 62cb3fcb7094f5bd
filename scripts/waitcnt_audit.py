"""Wait-count audit of the compiled kernels: per kernel, the `s_waitcnt vmcnt(0)` instructions inside loop blocks
(a full wait inside a loop usually means a conditional load left the compiler unable to count the younger loads).
usage: python scripts/waitcnt_audit.py FILE.s [FILTER]"""
import re
import sys

src = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\n(_Z\S+):\s*;\s*@", src):
    name = m.group(1)
    if flt not in name:
        continue
    end = src.find(".Lfunc_end", m.end())
    body = src[m.end():end].split("\n")
    in_loop, hits, total = False, 0, 0
    for ln in body:
        t = ln.strip()
        if t.startswith(".LBB"):
            in_loop = "Loop" in t
        elif t.startswith("s_waitcnt") and "vmcnt(0)" in t:
            total += 1
            hits += in_loop
    if hits:
        print(f"{hits:3d} in-loop / {total:3d} vmcnt(0)  {name[:150]}")
