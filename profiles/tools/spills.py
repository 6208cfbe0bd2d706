"""Where a kernel's scratch spills/reloads sit: loop depth and block label of every scratch_*
instruction (python3 profiles/tools/spills.py file.s kernel-substring)."""
import re
import sys

txt = open(sys.argv[1]).read()
for m in re.finditer(r"^(_Z\S+):\s*;", txt, re.M):
    if sys.argv[2] not in m.group(1):
        continue
    body = txt[m.end():txt.index(".Lfunc_end", m.end())].split("\n")
    depth, cur = 0, ""
    for l in body:
        if re.match(r"^(\.LBB\S+|; %bb\.\d+):", l):
            cur = l.split(":")[0]
            d = re.search(r"Depth=(\d+)", l)
            depth = int(d.group(1)) if d else 0
        if "scratch_" in l:
            print(depth, cur, l.strip().split(";")[0])
