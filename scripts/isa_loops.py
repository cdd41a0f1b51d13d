"""Per-loop instruction counts of one kernel in an ISA dump (make isa): which loop nest
each scratch / VALU / LDS / global instruction sits in (the compiler's loop comments).
  python scripts/isa_loops.py build/wgt_pool.s <kernel-symbol-substring>"""
import re
import sys
from collections import defaultdict

s = open(sys.argv[1]).read()
key = sys.argv[2]
names = [m.group(1) for m in re.finditer(r"^(\S+):\s*;\s*@\1", s, re.M) if key in m.group(1)]
name = names[0]
i = s.find(name + ":")
j = s.find(".Lfunc_end", i)
body = s[i:j].splitlines()
cur = ("entry", 0)
cnt = defaultdict(lambda: defaultdict(int))
for ln in body:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)", ln)
    if m:
        c = m.group(2)
        h = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", c)
        h2 = re.search(r"This Loop Header: Depth=(\d+)", c)
        lbl = m.group(1).replace(".LBB", "BB")
        if h2:
            cur = (lbl, int(h2.group(1)))
        elif h:
            cur = ("BB" + h.group(1), int(h.group(2)))
        else:
            cur = ("top", 0)
        continue
    t = ln.strip().split()
    if not t or t[0].startswith((".", ";")):
        continue
    op = t[0]
    d = cnt[cur]
    d["all"] += 1
    for p, k in (("scratch_", "scratch"), ("v_", "valu"), ("s_", "salu"), ("ds_", "lds"), ("global_", "global"),
                 ("v_readlane", "readlane"), ("v_writelane", "writelane")):
        if op.startswith(p):
            d[k] += 1
print(name)
for k in sorted(cnt, key=lambda x: (x[1], x[0])):
    print(k, dict(cnt[k]))
