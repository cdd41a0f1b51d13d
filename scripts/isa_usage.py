"""Per-kernel resource usage from `make -C webgputracer_amd isa` remarks (stdin):
name, VGPRs, SGPR spill, scratch bytes/lane, occupancy."""
import re
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("sgpr_spill", r"SGPRs Spill: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    if "k_render_ps" in r["name"] or "k_trace" in r["name"]:
        n = re.sub(r"EEEvNS_8DevScene.*", "", r["name"]).replace("_ZN3wgt11", "")
        print(f"{n:40s} vgpr={r.get('vgpr')} sgpr_spill={r.get('sgpr_spill')} scratch={r.get('scratch')} occ={r.get('occ')}")
