"""Print per-kernel PMC totals of every p*/ pass under a gpurun_out directory
(scripts/gpu_pmc_mem.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import pmc  # noqa: E402

src = sys.argv[1]
for d in sorted(os.listdir(src)):
    p = os.path.join(src, d)
    if not (d.startswith("p") and os.path.isdir(p)):
        continue
    agg, calls = pmc(p)
    for (k, c), v in sorted(agg.items()):
        print(f"{d} {k} calls={calls[k]} {c} {v / max(calls[k], 1):,.1f}")
