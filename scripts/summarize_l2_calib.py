"""profiles/l2_calibration.json from scripts/gpu_l2_calib.sh's PMC pass: L2 (TCC)
requests per byte for kernels that read a known number of bytes once.
  python scripts/summarize_l2_calib.py gpurun_out/<tag>"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(os.path.join(src, "pmc", "run_counter_collection.csv"))):
    agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"]
SUM_BYTES, GATHER_BYTES = (1 << 28) * 4, (1 << 24) * 16
rows = []
for d, c in sorted(agg.items(), key=lambda kv: int(kv[0])):
    n = names[d]
    kind = "stream" if "reduce_kernel" in n else ("gather" if "gather_kernel" in n else None)
    if kind is None:
        continue
    req = c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)
    byts = SUM_BYTES if kind == "stream" else GATHER_BYTES
    rows.append({"kind": kind, "kernel": n[:80], "tcc_hit_plus_miss": req, "tcc_req": c.get("TCC_REQ_sum"),
                 "bytes_read": byts, "bytes_per_request": round(byts / req, 2) if req else None})
stream = [r["bytes_per_request"] for r in rows if r["kind"] == "stream" and r["bytes_per_request"]]
gather = [r["bytes_per_request"] for r in rows if r["kind"] == "gather" and r["bytes_per_request"]]
out = {"bytes_per_request": round(sorted(stream)[len(stream) // 2], 2) if stream else None,
       "gather_bytes_per_request": round(sorted(gather)[len(gather) // 2], 2) if gather else None,
       "note": "bytes_per_request: a coalesced 16-B-per-lane float4 stream read once (torch sum of 1 GiB); "
               "its requests carry that many useful bytes each, the figure bench.py prices TCC_HIT+TCC_MISS "
               "with against the ~34.5 TB/s L2 peak. gather_bytes_per_request: random 16-B granules, one per "
               "lane (the traversal's divergent node-load shape): useful bytes per request there.",
       "source": f"scripts/gpu_l2_calib.sh -> {os.path.relpath(src, ROOT)}", "dispatches": rows}
json.dump(out, open(os.path.join(ROOT, "profiles", "l2_calibration.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
