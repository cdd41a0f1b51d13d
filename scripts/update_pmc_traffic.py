"""Write the live PMC figures of a gpurun_out/<tag> run of scripts/gpu_r06_final.sh (earlier: gpu_r04_final.sh, in git history) (bench20.log: the
driver's sponza command; bench_bunny.log: the C3 line) into profiles/pmc_traffic.json, keyed by the
build they were measured on, so that bench.py's profile fallback (--pmc off, N > 1) has them too.
  python scripts/update_pmc_traffic.py TAG"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
table = json.load(open(path))
for log in ("bench20.log", "bench_bunny.log"):
    lines = [ln for ln in open(os.path.join(ROOT, "gpurun_out", tag, log)).read().splitlines() if ln.startswith("{")]
    b = json.loads(lines[-1])
    r = b["roofline"]
    if r.get("traffic_source") != "live":
        print(log, "has no live PMC figures; skipped")
        continue
    table[b["config"]["workload"]] = {
        "build_id": b["build_id"], "kernel": b["per_launch"]["kernel"], "n_gpus": 1,
        "hbm_bytes_per_launch": r["traffic"], "write_bytes_per_launch": r.get("write_bytes_per_launch"),
        "tcc_requests_per_launch": (r.get("l2") or {}).get("requests_per_launch"),
        "tcc_hit_rate": (r.get("l2") or {}).get("hit_rate"),
        "sq": {"valu_busy": r.get("valu_busy"), "wave_split": r.get("wave_split")},
        "source": f"live rocprofv3 --pmc passes in bench.py, gpurun_out/{tag} ({log}), profiles/r04_{tag}_summary.md"}
    print(log, b["config"]["workload"], b["build_id"], r["traffic"])
json.dump(table, open(path, "w"), indent=1)
