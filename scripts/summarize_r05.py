"""profiles/r05_<tag>_summary.md from a gpurun_out/<tag> directory of scripts/gpu_r05_final.sh: the
driver-command bench line (live PMC fields), the rocprofv3 kernel-trace statistics of the same
command, the per-dispatch durations and completion intervals of the main kernel, the C3 line, the
node-form A/B (80-B, 64-B, wide) and the two-rank rehearsal line."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", tag)
dst = os.path.join(ROOT, "profiles")


def last_json(name):
    lines = [ln for ln in open(os.path.join(src, name)).read().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


b = last_json("bench20.log")
kt = last_json("bench20_kt.log")
shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, f"r05_{tag}_kernel_stats.csv"))
out = [f"# r05 profile `{tag}` — {b['config']['workload']}, build {b['build_id']}", "",
       "The driver's command (`python bench.py --gpus 1 --steps 20 --warmup 5`), live PMC passes and the CPU "
       "baseline included:", "", "```json", json.dumps(b, indent=1), "```", "",
       "rocprofv3 --kernel-trace --stats of the same command (`--pmc off --no-cpu-baseline`; its line: "
       f"{kt['value']} Mrays/s, {kt['kernel_ms']} ms per launch):", "", "| kernel | calls | avg ms | total ms |",
       "|---|---|---|---|"]
for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))):
    if "wgt::" in r["Name"]:
        out.append(f"| `{r['Name'].split('(')[0].replace('void ', '')}` | {r['Calls']} | "
                   f"{float(r['AverageNs']) / 1e6:.3f} | {float(r['TotalDurationNs']) / 1e6:.1f} |")
rows = [r for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv")))
        if r["Kernel_Name"].split("(")[0].replace("void ", "").strip() == kt["per_launch"]["kernel"]]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
ends = sorted(int(r["End_Timestamp"]) for r in rows)
iv = [(b2 - a) / 1e6 for a, b2 in zip(ends, ends[1:])]
out += ["", f"`{kt['per_launch']['kernel']}`: {len(rows)} dispatches (warm-up, 20 timed, the isolated one, "
        "the instrumented passes excluded by name); dispatch begin-to-end ms "
        f"{[round(x, 1) for x in durs]}; intervals between consecutive completions ms {[round(x, 1) for x in iv]}"]
timed = iv[5:25] if len(iv) >= 25 else iv
if timed:
    out.append(f"median completion interval of the timed region: {sorted(timed)[len(timed) // 2]:.2f} ms "
               f"(bench kernel_ms {kt['kernel_ms']})")
bb = last_json("bench_bunny.log")
out += ["", "C3 (bunny stand-in 1080p/256 spp, 30 steps):", "", "```json", json.dumps(
    {k: bb[k] for k in ("value", "kernel_ms", "timing", "simt_utilisation")} | {"roofline": {
        k: bb["roofline"][k] for k in ("bound", "frac", "hbm_frac", "valu_busy", "wave_split", "traffic")}},
    indent=1), "```", "", "Node forms A/B (same box, the driver's command, two rounds):", ""]
out += ["| WGT_CNODE | round | Mrays/s | ms per launch | alone ms | node visits / ray | triangle tests / ray |",
        "|---|---|---|---|---|---|---|"]
for r in (1, 2):
    for c in (2, 3, 4):
        name = f"bench20_c{c}_{r}.log"
        if not os.path.exists(os.path.join(src, name)):
            continue
        d = last_json(name)
        p = d["per_launch"]
        out.append(f"| {c} ({p['bvh_nodes']}) | {r} | {d['value']} | {d['kernel_ms']} | "
                   f"{d['timing']['isolated_launch_ms']} | {p['node_visits'] / p['traced_rays']:.3f} | "
                   f"{p['tri_tests'] / p['traced_rays']:.3f} |")
n2 = last_json("bench_n2.log")
out += ["", "Two ranks on cuda:0 over gloo (`torch.distributed.run --nproc-per-node 2 bench.py --gpus 2 "
        "--dist-backend gloo`, 960x540/64 spp, 3 steps):", "", "```json",
        json.dumps({k: n2[k] for k in ("value", "n_gpus", "check_frames_bit_exact", "per_rank", "kernel_ms")},
                   indent=1), "```"]
open(os.path.join(dst, f"r05_{tag}_summary.md"), "w").write("\n".join(out) + "\n")
print("\n".join(out[-40:]))
