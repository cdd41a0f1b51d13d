"""Summarise a gpurun_out/<tag> profiling directory (scripts/gpu_profile.sh) into
profiles/<round>_<tag>_*: the rocprofv3 kernel stats CSV, a PMC summary per render
kernel, and profiles/pmc_traffic.json (HBM bytes per launch, read by bench.py).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB;
FETCH_SIZE reads half the bytes of 16-B-per-lane reads on gfx950, so it is doubled.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(dirpath):
    agg = collections.defaultdict(float)
    calls = collections.Counter()
    path = os.path.join(dirpath, "run_counter_collection.csv")
    if not os.path.exists(path):
        return agg, calls
    seen = set()
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "wgt::" not in name:
            continue
        short = name.split("(")[0].replace("void ", "")
        agg[(short, r["Counter_Name"])] += float(r["Counter_Value"])
        key = (short, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            calls[short] += 1
    return agg, calls


def main():
    tag, rnd = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01"
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, f"{rnd}_{tag}_kernel_stats.csv"))
    bench = open(os.path.join(src, "bench.log")).read().strip().splitlines()[-1]
    line = json.loads(bench)
    out = [f"# {rnd} profile `{tag}` — {line['config']['workload']}, build {line.get('build_id')}", "",
           "rocprofv3 --kernel-trace --stats (same bench command, 4 timed steps, 2 frames in flight):", "", "| kernel | calls | avg ms |",
           "|---|---|---|"]
    for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))):
        if "wgt::" in r["Name"]:
            out.append(f"| `{r['Name'].split('(')[0].replace('void ', '')}` | {r['Calls']} | "
                       f"{float(r['AverageNs']) / 1e6:.3f} |")
    # pipelined launches overlap, so a dispatch's begin-to-end also counts the time its waves
    # waited for the CUs the previous frame still held: the per-launch figure to compare with
    # the bench's kernel_ms is the interval between consecutive completions of the main kernel
    kt = os.path.join(src, "kt", "run_kernel_trace.csv")
    if os.path.exists(kt):
        rows = [r for r in csv.DictReader(open(kt)) if "wgt::" in r["Kernel_Name"]]
        main_k = line["per_launch"]["kernel"]
        ends, durs = [], []
        for r in rows:
            if r["Kernel_Name"].split("(")[0].replace("void ", "") == main_k:
                ends.append(int(r["End_Timestamp"]))
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        ends.sort()
        if len(ends) >= 3:
            gaps = [(b - a) / 1e6 for a, b in zip(ends, ends[1:])]
            out += ["", f"kernel trace, `{main_k}` ({len(ends)} launches: warm-up, timed, isolated): dispatch "
                        f"begin-to-end ms {[round(d, 1) for d in durs]}; intervals between consecutive "
                        f"completions ms {[round(g, 1) for g in gaps]}"]
    out += ["", f"bench.py line: value {line['value']} {line['unit']}, kernel_ms {line['kernel_ms']}, "
                f"roofline {json.dumps(line['roofline'])}", "", "PMC (separate passes, 1 timed step each):", "",
            "| kernel | counter | value per launch |", "|---|---|---|"]
    per = {}
    for d in sorted(os.listdir(src)):
        if not d.startswith("pmc_") or not os.path.isdir(os.path.join(src, d)):
            continue
        agg, calls = pmc(os.path.join(src, d))
        for (k, c), v in sorted(agg.items()):
            v /= max(calls[k], 1)
            per[(k, c)] = v
            out.append(f"| `{k}` | {c} | {v:,.1f} |")
    sys.path.insert(0, ROOT)
    timed = line["per_launch"]["kernel"]
    if not any(k == timed for k, _ in per):  # older bench lines name fewer template arguments
        cand = sorted({k for k, _ in per if k.startswith(timed[:-1] + ",")})
        timed = cand[0] if len(cand) == 1 else timed
    fetch = per.get((timed, "FETCH_SIZE"))
    write = per.get((timed, "WRITE_SIZE"))
    if fetch is not None and write is not None:
        hbm = (2.0 * fetch + write) * 1024.0
        hit, miss = per.get((timed, "TCC_HIT_sum"), 0), per.get((timed, "TCC_MISS_sum"), 0)
        out += ["", f"HBM bytes per launch of `{timed}` = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 = {hbm / 1e9:.3f} GB "
                    f"(FETCH doubled per MI355X_MICROARCH.md §HBM); L2 hit rate "
                    f"{hit / max(hit + miss, 1):.4f}."]
        # one entry per workload (bench.py reads the entry of its own workload)
        tpath = os.path.join(dst, "pmc_traffic.json")
        try:
            table = json.load(open(tpath))
        except (OSError, ValueError):
            table = {}
        if "workload" in table:  # the old single-entry format
            table = {table["workload"]: table}
        wl = line["config"]["workload"]
        # the build the counters were measured on (bench.py applies them to that build only)
        table[wl] = {"workload": wl, "n_gpus": 1, "kernel": timed, "build_id": line.get("build_id"),
                     "hbm_bytes_per_launch": hbm, "fetch_size_kib": fetch, "write_size_kib": write,
                     "source": f"profiles/{rnd}_{tag}_summary.md"}
        if hit + miss > 0:  # L2 requests of the timed kernel (bench.py's roofline.l2)
            table[wl]["tcc_requests_per_launch"] = hit + miss
            table[wl]["tcc_hit_rate"] = round(hit / (hit + miss), 4)
        json.dump(table, open(tpath, "w"), indent=1)
    sq = {c: per.get((timed, c)) for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
    if all(v for v in sq.values()):
        wc = sq["SQ_WAVE_CYCLES"]
        out += ["", f"wave-cycle split: active {sq['SQ_ACTIVE_INST_ANY'] / wc:.2f}, waiting (s_waitcnt) "
                    f"{sq['SQ_WAIT_ANY'] / wc:.2f}, issue-stalled {sq['SQ_WAIT_INST_ANY'] / wc:.2f}"]
    open(os.path.join(dst, f"{rnd}_{tag}_summary.md"), "w").write("\n".join(out) + "\n")
    shutil.copy(os.path.join(src, "bench.log"), os.path.join(dst, f"{rnd}_{tag}_bench.log"))
    print("\n".join(out))


if __name__ == "__main__":
    main()
