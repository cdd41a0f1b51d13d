"""Per-kernel PMC totals of rocprofv3 output directories (run_counter_collection.csv), with the
kernel-trace duration: prints one line per (directory, wgt kernel).
  python scripts/summarize_pmc_dirs.py gpurun_out/pmc1/p*_[AB]"""
import collections
import csv
import os
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "wgt::" not in k or "lpt" in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(float)
    kt = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(kt):
        for r in csv.DictReader(open(kt)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for k, v in agg.items():
        if "true, true" in k and "k_render_ps<false, true" in k:
            continue
        extra = ""
        if "SQ_WAVE_CYCLES" in v and dur.get(k):
            # SQ_WAVE_CYCLES counts in units of 4 cycles (quad-cycles) per the summaries
            extra = f" waves_in_flight~{v['SQ_WAVE_CYCLES'] * 4 / (dur[k] * 1e-3 * 2.4e9) / 256:.1f}/CU"
            wc = v["SQ_WAVE_CYCLES"]
            extra += f" active {v['SQ_ACTIVE_INST_ANY'] / wc:.2f} wait {v['SQ_WAIT_ANY'] / wc:.2f} " \
                     f"stall {v['SQ_WAIT_INST_ANY'] / wc:.2f}"
        print(os.path.basename(d), k[:60], f"{dur.get(k, 0):.2f} ms",
              " ".join(f"{c}={x:.4g}" for c, x in sorted(v.items())), extra)
