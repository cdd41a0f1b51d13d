"""Summarise scripts/ab_run.sh logs: per (library, scene) the kernel ms of every round,
their median, and the change against the first library.  python scripts/ab_table.py LOG"""
import json
import statistics
import sys
from collections import defaultdict

times = defaultdict(list)
head = None
for line in open(sys.argv[1]):
    line = line.strip()
    if line.endswith(".so") or ".so r" in line:
        parts = line.split()
        head = (parts[0], " ".join(parts[2:6]))
    if line.startswith('{"WGT_KERNEL') and head:
        times[head].append(json.loads(line)["ms"])
libs = list(dict.fromkeys(k[0] for k in times))
scenes = list(dict.fromkeys(k[1] for k in times))
for sc in scenes:
    base = statistics.median(times[(libs[0], sc)])
    for lib in libs:
        t = times[(lib, sc)]
        med = statistics.median(t)
        print(f"{sc:24s} {lib:14s} med {med:8.2f} ms  {100 * (med / base - 1):+6.2f}%  runs {t}")
