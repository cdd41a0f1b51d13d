"""Print an A/B log (scripts/ab_run.sh) as a table: python scripts/ab_table.py gpurun_out/<tag>/ab.log"""
import json
import sys

name = None
for line in open(sys.argv[1]):
    line = line.strip()
    if " {" in line and not line.startswith("{"):
        name, line = line.split(" {", 1)[0], "{" + line.split(" {", 1)[1]
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "ms" not in d:
        continue
    print(f"{name:34s} ms={d['ms']:7.2f} Mrays/s={d['Mrays_s']:7.1f} trav_cyc/step={d['trav_cyc_per_step']:7.1f} "
          f"svc_cyc/iter={d['svc_cyc_per_iter']:8.1f} steps={d['wave_steps']:>11,} nodes={d['nodes']:>13,} "
          f"util={d['trav_util']} same={d['identical']}")
