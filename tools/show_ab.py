"""Print the bench lines of a tools/gpu_ab.sh output directory: python tools/show_ab.py gpurun_out/<tag>"""
import json
import os
import sys

d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if not f.endswith(".json"):
        continue
    lines = [ln for ln in open(os.path.join(d, f)).read().splitlines() if ln.startswith("{")]
    if not lines:
        print(f, "(no line)")
        continue
    x = json.loads(lines[-1])
    k = x.get("kernels_us_per_launch", {})
    print("%-18s ms/step %.4f  pair %s step %s scan %s  %s" % (f, x["ms_per_step"], round(k.get("pair", 0), 1),
          round(k.get("step", 0), 1), round(k.get("scan", 0), 1), x.get("engine_events")))
