"""Fold the two rocprofv3 PMC passes of tools/pmc_bench.sh into profiles/pmc_traffic.json:
per kernel, mean FETCH_SIZE / WRITE_SIZE per dispatch (after the first 10), FETCH_SIZE
doubled as MI355X_MICROARCH.md prescribes for gfx950 16-B streaming reads."""
import csv
import glob
import json
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "pmcb"
out = sys.argv[2] if len(sys.argv) > 2 else None
workload = sys.argv[3] if len(sys.argv) > 3 else "c3"
git_head = sys.argv[4] if len(sys.argv) > 4 else None      # the tree the passes ran on


def per_kernel(counter):
    files = glob.glob("gpurun_out/%s_%s/**/*counter_collection.csv" % (tag, counter), recursive=True)
    vals = defaultdict(dict)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            k = "k_scan" if "k_scan" in name else "k_step" if "k_step" in name else None
            if k:
                d = int(r["Dispatch_Id"])
                vals[k][d] = vals[k].get(d, 0.0) + float(r["Counter_Value"])
    res = {}
    for k, m in vals.items():
        xs = [m[d] for d in sorted(m)][10:]
        if k == "k_scan" and xs:
            # full scans only: the conditional bound passes (ubpass) return after their
            # first-tile prefetch and would drag the mean below one scan's traffic
            top = max(xs)
            xs = [x for x in xs if x >= 0.5 * top]
        res[k] = (sum(xs) / max(len(xs), 1), len(xs))
    return res


fetch, write = per_kernel("FETCH_SIZE"), per_kernel("WRITE_SIZE")
doc = {}
for k in sorted(set(fetch) & set(write)):
    rd = 2 * fetch[k][0] * 1024
    wr = write[k][0] * 1024
    doc[k] = {"FETCH_SIZE_kb_mean": fetch[k][0], "dispatches": fetch[k][1], "WRITE_SIZE_kb_mean": write[k][0],
              "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "traffic_bytes_per_launch": rd + wr}
doc["method"] = ("rocprofv3 --kernel-trace --pmc FETCH_SIZE, then --pmc WRITE_SIZE (separate passes) over "
                 "the bench command of the workload (tools/pmc_bench.sh, tools/gpu_bench_r02.sh); mean over "
                 "dispatches after the first 10 (k_scan: full scans only, FETCH >= half the largest); FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half "
                 "of 16-B/lane streaming reads); KB = 1024 B. k_step's reads are not 16-B streaming, so its "
                 "doubled figure is an upper estimate.")
method = doc.pop("method")
merged = {}
if out:
    try:
        merged = json.load(open(out))
    except (OSError, ValueError):
        merged = {}
if git_head:
    doc["git_head"] = git_head
merged[workload] = doc
merged["method"] = method + " Keyed by bench workload."
s = json.dumps(merged, indent=1)
if out:
    open(out, "w").write(s + "\n")
print(s)
