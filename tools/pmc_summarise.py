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


def kernel_key(name):
    """k_scan = the full-scan instantiations (k_scan<RC, LSETS, false, GT>); k_scan_bound = the
    block-list instantiation (k_scan<RC, LSETS, true, GT>: the conditional bound passes and the
    incremental mode); k_pair (the fused scan + step launch); k_step; k_ubinit."""
    if "k_scansum" in name:                 # (the sharded scan + rank summary launch)
        return "k_scansum"
    if "k_scan" in name:
        params = name.replace(" ", "").split("<", 1)[-1].split(">")[0].split(",")
        return "k_scan_bound" if len(params) > 2 and params[2] == "true" else "k_scan"
    for k in ("k_pair", "k_step", "k_ubinit", "k_refresh", "k_summary"):
        if k in name:
            return k
    return None


def per_kernel(counter):
    files = glob.glob("gpurun_out/%s_%s/**/*counter_collection.csv" % (tag, counter), recursive=True)
    vals = defaultdict(dict)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = kernel_key(r["Kernel_Name"])
            if k:
                d = int(r["Dispatch_Id"])
                vals[k][d] = vals[k].get(d, 0.0) + float(r["Counter_Value"])
    res = {}
    for k, m in vals.items():
        xs = [m[d] for d in sorted(m)][10:]
        if k == "k_scan" and xs:
            # full scans only: a scan of a step that was already decided (a census-free
            # retry, a halted pair's no-op launch) returns after its first-tile prefetch
            med = sorted(xs)[len(xs) // 2]
            xs = [x for x in xs if x >= 0.5 * med]
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
                 "dispatches after the first 10 (k_scan = the full-scan instantiation, its launches with FETCH >= half "
                 "the median; k_scan_bound = the block-list instantiation of the bound passes); FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half "
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
