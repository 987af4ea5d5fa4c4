#!/bin/bash
# Diagnostic PMC passes over the c3 bench (k_step instruction-fetch behaviour), one pass per block set.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmcic; mkdir -p $O
timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $O/a -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/a.log 2>&1 || exit $?
timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $O/b -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for p in ("a", "b"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob("gpurun_out/pmcic/%s/**/*counter_collection.csv" % p, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-12:]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        if "k_step" in k or "k_scan" in k:
            print(p, k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
