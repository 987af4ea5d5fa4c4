#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# SQ counter passes over a short bench run (k_step / k_scan instruction mix and waits).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-pmcs}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 5 -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o run \
      -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done

python3 - "$TAG" <<'PY'
import csv, glob, collections, sys
tag = sys.argv[1]
for p in ("%s_p1" % tag, "%s_p2" % tag):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob("gpurun_out/%s/**/*counter_collection.csv" % p, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-14:]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        if "k_step" in k or "k_scan" in k:
            print(p, k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
