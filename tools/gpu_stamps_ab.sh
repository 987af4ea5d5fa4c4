#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# per-phase k_step stamps (-DKB_STAMPS build) of the fused and the two-launch pair on one
# workload ($WL, default c2): which phase the fused step pays for
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-stab}; mkdir -p $O
WL=${WL:-c2}; ST=${ST:-80}
for f in 1 0; do
  KB_FUSE=$f timeout -k 10 200 python3 -u bench.py --stamps --workload $WL --steps $ST --warmup 10 > $O/st_$f.json 2> $O/st_$f.err || { tail -5 $O/st_$f.err; exit 1; }
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
rows = {f: [json.loads(l) for l in open("%s/st_%s.json" % (O, f)) if l.startswith("{")][0] for f in ("1", "0")}
ks = list(rows["0"]["stamps_us_per_step"])
print("%-18s %8s %8s" % ("phase", "fused", "2-launch"))
for k in ks:
    print("%-18s %8.3f %8.3f" % (k, rows["1"]["stamps_us_per_step"].get(k, 0), rows["0"]["stamps_us_per_step"][k]))
print("k_step_us", rows["1"].get("k_step_us"), rows["0"].get("k_step_us"))
PY
