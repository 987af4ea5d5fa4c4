#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# rocprofv3 kernel-trace summary of the bench on each workload in $WLS (default c3 c2):
# gpurun_out/prof/<wl>/ holds the trace; prints each kernel's calls and average duration.
# STEPS_<wl> overrides the step count (default 200, the default bench's; c2 80, its plan's length).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for w in ${WLS:-c3 c2}; do
  v=STEPS_$w; st=${!v:-$([ $w = c2 ] && echo 80 || echo 200)}
  O=gpurun_out/prof/$w; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 -u bench.py --workload $w --steps $st --warmup 20 --no-cpu-baseline --no-secondary $EXTRA > $O/bench.out 2>&1 || { echo "$w failed"; tail -5 $O/bench.out; exit 1; }
  f=$(find $O -name 'run_kernel_stats.csv' | head -1)
  echo "== $w ($st steps): $f"
  python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print("%-40s calls %7s  avg %9.2f us  total %6.1f%%" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
EOF
  grep -h '^{' $O/bench.out | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('ms/step', d['ms_per_step'], d['kernels_us_per_launch'])"
done
