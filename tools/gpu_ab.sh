#!/bin/bash
# A/B of library variants on c3 and c2 (ms/step and per-kernel device times), alternating twice
cd /tmp/co 2>/dev/null; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for w in ${WLS:-c3 c2}; do
  echo "== $w"
  WL=$w STEPS=${STEPS:-1000} tools/exp_step.sh "$@" || exit 1
done
