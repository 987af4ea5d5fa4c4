#!/bin/bash
# Diagnostic: isolated c3 k_scan time under the KB_DEBUG_SCAN knobs (0 full, 2 stream
# only, 4 tables only) and scan workgroup counts (KB_NSCAN): the scan's fixed cost.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for n in 256 128 64; do
  for d in 0 2 4; do
    KB_NSCAN=$n KB_DEBUG_SCAN=$d timeout -k 10 120 python3 -u tools/scan_probe.py c3 >> gpurun_out/scan_fixed.jsonl 2>gpurun_out/scan_fixed.err || exit 1
  done
done
