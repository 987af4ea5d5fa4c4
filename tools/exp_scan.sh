cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for s in 5 200; do
  KB_PROBE_STEPS=$s timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/exp.log 2>&1 || exit 1
  KB_PROBE_STEPS=$s KB_DEBUG_SCAN=1 timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/exp.log 2>&1 || exit 1
done
for n in 256 1024; do KB_NSCAN=$n timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/exp.log 2>&1 || exit 1; done
