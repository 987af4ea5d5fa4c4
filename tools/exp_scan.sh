# Diagnostic: isolated k_scan timings under the KB_DEBUG_SCAN knobs
# (1 no census, 2 stream only (no scoring), 4 prologue only) and scan grid sizes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for d in 0 1 2 4; do
  KB_PROBE_STEPS=5 KB_DEBUG_SCAN=$d timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/exp.log 2>&1 || exit 1
done
for n in 128 256 384; do KB_NSCAN=$n timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/exp.log 2>&1 || exit 1; done
for n in 256 512; do KB_NSCAN=$n KB_DEBUG_SCAN=2 timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/exp.log 2>&1 || exit 1; done
