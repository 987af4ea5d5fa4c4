#!/bin/bash
# PMC passes over the isolated scan probe (one counter group per rocprofv3 run).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-pmc}
timeout -k 10 120 python -u tools/scan_probe.py > gpurun_out/${TAG}_probe.log 2>&1 || exit $?
KB_DEBUG_SCAN=1 timeout -k 10 120 python -u tools/scan_probe.py >> gpurun_out/${TAG}_probe.log 2>&1 || exit $?
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o run \
      -- python3 tools/scan_probe.py > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/${TAG}_p$i.log; }
done
exit 0
