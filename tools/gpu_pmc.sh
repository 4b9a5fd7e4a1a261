#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run, --kernel-trace only beside --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ONLY=${ONLY:-4}
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- \
     python3 tools/sweep_tb.py --reps 1 --only $ONLY > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/calib -o run -- \
   python3 tools/pmc_calib.py > gpurun_out/pmc/calib.log 2>&1
rc=$?; echo "pmc calib rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
