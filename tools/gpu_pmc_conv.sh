#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/unet_prof.py: where the batched bf16
# U-Net convolutions spend their cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcc
export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcc/p$i -o run -- \
     python3 tools/unet_prof.py --reps 2 > gpurun_out/pmcc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
GROUPS
exit 0
