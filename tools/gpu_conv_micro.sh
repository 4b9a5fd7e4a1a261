#!/bin/bash
# Per-shape conv timing (B = 1 and 8) + PMC passes over the level-72 3x3 conv.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/conv_micro
mkdir -p $O
timeout -k 10 300 python -u tools/conv_micro.py --B 1 8 > $O/time.jsonl 2> $O/time.err || { cat $O/time.err; exit 1; }
cat $O/time.jsonl
SHAPE=${SHAPE:-l72_3x3_64_64}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- \
     python3 tools/conv_micro.py --only $SHAPE --reps 2 > $O/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM
GROUPS
python3 tools/pmc_summary.py $O k_conv_cc 1
exit 0
