#!/bin/bash
# The batched U-Net's halo-staged 3x3 conv classes under two PMC passes each: MFMA busy and wave waits;
# LDS / memory instruction mix.  PREC=bf16 (default: k_conv3_bf16, B = 344) or PREC=fp32 (k_conv3_f32,
# B = 25).  Summaries -> gpurun_out/conv_pmc_$PREC/summary.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PREC=${PREC:-bf16}
if [ "$PREC" = bf16 ]; then K=k_conv3_bf16; B=${B:-344}; FL=--bf16; else K=k_conv3_f32; B=${B:-25}; FL=; fi
export TMPDIR=/tmp PMC_KERNEL=$K
O=gpurun_out/conv_pmc_$PREC
mkdir -p $O
: > $O/summary.jsonl
for SHAPE in ${SHAPES:-l72_3x3_64_64 l9_3x3_512_512}; do
  P=$O/${SHAPE}_a
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d $P -o run -- \
      python3 tools/conv_micro.py --only $SHAPE --B $B $FL --reps 2 > $P.log 2>&1
  rc=$?; echo "pmc a $SHAPE rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_conv_summary.py $P ${SHAPE}_a >> $O/summary.jsonl || exit 1
  P=$O/${SHAPE}_b
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD \
      SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $P -o run -- \
      python3 tools/conv_micro.py --only $SHAPE --B $B $FL --reps 2 > $P.log 2>&1
  rc=$?; echo "pmc b $SHAPE rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_conv_summary.py $P ${SHAPE}_b >> $O/summary.jsonl || exit 1
done
cat $O/summary.jsonl
exit 0
