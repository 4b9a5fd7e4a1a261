#!/bin/bash
# Per conv class: timing (tools/conv_micro.py) and one PMC pass (MFMA busy, wave waits) each, for the
# U-Net's fp32 k_conv_cc launches at B = 1 and 8.  Summaries -> gpurun_out/conv_pmc/summary.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/conv_pmc
mkdir -p $O
timeout -k 10 300 python -u tools/conv_micro.py --B 1 8 > $O/time.jsonl 2> $O/time.err || { cat $O/time.err; exit 1; }
cat $O/time.jsonl
: > $O/summary.jsonl
for SHAPE in l72_3x3_64_64 l72_3x3_128_64 l36_3x3_64_64 l9_3x3_512_512 l72_1x1_64_384; do
  for B in 1 8; do
    P=$O/${SHAPE}_B$B
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d $P -o run -- \
        python3 tools/conv_micro.py --only $SHAPE --B $B --reps 2 > $P.log 2>&1
    rc=$?; echo "pmc $SHAPE B=$B rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 tools/pmc_conv_summary.py $P ${SHAPE}_B$B >> $O/summary.jsonl || exit 1
  done
done
cat $O/summary.jsonl
exit 0
