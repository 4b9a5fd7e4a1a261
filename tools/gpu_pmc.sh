#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run, --kernel-trace only beside --pmc),
# then the calibrated per-launch traffic of the dominant kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ONLY=${ONLY:-4}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- \
     python3 tools/sweep_tb.py --reps 1 --only $ONLY > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum
GROUPS
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/calib_$c -o run -- \
     python3 tools/pmc_calib.py > gpurun_out/pmc/calib_$c.log 2>&1
  rc=$?; echo "pmc calib $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for k in k_fwd_pt k_adj_pr; do
  # file name = what bench.py looks up: profiles/pmc_traffic_<kernel><T>_ns<ns>_B<B>.json
  python3 tools/pmc_traffic.py gpurun_out/pmc/p1 gpurun_out/pmc/p2 gpurun_out/pmc/calib_FETCH_SIZE \
     gpurun_out/pmc/calib_WRITE_SIZE "$k<$ONLY," gpurun_out/pmc/pmc_traffic_${k}${ONLY}_ns8_B1.json
done
exit 0
