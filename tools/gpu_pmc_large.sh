#!/bin/bash
# PMC passes over one configs[4]-grid forward + adjoint (tools/large_once.py), one group per run.
# usage: tools/gpu_pmc_large.sh <outdir> [large_once args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/p$i -o run -- \
     python3 tools/large_once.py "$@" > $out/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum
GROUPS
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out/calib_$c -o run -- \
     python3 tools/pmc_calib.py > $out/calib_$c.log 2>&1
  rc=$?; echo "pmc calib $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for k in k_fwd_tw k_adj_tw k_fwd_tb k_adj_tb; do
  python3 tools/pmc_traffic.py $out/p1 $out/p2 $out/calib_FETCH_SIZE $out/calib_WRITE_SIZE "$k<" \
     $out/pmc_traffic_$k.json 2>/dev/null
done
exit 0
