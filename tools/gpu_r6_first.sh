#!/bin/bash
# Round 6 first box: contract tests + suite + N>1 rehearsals, then the latency-hiding probe and the B = 25
# reg_losses diagnostic.  A test failure does not stop the probes; a fault, abort or time limit does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/first}
mkdir -p $O
bash tools/gpu_r6_contract.sh $O/contract; rc=$?
echo "contract rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
bash tools/gpu_r6_busy.sh $O/busy || exit $?
timeout -k 10 300 python -u tools/b25_reg_diag.py $O/b25_reg_diag.json 2> $O/b25_reg_diag.err || { echo "diag rc=$?"; tail -20 $O/b25_reg_diag.err; exit 1; }
tail -8 $O/b25_reg_diag.err
exit $rc
