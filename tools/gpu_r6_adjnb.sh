#!/bin/bash
# Round 6: barrier-free persistent adjoint (ADJR_STEP_NB, wave priorities).  FWI parity tests first, then
# the interleaved A/B against the barrier-per-step build (lib_exp/libadjbar.so, ADJ_NB = false), then
# the whole GPU suite.  A failure stops the run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/adjnb}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fwi.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/fwi_tests.log 2>&1 || { echo "fwi pytest rc=$?"; tail -30 $O/fwi_tests.log; exit 1; }
tail -1 $O/fwi_tests.log
bash tools/gpu_r6_spin.sh $O/ab adjbar || exit $?
RDQ_EVIDENCE_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
