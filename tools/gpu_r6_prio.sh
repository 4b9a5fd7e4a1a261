#!/bin/bash
# Round 6: wave-priority variants of the persistent forward (A/B), then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/prio2}
bash tools/gpu_r6_spin.sh $O/ab noprio body2 swept3 || exit $?
mkdir -p $O
RDQ_EVIDENCE_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
