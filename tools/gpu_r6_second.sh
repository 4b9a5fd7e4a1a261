#!/bin/bash
# Round 6 second box: the delay test, the delay sweep, then the whole suite + bench + rocprofv3 stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/r6/second}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "tests/test_gpu_plan_contract.py::test_sweep_delay_changes_timing_only" > $O/delay_test.log 2>&1 \
    || { echo "delay test rc=$?"; tail -30 $O/delay_test.log; exit 1; }
tail -1 $O/delay_test.log
bash tools/gpu_r6_delay.sh $O/delay 0,0 15,15 25,25 35,35 50,50 || exit $?
bash tools/gpu_evidence.sh $O/evidence || exit $?
