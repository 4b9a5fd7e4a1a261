#!/bin/bash
# Round 6: flag-word exchange (xf_*) and scalar-branch trims of the persistent forward.  FWI parity tests
# first, then the interleaved A/B against the previous commit's build (lib_exp/libhead.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/xf}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fwi.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/fwi_tests.log 2>&1 || { echo "fwi pytest rc=$?"; tail -30 $O/fwi_tests.log; exit 1; }
tail -1 $O/fwi_tests.log
bash tools/gpu_r6_spin.sh $O/ab ${2:-head} || exit $?
