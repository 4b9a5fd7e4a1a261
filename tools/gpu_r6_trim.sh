#!/bin/bash
# Round 6: adjoint step trims (lib_exp/libtrim.so: one scalar branch for the source row's two gradient
# terms, the receiver test only in the half holding the receiver's pair, the history-slot test once per
# epoch).  FWI parity tests on that build, then the interleaved A/B against the product build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/trim}
mkdir -p $O
RDQ_HIP_LIB=red-diffeq_amd/lib_exp/libtrim.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fwi.py tests/test_gpu_plan_contract.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/fwi_tests.log 2>&1 || { echo "fwi pytest rc=$?"; tail -30 $O/fwi_tests.log; exit 1; }
tail -1 $O/fwi_tests.log
bash tools/gpu_r6_spin.sh $O/ab trim || exit $?
