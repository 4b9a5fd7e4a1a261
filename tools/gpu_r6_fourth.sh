#!/bin/bash
# Round 6: scalar-cache wavelet loads A/B (vecwav = the vector loads of before), then the whole suite +
# bench + rocprofv3 stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/fourth}
bash tools/gpu_r6_spin.sh $O/wav old wavlate || exit $?
bash tools/gpu_evidence.sh $O/evidence || exit $?
