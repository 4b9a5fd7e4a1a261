#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r6_pairs.sh gpurun_out/r6/pairs || exit $?
bash tools/gpu_r6_spin.sh gpurun_out/r6/reorder fh fhi ai
