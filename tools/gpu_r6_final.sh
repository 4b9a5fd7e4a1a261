#!/bin/bash
# Round 6 evidence on the final kernels: suite + bench + rocprofv3 stats, PMC passes (calibrated HBM
# traffic per launch + instruction mix) and the persistent kernels' per-wave phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/r6/final}
mkdir -p $O
bash tools/gpu_evidence.sh $O/evidence || exit $?
bash tools/gpu_pmc.sh || exit $?
{ python -u tools/pmc_summary.py gpurun_out/pmc "k_fwd_pt<4" 1000 3584; python -u tools/pmc_summary.py gpurun_out/pmc "k_adj_pr<4" 1000 3584; } > $O/pmc_summary.txt 2>&1 || echo "pmc_summary rc=$?"
timeout -k 10 200 python -u tools/sweep_tb.py --only 4 --profile --reps 3 > $O/phase_profile.json 2> $O/phase_profile.err || exit $?
tail -c 400 $O/phase_profile.json
