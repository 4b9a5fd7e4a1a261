#!/bin/bash
# Round 6: the serial final reductions (L1 misfit, metrics) as one workgroup per model, and the batched time
# projection's x reads vectorised (k_wdot_silu_b).  Bitwise fingerprint of the bf16 convs / 344-tile U-Net
# against the committed one, the 344-tile U-Net forward time with its kernel stats, then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/r6/small}
mkdir -p $O
timeout -k 10 200 python -u tools/c3_pair_check.py $O/fp.json > $O/fp.log 2>&1 || { echo "fp rc=$?"; tail -5 $O/fp.log; exit 1; }
python3 tools/c3_pair_check.py --cmp profiles/r6/conv_pair/fp_base.json $O/fp.json
for rep in 1 2; do
  timeout -k 10 300 python -u tools/bench_configs4.py --unet-only --precision bf16 >> $O/unet.jsonl 2>> $O/unet.err || { echo "unet rc=$?"; tail -5 $O/unet.err; exit 1; }
done
tail -2 $O/unet.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o unet -- \
    python3 tools/bench_configs4.py --unet-only --precision bf16 > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
