#!/bin/bash
# bf16 batched U-Net with the GroupNorm statistics in the halo conv's epilogue: tests, then the
# configs[4] 344-tile U-Net forward (bf16) and its per-kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/bf16gn
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u tools/bench_configs4.py --unet-only --precision bf16 > $O/unet.jsonl 2> $O/unet.err || exit $?
cat $O/unet.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 tools/bench_configs4.py --unet-only --precision bf16 > $O/prof.log 2>&1 || exit $?
ls $O/prof
timeout -k 10 300 python -u tools/unet_prof_b1.py 1 200 > $O/time.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 8 50 >> $O/time.log 2>&1 || exit $?
grep -v amdgpu.ids $O/time.log
