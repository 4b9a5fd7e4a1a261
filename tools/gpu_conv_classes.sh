#!/bin/bash
# U-Net / op tests, then per-class fp32 conv rates (bench.conv_class_rates) and U-Net B = 1 / 8 timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/conv_cls
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "
import sys, json, torch; sys.path.insert(0, 'red-diffeq_amd'); sys.path.insert(0, '.')
import bench, red_diffeq.ops
print(json.dumps(bench.conv_class_rates(torch.device('cuda'))), flush=True)
" > $O/classes.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 1 200 > $O/time.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 8 50 >> $O/time.log 2>&1 || exit $?
grep -v amdgpu.ids $O/classes.log $O/time.log
