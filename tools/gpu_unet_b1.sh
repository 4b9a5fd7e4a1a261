#!/bin/bash
# B = 1 U-Net iteration: U-Net parity tests + op checks -> graph-replay timing -> rocprofv3 kernel
# trace of the same forward (per-launch timeline of the last forward in gpurun_out/unet_b1/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/unet_b1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ops.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/unet_prof_b1.py 1 200 > $O/time.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 8 50 >> $O/time.log 2>&1 || exit $?
cat $O/time.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 tools/unet_prof_b1.py 1 5 > $O/prof.log 2>&1 || exit $?
python3 tools/unet_timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/timeline.txt || exit $?
tail -40 $O/timeline.txt
