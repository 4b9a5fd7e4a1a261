#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/unet_f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_unet.py tests/test_gpu_loop_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/unet_prof_b1.py 1 200 > $O/time.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 8 50 >> $O/time.log 2>&1 || exit $?
cat $O/time.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 tools/unet_prof_b1.py 1 5 > $O/prof.log 2>&1 || exit $?
python3 tools/unet_timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/timeline.txt || exit $?
tail -30 $O/timeline.txt
