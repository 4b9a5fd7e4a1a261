#!/bin/bash
# U-Net GPU iteration: parity tests -> timing vs torch eager -> rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_unet.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_unet.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/unet_bench.py --B 1 4 > gpurun_out/unet_bench.log 2>&1
rc=$?; echo "unet_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/unet_bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unet -o run --output-format csv -- python3 tools/unet_bench.py --B 1 --reps 5 > gpurun_out/unet_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
fi
exit $rc
