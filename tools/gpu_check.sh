#!/bin/bash
# One GPU-box session: smoke -> gpu parity tests -> blocking sweep -> bench -> rocprofv3 stats.
# Every GPU step has its own time limit; a crash/timeout/fault stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc

if [ -z "${SKIP_TESTS}" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
# 0 = pass, 1 = test failure (safe to continue); anything else (crash, timeout) stops here
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi

timeout -k 10 300 python tools/sweep_tb.py ${SWEEP_ARGS} > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -8 gpurun_out/sweep.log; [ $rc -eq 0 ] || exit $rc

timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc

if [ -n "${PROFILE}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
     python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
