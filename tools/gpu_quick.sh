#!/bin/bash
# Quick GPU iteration: FWI parity tests -> sweep with phase profile -> bench (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fwi.py -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_fwi.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_fwi.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/sweep_tb.py --only 4 --profile --reps 3 > gpurun_out/sweep_prof.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -c 1500 gpurun_out/sweep_prof.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; exit $rc
