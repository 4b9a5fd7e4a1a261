#!/bin/bash
# rocprofv3 kernel trace + stats of the blocking sweep and of bench.py (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep -o run --output-format csv -- \
   python3 tools/sweep_tb.py --reps 2 ${SWEEP_ARGS} > gpurun_out/prof_sweep.log 2>&1
rc=$?; echo "prof sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- \
   python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
