#!/bin/bash
# Evidence pass on one MI355X: GPU test suite, bench line, rocprofv3 kernel stats of the same
# bench command.  Usage: tools/gpu_evidence.sh OUTDIR [notests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/r3/evidence}
mkdir -p $O
if [ "$2" != "notests" ]; then
  RDQ_EVIDENCE_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 800 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-loop --no-red --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || exit $?
echo done
