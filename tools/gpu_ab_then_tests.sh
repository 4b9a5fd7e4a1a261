#!/bin/bash
# A/B of library builds on the persistent FWI kernels (tools/ab_libs.sh), then a pytest selection
# against the default build.  Usage: tools/gpu_ab_then_tests.sh OUTDIR "pytest args" lib/a.so lib/b.so ...
# Stops at the first GPU fault / abort / time limit (exit status >= 124).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$1; shift
T=$1; shift
mkdir -p $O
bash tools/ab_libs.sh "$@" > $O/ab.txt 2>&1
rc=$?
cat $O/ab.txt
[ $rc -ge 124 ] && { echo "ab rc=$rc"; exit $rc; }
if [ -n "$T" ]; then
  RDQ_EVIDENCE_DIR=$O timeout -k 10 600 python -u -m pytest $T -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
  rc=$?
  tail -15 $O/tests.log
  exit $rc
fi
