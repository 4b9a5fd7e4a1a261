#!/bin/bash
# Round-end evidence: full GPU test suite, bench line, configs[4] RED iteration (bf16 / fp32 U-Net)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 600 $O/bench.json
timeout -k 10 600 python -u tools/bench_configs4.py > $O/configs4.jsonl 2> $O/configs4.err || exit $?
cat $O/configs4.jsonl
