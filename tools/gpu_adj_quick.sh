#!/bin/bash
# FWI parity tests + bench phases for a kernel change (run under gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fwi.py > gpurun_out/fwi_tests.log 2>&1
rc=$?
tail -5 gpurun_out/fwi_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-loop --no-red --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
rc=$?
python -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print(d['value'], d['ms_per_step'], d['phases_ms'], d['roofline']['frac'])"
exit $rc
