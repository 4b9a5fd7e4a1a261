#!/bin/bash
# Round 6, first box: the plan-contract / production-tuning tests and the SSIM-module test first,
# then the whole GPU suite with margins, then the N > 1 rehearsals of bench.py (2 gloo ranks sharing
# the GPU; one torchrun rank through RCCL).  Usage: tools/gpu_r6_contract.sh OUTDIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/r6/contract}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plan_contract.py \
    "tests/test_gpu_loop_parity.py::test_engine_calls_a_non_reference_ssim_module" > $O/new_tests.log 2>&1 \
    || { echo "new tests rc=$?"; tail -40 $O/new_tests.log; exit 1; }
tail -2 $O/new_tests.log
RDQ_EVIDENCE_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
RDQ_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo "gloo rehearsal rc=$?"; tail -20 $O/bench_gloo2.err; exit 1; }
tail -c 600 $O/bench_gloo2.json
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --steps 10 --warmup 3 --no-red --no-configs4 --no-cpu-baseline \
    > $O/bench_nccl_ws1.json 2> $O/bench_nccl_ws1.err || { echo "nccl ws1 rc=$?"; tail -20 $O/bench_nccl_ws1.err; exit 1; }
tail -c 600 $O/bench_nccl_ws1.json
echo done
