#!/bin/bash
# Round 6, final code: the N > 1 rehearsals of bench.py again (2 gloo ranks sharing the GPU; one torchrun
# rank through RCCL), so the multi-rank JSON line is known to parse on the kernels the driver will run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/multi}
mkdir -p $O
RDQ_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo "gloo rehearsal rc=$?"; tail -20 $O/bench_gloo2.err; exit 1; }
tail -c 400 $O/bench_gloo2.json
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --steps 10 --warmup 3 --no-red --no-configs4 --no-cpu-baseline \
    > $O/bench_nccl_ws1.json 2> $O/bench_nccl_ws1.err || { echo "nccl ws1 rc=$?"; tail -20 $O/bench_nccl_ws1.err; exit 1; }
tail -c 400 $O/bench_nccl_ws1.json
