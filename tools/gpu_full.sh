set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
RDQ_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-loop > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
