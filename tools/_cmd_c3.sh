export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/bp2 \
 "tests|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread" \
 "c4|400|python -u tools/bench_configs4.py --precision bf16 --iters 2"
