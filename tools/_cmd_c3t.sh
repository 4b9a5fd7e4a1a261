export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/c3t
tools/gpu_steps.sh gpurun_out/r4/c3t \
 "tests|600|python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_loop.py -x -q --timeout 200 --timeout-method thread" \
 "cfg4|400|python -u tools/bench_configs4.py"
