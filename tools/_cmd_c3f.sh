export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/c3f
tools/gpu_steps.sh gpurun_out/r4/c3f \
 "tests|600|python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ops.py tests/test_gpu_loop.py tests/test_gpu_loop_parity.py -x -q --timeout 200 --timeout-method thread" \
 "ab|400|python -u tools/conv3_threshold_ab.py --precision fp32 --B 344 100 25 8 1 --min-tiles 64 --f32-min-tiles 0 192" \
 "cfg4|400|python -u tools/bench_configs4.py" \
 "bench|600|python -u bench.py"
