export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/h16
tools/gpu_steps.sh gpurun_out/r4/h16 \
 "tests|600|python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ops.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread" \
 "ab|300|python -u tools/conv3_threshold_ab.py --B 344 100 25 --min-tiles 64" \
 "cfg4|400|python -u tools/bench_configs4.py"
