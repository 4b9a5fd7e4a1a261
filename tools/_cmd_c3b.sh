export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/c3b
tools/gpu_steps.sh gpurun_out/r4/c3b \
 "tests|400|python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread -k 'bf16 or conv3 or configs4'" \
 "ab|300|python -u tools/conv3_threshold_ab.py --B 344 100 25" \
 "micro|300|python -u tools/conv_micro.py --B 344 --bf16 --reps 5 --inner 5"
