export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/ov \
 "unet|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -k 'time_mlp'" \
 "ovl|600|python -u bench.py --no-configs4 --no-cpu-baseline" \
 "serial|600|RDQ_NO_OVERLAP=1 python -u bench.py --no-configs4 --no-cpu-baseline"
