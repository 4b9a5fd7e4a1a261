export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/ga \
 "tests|400|python -u -m pytest tests/test_gpu_fwi.py -x -q --timeout 300 --timeout-method thread -k 'wide or marmousi or chunked'" \
 "large|400|python -u tools/bench_large.py --T 4" \
 "pmc|900|bash tools/gpu_pmc.sh"
