export TMPDIR=/tmp
L=red-diffeq_amd/lib_exp
A="tools/conv3_threshold_ab.py --B 344 100 --reps 20"
F="tools/conv3_threshold_ab.py --precision fp32 --B 100 25 --reps 10"
tools/gpu_steps.sh gpurun_out/r4/epi \
 "tests|400|python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_configs4.py -x -q --timeout 200 --timeout-method thread -k 'bf16 or conv3 or configs4 or fp32_halo or gn'" \
 "head1|200|env RDQ_HIP_LIB=$L/libunet_head.so python -u $A" \
 "new1|200|env RDQ_HIP_LIB=$L/libunet_new.so python -u $A" \
 "head2|200|env RDQ_HIP_LIB=$L/libunet_head.so python -u $A" \
 "new2|200|env RDQ_HIP_LIB=$L/libunet_new.so python -u $A" \
 "fhead|200|env RDQ_HIP_LIB=$L/libunet_head.so python -u $F" \
 "fnew|200|env RDQ_HIP_LIB=$L/libunet_new.so python -u $F"
