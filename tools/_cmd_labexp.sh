export TMPDIR=/tmp
L=red-diffeq_amd/lib_exp
A="tools/conv3_threshold_ab.py --B 344 100 --reps 20"
tools/gpu_steps.sh gpurun_out/r4/labexp \
 "head1|200|env RDQ_HIP_LIB=$L/libunet_head.so python -u $A" \
 "new1|200|env RDQ_HIP_LIB=$L/libunet_new.so python -u $A" \
 "head2|200|env RDQ_HIP_LIB=$L/libunet_head.so python -u $A" \
 "new2|200|env RDQ_HIP_LIB=$L/libunet_new.so python -u $A" \
 "tests|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 200 --timeout-method thread -k 'linear_attention or bf16'"
