set -o pipefail
O=gpurun_out/r5/ldspad
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-configs4 --no-cpu-baseline > $O/base_$i.json 2> $O/base_$i.err || exit $?
  RDQ_HIP_LIB=red-diffeq_amd/lib_exp/libldspad.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-configs4 --no-cpu-baseline > $O/pad_$i.json 2> $O/pad_$i.err || exit $?
done
