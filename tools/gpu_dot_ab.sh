set -o pipefail
cd "${GRAFT_REPO_ROOT}"
for lib in fin nofin fin nofin; do
  cp red-diffeq_amd/lib/lib_$lib.so red-diffeq_amd/lib/libred_diffeq_hip.so
  for i in 1 2 3; do
    timeout -k 10 200 python -u -m pytest tests/test_gpu_fwi.py -q -k "dot_product_openfwi_ns8" --timeout 150 --timeout-method thread 2>&1 | tail -1 | sed "s/^/$lib: /"
  done
done
