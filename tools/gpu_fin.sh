set -o pipefail
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fwi.py tests/test_gpu_loop.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/prof -o b -- python3 bench.py --steps 10 --warmup 3 --no-loop --no-red --no-cpu-baseline > gpurun_out/fin/b.json 2>/dev/null || exit 1
python3 -c "
import csv; rows=list(csv.DictReader(open('gpurun_out/fin/prof/b_kernel_stats.csv')))
[print(r['Name'][:60], r['AverageNs']) for r in rows if 'fin' in r['Name'] or 'k_adj_pr' in r['Name']]"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-loop --no-red --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'])"
