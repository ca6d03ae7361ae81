#!/bin/bash
# Bulyan final stage: tests + bench (bulyankrum, bulyantrimmedmean) + kernel stats
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/fin
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py tests/test_gpu_shard.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for a in bulyankrum bulyankrum; do
  timeout -k 10 240 python bench.py --warmup 2 --no-host --no-cpu --agg $a --d 1e7 --steps 10 > "$OUT/b.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/b.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$a', d['ms_per_step'])"
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyankrum --d 1e7 --steps 5 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; exit 1; }
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:5]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
