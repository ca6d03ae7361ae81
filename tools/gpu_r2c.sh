#!/bin/bash
# fused Bulyan round (from4 network, global loads): tests + bench + kernel stats
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r2c
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_shard.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for a in bulyantrimmedmean bulyanmedian; do
  timeout -k 10 240 python bench.py --warmup 1 --no-host --no-cpu --agg $a --d 1e7 --steps 3 > "$OUT/b_$a.log" 2>&1 || { echo "bench $a failed"; tail -5 "$OUT/b_$a.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b_$a.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$a', d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_btm" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyantrimmedmean --d 1e7 --steps 2 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; exit 1; }
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_btm/run_kernel_stats.csv')))[:9]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
