#!/bin/bash
# filter solver: tests + bench
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r2d
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_filters.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed (continuing)"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -5; }
tail -1 "$OUT/pytest.log"
for a in "filterl2 --d 1e7" "mom_filterl2 --clients 512 --d 1.25e7"; do
  timeout -k 10 240 python bench.py --warmup 1 --no-host --no-cpu --steps 3 --agg $a > "$OUT/b.log" 2>&1 || { echo "bench $a failed"; tail -5 "$OUT/b.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$a', d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 2 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; exit 1; }
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:6]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
