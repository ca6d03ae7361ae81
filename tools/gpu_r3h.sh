#!/bin/bash
# Round 3, session h: register-only Bulyan stage: tests + C3 bulyankrum / bulyantrimmedmean bench + kernel stats.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3h
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py tests/test_gpu_shard.py tests/test_gpu_dispatch.py > "$OUT/pytest_bulyan.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" "$OUT/pytest_bulyan.log" | tail -15
[[ $rc -gt 1 ]] && { echo "bulyan pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
for agg in bulyankrum bulyantrimmedmean; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$agg" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg $agg --d 1e7 --steps 3 > "$OUT/prof_$agg.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_$agg.log"; exit 1; }
grep '"metric"' "$OUT/prof_$agg.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$agg', l['ms_per_step'], l['roofline']['frac'])"
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_$agg/run_kernel_stats.csv')))[:5]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
done
