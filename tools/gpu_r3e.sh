#!/bin/bash
# Round 3, session e: N > 128 paths (Bulyan, Krum / Gram, filters) + shard tests, filter parity, filterl2 bench + kernel stats.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3e
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_shard.py tests/test_gpu_krum.py > "$OUT/pytest_bulyan.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" "$OUT/pytest_bulyan.log" | tail -15
[[ $rc -gt 1 ]] && { echo "bulyan pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filters.py tests/test_gpu_filter_trace.py > "$OUT/pytest_filters.log" 2>&1
rc=$?
grep -E "decisions compared|agreed prefix|error / bound|error .* of max|not compared|passed|failed|FAILED" "$OUT/pytest_filters.log" | tail -40
[[ $rc -gt 1 ]] && { echo "filter pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 2 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof.log"; exit 1; }
tail -1 "$OUT/prof.log"
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:6]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
