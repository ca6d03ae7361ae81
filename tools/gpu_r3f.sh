#!/bin/bash
# Round 3, session f: filter solver with in-kernel re-orthogonalising attempt + single batch: parity, bench, kernel stats.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3f
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filters.py tests/test_gpu_filter_trace.py tests/test_gpu_shard.py > "$OUT/pytest_filters.log" 2>&1
rc=$?
grep -E "decisions compared|error / bound|passed|failed|FAILED" "$OUT/pytest_filters.log" | tail -20
[[ $rc -gt 1 ]] && { echo "filter pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 200 python -u tools/filter_debug.py filterL2_n128_c4 synthetic > "$OUT/fdebug.log" 2>&1 || { echo "filter_debug failed"; tail -5 "$OUT/fdebug.log"; exit 1; }
tail -14 "$OUT/fdebug.log"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 2 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof.log"; exit 1; }
grep '"metric"' "$OUT/prof.log" | cut -c1-300
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:6]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
