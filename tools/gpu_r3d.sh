#!/bin/bash
# Round 3, session d: new lanczos_solve_kernel -- filter parity tests, then the filterl2 bench + kernel stats.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3d
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filter_trace.py tests/test_gpu_filters.py > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "decisions compared|error / bound|error .* of max|not compared|passed|failed|FAILED" "$OUT/pytest.log" | tail -40
[[ $rc -gt 1 ]] && { echo "pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 300 python -u tools/filter_debug.py filterL2_n128_c4 synthetic > "$OUT/fdebug.log" 2>&1 || { echo "filter_debug failed"; tail -5 "$OUT/fdebug.log"; exit 1; }
tail -12 "$OUT/fdebug.log"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 2 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof.log"; exit 1; }
tail -1 "$OUT/prof.log"
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:6]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
