#!/bin/bash
# Round 3, session m: checks skip the eigenvector when they cannot accept: filter parity + traces, bench A/B.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3m
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filters.py tests/test_gpu_filter_trace.py tests/test_gpu_dba.py > "$OUT/pytest_filters.log" 2>&1
rc=$?
grep -E "decisions compared|error / bound|passed|failed|FAILED" "$OUT/pytest_filters.log" | tail -20
[[ $rc -gt 1 ]] && { echo "filter pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 200 python -u tools/filter_debug.py filterL2_n128_c4 synthetic > "$OUT/fdebug.log" 2>&1 && grep -E "mode|cycles|d=" "$OUT/fdebug.log" | tail -12
cd /tmp
for sk in 1 0; do
  SRA_SKIP_Z=$sk timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 3 > "$OUT/fl_$sk.log" 2>&1 || { echo "bench failed"; tail -3 "$OUT/fl_$sk.log"; exit 1; }
  echo "SKIP_Z=$sk filterl2 $(grep '"metric"' "$OUT/fl_$sk.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg ex_noregret --d 1e7 --steps 2 > "$OUT/ex.log" 2>&1 && echo "ex_noregret $(grep '"metric"' "$OUT/ex.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
SRA_NOREGRET_PLAIN=0 timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg ex_noregret --d 1e7 --steps 2 > "$OUT/ex_reorth.log" 2>&1 && echo "ex_noregret (reorth kernel) $(grep '"metric"' "$OUT/ex_reorth.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
