#!/bin/bash
# Round 3, session n: ex_noregret on the cold-started plain solver (in-kernel re-orthogonalising attempt): parity + bench.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3n
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filters.py tests/test_gpu_filter_trace.py tests/test_gpu_dba.py > "$OUT/pytest_filters.log" 2>&1
rc=$?
grep -E "decisions compared|error / bound|passed|failed|FAILED" "$OUT/pytest_filters.log" | tail -20
[[ $rc -gt 1 ]] && { echo "filter pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
for plain in 1 0; do
  SRA_NOREGRET_PLAIN=$plain timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg ex_noregret --d 1e7 --steps 2 > "$OUT/ex_$plain.log" 2>&1 || { echo "bench failed"; tail -3 "$OUT/ex_$plain.log"; exit 1; }
  echo "NOREGRET_PLAIN=$plain ex_noregret $(grep '"metric"' "$OUT/ex_$plain.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 3 > "$OUT/fl.log" 2>&1 && echo "filterl2 $(grep '"metric"' "$OUT/fl.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
