#!/bin/bash
# Round 3, session q: software-pipelined Gram (SRA_GRAM_V=5) vs per-wave means (3)
# vs round 2 (0): Krum tests, krum + bulyankrum kernel stats.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3r
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 6 5 3 0; do
  cd "$R"
  SRA_GRAM_V=$v timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_krum.py tests/test_gpu_c3_bulyan.py > "$OUT/pytest_v$v.log" 2>&1
  rc=$?
  echo "V=$v pytest: $(grep -E "passed|failed" "$OUT/pytest_v$v.log" | tail -1)"
  [[ $rc -gt 1 ]] && { echo "pytest rc=$rc, stopping"; tail -20 "$OUT/pytest_v$v.log"; exit $rc; }
  cd /tmp
  for agg in krum bulyankrum; do
    SRA_GRAM_V=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${agg}_v$v" -o run -- python3 "$R/bench.py" --warmup 2 --no-cpu --no-host --agg $agg --d 1e7 --steps 10 > "$OUT/prof_${agg}_v$v.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_${agg}_v$v.log"; exit 1; }
    echo "V=$v $agg $(grep '"metric"' "$OUT/prof_${agg}_v$v.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms_per_step'], l['roofline']['frac'])")"
    python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_${agg}_v$v/run_kernel_stats.csv')))[:3]: print('   ', x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
  done
done
