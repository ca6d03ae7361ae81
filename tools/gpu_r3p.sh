#!/bin/bash
# Round 3, session p: Gram prefetch-depth / per-wave-means variants (SRA_GRAM_V
# 0..3): Krum tests per variant, krum + bulyankrum kernel stats; then the
# whole-op PMC traffic passes (tools/gpu_pmcw.sh).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3p
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 0 1 2 3; do
  cd "$R"
  SRA_GRAM_V=$v timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_krum.py > "$OUT/pytest_v$v.log" 2>&1
  rc=$?
  echo "V=$v pytest: $(grep -E "passed|failed" "$OUT/pytest_v$v.log" | tail -1)"
  [[ $rc -gt 1 ]] && { echo "pytest rc=$rc, stopping"; exit $rc; }
  cd /tmp
  for agg in krum bulyankrum; do
    SRA_GRAM_V=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${agg}_v$v" -o run -- python3 "$R/bench.py" --warmup 2 --no-cpu --no-host --agg $agg --d 1e7 --steps 10 > "$OUT/prof_${agg}_v$v.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_${agg}_v$v.log"; exit 1; }
    echo "V=$v $agg $(grep '"metric"' "$OUT/prof_${agg}_v$v.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms_per_step'], l['roofline']['frac'])")"
    python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_${agg}_v$v/run_kernel_stats.csv')))[:3]: print('   ', x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
  done
done
bash "$R/tools/gpu_pmcw.sh"
