#!/bin/bash
# Round 3, session v: per-wave means on the eight-wave Gram (SRA_GRAM_V=8) vs
# default: Krum tests (N 129..256 unpaired use it), mom_krum kernel stats.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3v
mkdir -p "$OUT"
for v in 8 -1; do
  cd "$R"
  SRA_GRAM_V=$v timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_krum.py > "$OUT/pytest_v$v.log" 2>&1
  rc=$?
  echo "V=$v pytest: $(grep -E "passed|failed" "$OUT/pytest_v$v.log" | tail -1)"
  [[ $rc -gt 1 ]] && { tail -20 "$OUT/pytest_v$v.log"; exit $rc; }
  cd /tmp
  SRA_GRAM_V=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_v$v" -o run -- python3 "$R/bench.py" --warmup 2 --no-cpu --no-host --agg mom_krum --clients 512 --d 1.25e7 --steps 10 > "$OUT/v$v.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/v$v.log"; exit 1; }
  echo "V=$v mom_krum $(grep '"metric"' "$OUT/v$v.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms_per_step'])")"
  python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_v$v/run_kernel_stats.csv')))[:2]: print('   ', x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
done
