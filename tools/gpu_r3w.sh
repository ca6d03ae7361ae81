#!/bin/bash
# Round 3, session w: one-read median rounds (median_pass_kernel + finisher):
# Bulyan GPU tests, then bulyanmedian C3 A/B with the fused two-read rounds.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3w
mkdir -p "$OUT"
cd "$R"
SRA_BULYAN_MEDIAN_1READ=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py tests/test_gpu_shard.py > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest: $(grep -E "passed|failed" "$OUT/pytest.log" | tail -1)"
[[ $rc -ne 0 ]] && { grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -20; exit $rc; }
cd /tmp
for v in 1 0; do
  SRA_BULYAN_MEDIAN_1READ=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_v$v" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyanmedian --d 1e7 --steps 3 > "$OUT/v$v.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/v$v.log"; exit 1; }
  echo "1READ=$v bulyanmedian $(grep '"metric"' "$OUT/v$v.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms_per_step'], l['roofline']['frac'])")"
  python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_v$v/run_kernel_stats.csv')))[:6]: print('   ', x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
done
