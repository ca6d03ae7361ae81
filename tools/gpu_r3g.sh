#!/bin/bash
# Round 3, session g: Bulyan stage rewrite (per-wave LDS tile, register tie-break) tests + C3 bench/stats;
# filterL2 check-schedule A/B (SRA_FCHECK / SRA_FADV).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3g
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py tests/test_gpu_shard.py > "$OUT/pytest_bulyan.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" "$OUT/pytest_bulyan.log" | tail -15
[[ $rc -gt 1 ]] && { echo "bulyan pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bk" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyankrum --d 1e7 --steps 5 > "$OUT/prof_bk.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_bk.log"; exit 1; }
grep '"metric"' "$OUT/prof_bk.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('bulyankrum', l['ms_per_step'], l['roofline']['frac'])"
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_bk/run_kernel_stats.csv')))[:6]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
for fc in -8 -4 0 2 4; do
  SRA_FCHECK=$fc timeout -k 10 120 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 3 > "$OUT/fl_$fc.log" 2>&1 || { echo "filter bench failed"; tail -3 "$OUT/fl_$fc.log"; exit 1; }
  echo "FCHECK=$fc $(grep '"metric"' "$OUT/fl_$fc.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
SRA_FCHECK=0 SRA_FADV=4 timeout -k 10 120 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 3 > "$OUT/fl_0_4.log" 2>&1 && echo "FCHECK=0 FADV=4 $(grep '"metric"' "$OUT/fl_0_4.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
