#!/bin/bash
# Round 3, session k: ex_noregret on the warm-started plain solver: filter parity + traces, bench A/B.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3k
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filters.py tests/test_gpu_filter_trace.py > "$OUT/pytest_filters.log" 2>&1
rc=$?
grep -E "decisions compared|error / bound|passed|failed|FAILED" "$OUT/pytest_filters.log" | tail -20
[[ $rc -gt 1 ]] && { echo "filter pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
for plain in 1 0; do
  SRA_NOREGRET_PLAIN=$plain timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg ex_noregret --d 1e7 --steps 2 > "$OUT/ex_$plain.log" 2>&1 || { echo "bench failed"; tail -3 "$OUT/ex_$plain.log"; exit 1; }
  echo "NOREGRET_PLAIN=$plain ex_noregret $(grep '"metric"' "$OUT/ex_$plain.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ex" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg ex_noregret --d 1e7 --steps 2 > "$OUT/prof_ex.log" 2>&1 || { echo "prof failed"; exit 1; }
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_ex/run_kernel_stats.csv')))[:5]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg mom_ex_noregret --clients 512 --d 1e7 --steps 2 > "$OUT/mex.log" 2>&1 && echo "mom_ex_noregret N=512 $(grep '"metric"' "$OUT/mex.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
cd "$R"
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py > "$OUT/pytest_bulyan.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" "$OUT/pytest_bulyan.log" | tail -8
[[ $rc -gt 1 ]] && { echo "bulyan pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bk" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyankrum --d 1e7 --steps 5 > "$OUT/prof_bk.log" 2>&1 || { echo "prof failed"; exit 1; }
grep '"metric"' "$OUT/prof_bk.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('bulyankrum', l['ms_per_step'], l['roofline']['frac'])"
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_bk/run_kernel_stats.csv')))[:4]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
cd "$R/tools/ubench" && mkdir -p bin && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bin/check_bench check_bench.hip ../../secure-robust-federated-learning_amd/csrc/common.hip > "$OUT/cb_build.log" 2>&1 && timeout -k 10 120 bin/check_bench > "$OUT/check_bench.txt" 2>&1; tail -12 "$OUT/check_bench.txt"
