#!/bin/bash
# Round 3, session j: register-only Bulyan stage + row clamps: tests, C3 bench + kernel stats, fused-round
# occupancy A/B (SRA_ROUND_LDS) with FETCH_SIZE.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3j
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py tests/test_gpu_dba.py tests/test_gpu_shard.py tests/test_gpu_dispatch.py > "$OUT/pytest_bulyan.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" "$OUT/pytest_bulyan.log" | tail -15
[[ $rc -gt 1 ]] && { echo "bulyan pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
for agg in bulyankrum bulyantrimmedmean; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$agg" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg $agg --d 1e7 --steps 3 > "$OUT/prof_$agg.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_$agg.log"; exit 1; }
grep '"metric"' "$OUT/prof_$agg.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$agg', l['ms_per_step'], l['roofline']['frac'])"
python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_$agg/run_kernel_stats.csv')))[:5]: print(x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
done
for pad in 0 24000 64000; do
  SRA_ROUND_LDS=$pad timeout -k 10 120 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyantrimmedmean --d 1e7 --steps 2 > "$OUT/bt_$pad.log" 2>&1 || { echo "bench failed"; tail -3 "$OUT/bt_$pad.log"; exit 1; }
  echo "ROUND_LDS=$pad $(grep '"metric"' "$OUT/bt_$pad.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
  SRA_ROUND_LDS=$pad timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$pad" -o run -- python3 "$R/bench.py" --warmup 0 --no-cpu --no-host --agg bulyantrimmedmean --d 1e7 --steps 1 > "$OUT/pmc_$pad.log" 2>&1 || { echo "pmc failed"; tail -3 "$OUT/pmc_$pad.log"; exit 1; }
  python3 - "$OUT/pmc_$pad" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if 'select_dist_rows_kernel<128' in r['Kernel_Name'] or 'bulyan_final' in r['Kernel_Name']:
        acc[r['Kernel_Name'][:45]].append(float(r['Counter_Value']))
for k, v in acc.items():
    print("  %s launches %d, 2 x FETCH_SIZE per launch %.3f GB" % (k, len(v), 2 * sum(v) / len(v) * 1024 / 1e9))
PY
done
for st in 0 1; do
  SRA_GRAM_STAGE64=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_krum_$st" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg krum --d 1e7 --steps 5 > "$OUT/prof_krum_$st.log" 2>&1 || { echo "krum prof failed"; tail -3 "$OUT/prof_krum_$st.log"; exit 1; }
  echo "GRAM_STAGE64=$st krum $(grep '"metric"' "$OUT/prof_krum_$st.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
  python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_krum_$st/run_kernel_stats.csv')))[:3]: print('  ', x['Name'][:50], x['Calls'], float(x['AverageNs'])/1e6)"
done
timeout -k 10 120 tools/ubench/bin/check_bench > "$OUT/check_bench.txt" 2>&1 || { echo "check_bench failed"; tail -3 "$OUT/check_bench.txt"; }
tail -12 "$OUT/check_bench.txt"
for agg in median trimmedmean; do for nt in 1 0; do
  SRA_QUAD_NT=$nt timeout -k 10 120 python3 "$R/bench.py" --warmup 2 --no-cpu --no-host --agg $agg --clients 512 --d 1.25e7 --steps 10 > "$OUT/q_${agg}_$nt.log" 2>&1 || { echo "quad bench failed"; tail -3 "$OUT/q_${agg}_$nt.log"; exit 1; }
  echo "QUAD_NT=$nt $agg N=512 $(grep '"metric"' "$OUT/q_${agg}_$nt.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms_per_step'], l['roofline']['kernel_ms'], l['roofline']['frac'])")"
  SRA_QUAD_NT=$nt timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcq_${agg}_$nt" -o run -- python3 "$R/bench.py" --warmup 0 --no-cpu --no-host --agg $agg --clients 512 --d 1.25e7 --steps 1 > "$OUT/pmcq_${agg}_$nt.log" 2>&1 || { echo "pmc failed"; exit 1; }
  python3 - "$OUT/pmcq_${agg}_$nt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
v = [float(r['Counter_Value']) for r in csv.DictReader(open(f[0])) if 'select_quad' in r['Kernel_Name']]
print("  quad launches %d, 2 x FETCH_SIZE per launch %.3f GB (algorithmic 25.65)" % (len(v), 2 * sum(v) / max(1, len(v)) * 1024 / 1e9))
PY
done; done
