#!/bin/bash
# Round 3, session i: Bulyan tests after the row clamps; fused-round occupancy A/B (SRA_ROUND_LDS) with
# bench time and FETCH_SIZE of the rounds.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3i
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_c3_bulyan.py > "$OUT/pytest_bulyan.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" "$OUT/pytest_bulyan.log" | tail -8
[[ $rc -gt 1 ]] && { echo "bulyan pytest rc=$rc, stopping"; exit $rc; }
cd /tmp
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
