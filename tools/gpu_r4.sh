#!/bin/bash
# Round-4 GPU session driver.  usage (on the box, from the repo root):
#   bash tools/gpu_r4.sh TAG step [step ...]
# steps (run in order, stop at the first failure; logs under gpurun_out/TAG/):
#   tests[:<pytest -k expr>]     -m gpu suite (or a -k subset), 900 s cap
#   files:<f1,f2,...>            those test files only (-m gpu)
#   bench:<name>:<bench args>    one bench.py line (json in <name>.log)
#   prof:<name>:<bench args>     rocprofv3 --kernel-trace --stats of one bench run
#   pmc:<name>:<counters>:<bench args>   one rocprofv3 --pmc pass
set -u
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for st in "$@"; do
  kind=${st%%:*}; rest=${st#*:}
  case $kind in
    tests)
      k=""; [ "$rest" != "tests" ] && k="-k $rest"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread $k \
        > "$OUT/pytest.log" 2>&1
      rc=$?; echo "tests: $(tail -1 "$OUT/pytest.log")"
      [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" "$OUT/pytest.log" | head -20; exit $rc; } ;;
    files)
      timeout -k 10 900 python -u -m pytest ${rest//,/ } -m gpu -x -q --timeout 240 --timeout-method thread \
        > "$OUT/pytest_files.log" 2>&1
      rc=$?; echo "files: $(tail -1 "$OUT/pytest_files.log")"
      [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" "$OUT/pytest_files.log" | head -20; exit $rc; } ;;
    bench)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 400 python -u bench.py $args > "$OUT/$name.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "bench $name rc=$rc"; tail -5 "$OUT/$name.log"; exit $rc; }
      python3 -c "import json;d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]);print('bench $name', d['ms_per_step'], 'ms', d['roofline']['frac'], d['roofline'].get('kernel_ms'))" ;;
    prof)
      name=${rest%%:*}; args=${rest#*:}
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
        -- python3 "$R/bench.py" --no-cpu --no-host $args > "$OUT/prof_$name.log" 2>&1)
      rc=$?; [ $rc -ne 0 ] && { echo "prof $name rc=$rc"; tail -5 "$OUT/prof_$name.log"; exit $rc; }
      python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_$name/run_kernel_stats.csv')))[:8]: print('   ', x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e6, 4), 'ms')" ;;
    pmc)
      name=${rest%%:*}; rest2=${rest#*:}; ctr=${rest2%%:*}; args=${rest2#*:}
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } --kernel-trace --output-format csv -d "$OUT/pmc_$name" -o run \
        -- python3 "$R/bench.py" --no-cpu --no-host $args > "$OUT/pmc_$name.log" 2>&1)
      rc=$?; [ $rc -ne 0 ] && { echo "pmc $name rc=$rc"; tail -5 "$OUT/pmc_$name.log"; exit $rc; }
      echo "pmc $name ok" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
