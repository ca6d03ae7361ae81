#!/bin/bash
# k10 (DBA harness) kernels on one MI355X: bench lines (N=128, d=1e8) with the
# CPU port beside them, then rocprofv3 kernel stats of the same commands.
set -u
OUT=${OUT:-gpurun_out/dba}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for agg in dba_median dba_weighted_sum; do
  timeout -k 10 300 python "$R/bench.py" --agg $agg --steps 10 --warmup 2 --cpu-seconds 6 --no-host \
    > "$OUT/bench_$agg.log" 2>&1 || { echo "bench $agg failed rc=$?"; exit 1; }
  grep '^{' "$OUT/bench_$agg.log"
done
cd /tmp
for agg in dba_median dba_weighted_sum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$agg" -o run \
    -- python3 "$R/bench.py" --agg $agg --steps 10 --warmup 2 --no-cpu --no-host \
    > "$R/$OUT/prof_$agg.log" 2>&1 || { echo "prof $agg failed rc=$?"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_tests" -o run \
  -- python3 -m pytest "$R/tests/test_gpu_dba.py" -q -p no:cacheprovider > "$R/$OUT/prof_tests.log" 2>&1 \
  || { echo "prof tests failed rc=$?"; exit 1; }
echo done
