#!/bin/bash
# round-2 session 3: fused Bulyan round + sort4 canonicalisation fix
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r2a
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bulyan.py tests/test_gpu_shard.py tests/test_gpu_c3_bulyan.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for a in "bulyantrimmedmean --d 1e7 --steps 3" "bulyanmedian --d 1e7 --steps 3" "trimmedmean --steps 20"; do
  timeout -k 10 240 python bench.py --warmup 1 --no-host --no-cpu --agg $a > "$OUT/bench_${a%% *}.log" 2>&1 || { echo "bench $a failed"; exit 1; }
  tail -1 "$OUT/bench_${a%% *}.log" | cut -c1-400
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_btm" -o run -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg bulyantrimmedmean --d 1e7 --steps 2 > "$OUT/prof_btm.log" 2>&1 || { echo "prof failed"; exit 1; }
echo done
