#!/bin/bash
# rocprofv3 kernel stats of the three Bulyan modes at C3 (N=128, f=20, d=1e7).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/prof_bulyan"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
for agg in ${AGGS:-bulyankrum bulyantrimmedmean bulyanmedian}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/$agg" -o run \
    -- python3 "$ROOT/bench.py" --agg $agg --d 1e7 --steps 3 --warmup 1 --no-cpu --no-host > "$OUTD/$agg.log" 2>&1 || exit 1
  f=$(find "$OUTD/$agg" -name "*kernel_stats.csv" | head -1)
  echo "== $agg"; tail -1 "$OUTD/$agg.log" | cut -c1-200; cut -d, -f1-4 "$f" | head -10
done
