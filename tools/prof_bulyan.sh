#!/bin/bash
# rocprofv3 kernel stats of Bulyan (trimmed mean, N=128, d=1e7): default path
# and the row-list A/B variant.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/prof_bulyan"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/alive" -o run \
  -- python3 "$ROOT/bench.py" --agg bulyantrimmedmean --d 1e7 --steps 2 --warmup 1 --no-cpu --no-host > "$OUTD/alive.log" 2>&1 || exit 1
SRA_BULYAN_ROWLIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/rows" -o run \
  -- python3 "$ROOT/bench.py" --agg bulyantrimmedmean --d 1e7 --steps 2 --warmup 1 --no-cpu --no-host > "$OUTD/rows.log" 2>&1 || exit 1
for v in alive rows; do
  f=$(find "$OUTD/$v" -name "*kernel_stats.csv" | head -1)
  echo "== $v"; cut -d, -f1-4 "$f" | head -14
done
