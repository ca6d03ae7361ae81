#!/bin/bash
# kernel-trace --stats of bench.py for the listed workloads (name|args lines in $W); outputs gpurun_out/$TAG/
set -u
TAG=${TAG:-r5prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
while IFS='|' read -r name args; do
  [[ -z "$name" ]] && continue
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/$name" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu --no-host $args > "$OUTD/$name.log" 2>&1 \
    || { echo "trace $name failed rc=$?"; exit 1; }
  python3 "$ROOT/tools/kstats.py" $(find "$OUTD/$name" -name '*kernel_stats.csv') | head -12
  tail -1 "$OUTD/$name.log" | cut -c1-200
done <<< "$W"
