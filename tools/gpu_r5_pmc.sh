#!/bin/bash
# PMC passes (one rocprofv3 run each) of one bench.py workload; $ARGS = bench args, $PASSES = ';'-separated counter sets
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5pmc}
OUTD="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra PS <<< "$PASSES"
for ctrs in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUTD/p$i" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu --no-host $ARGS > "$OUTD/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok: $ctrs"
done
python3 "$ROOT/tools/pmc_summary.py" "$OUTD" 2>/dev/null | head -40 || true
