#!/bin/bash
# C2 (trimmedmean N=128, d=1e6) at steady state (200 timed steps: the 5-step
# line amortised the first launch and the final sync over 5 kernels of
# 0.1 ms), its kernel stats, and the default north-star line under the
# profiler (gpurun_out/c2/).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/c2"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
for st in 5 50 200 1000; do
  timeout -k 10 200 python3 "$ROOT/bench.py" --no-cpu --no-host --agg trimmedmean --d 1e6 --steps $st --warmup 20 > "$OUTD/c2_s$st.log" 2>&1 || { echo "c2 $st failed"; exit 1; }
  echo "steps $st $(grep '"metric"' "$OUTD/c2_s$st.log" | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/c2prof" -o run \
  -- python3 "$ROOT/bench.py" --agg trimmedmean --d 1e6 --steps 200 --warmup 20 > "$OUTD/c2prof.log" 2>&1 || { echo "c2 prof failed"; exit 1; }
grep -h select_plain $(find "$OUTD/c2prof" -name '*kernel_stats.csv') | cut -d, -f1-4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/defprof" -o run \
  -- python3 "$ROOT/bench.py" > "$OUTD/defprof.log" 2>&1 || { echo "default prof failed"; exit 1; }
grep -h select_plain $(find "$OUTD/defprof" -name '*kernel_stats.csv') | cut -d, -f1-4
grep '"metric"' "$OUTD/defprof.log" | grep -o '"ms_per_step": [0-9.]*'
