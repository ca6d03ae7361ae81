#!/bin/bash
# A/B of the filter chunk Gram variants (SRA_GRAM_V / SRA_GRAM_V4) on C4 filterL2:
# kernel stats per variant under gpurun_out/gab/, then the filter parity files.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/gab"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
for cfg in "0 0" "0 1" "1 1" "2 0"; do
  set -- $cfg
  tag=v$1_f$2
  SRA_GRAM_V=$1 SRA_GRAM_V4=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/$tag" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu --no-host --agg filterl2 --d 1e7 --steps 3 --warmup 1 > "$OUTD/$tag.log" 2>&1 \
    || { echo "trace $tag failed rc=$?"; exit 1; }
  echo "== $tag"
  python3 "$ROOT/tools/kstats.py" $(find "$OUTD/$tag" -name '*kernel_stats.csv') | grep -E "chunk_gram|wave_solve"
  tail -1 "$OUTD/$tag.log" | cut -c1-160
done
cd "$ROOT"
[ -n "${NOTEST:-}" ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_trace.py -x -q --timeout 300 --timeout-method thread \
  > "$OUTD/pytest.log" 2>&1
rc=$?
tail -3 "$OUTD/pytest.log"
exit $rc
