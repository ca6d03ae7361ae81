#!/bin/bash
# A/B of the full-bucket four-load fill (SRA_GRAM_B4=0/1) on C5 per-GPU
# mom_filterL2, then the filter parity files (gpurun_out/gb4/).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/gb4"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
for b in 0 1 0 1; do
  tag=b${b}_$RANDOM
  SRA_GRAM_B4=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/$tag" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu --no-host --agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3 --warmup 1 > "$OUTD/$tag.log" 2>&1 \
    || { echo "trace $tag failed rc=$?"; exit 1; }
  echo "== $tag $(grep '"metric"' "$OUTD/$tag.log" | grep -o '"ms_per_step": [0-9.]*')"
  grep -h "chunk_gram_kernel<true" $(find "$OUTD/$tag" -name '*kernel_stats.csv') | cut -d, -f1-4
done
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_trace.py tests/test_gpu_shard2.py -x -q --timeout 300 --timeout-method thread \
  > "$OUTD/pytest.log" 2>&1
rc=$?
tail -3 "$OUTD/pytest.log"
exit $rc
