#!/bin/bash
# A/B of the software-pipelined plain chunk-Gram fill (SRA_GRAM_PF=0/1) on C4
# filterL2 and ex_noregret, then the filter parity files (gpurun_out/gpf/).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/gpf"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
for cfg in "0 filterl2" "1 filterl2" "1 ex_noregret" "0 ex_noregret"; do
  set -- $cfg
  tag=pf$1_$2
  SRA_GRAM_PF=$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/$tag" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu --no-host --agg $2 --d 1e7 --steps 3 --warmup 1 > "$OUTD/$tag.log" 2>&1 \
    || { echo "trace $tag failed rc=$?"; exit 1; }
  echo "== $tag $(grep '"metric"' "$OUTD/$tag.log" | grep -o '"ms_per_step": [0-9.]*')"
  grep -h chunk_gram $(find "$OUTD/$tag" -name '*kernel_stats.csv') | cut -d, -f1-4
done
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_trace.py -x -q --timeout 300 --timeout-method thread \
  > "$OUTD/pytest.log" 2>&1
rc=$?
tail -3 "$OUTD/pytest.log"
exit $rc
