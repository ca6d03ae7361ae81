#!/bin/bash
# A/B of the MoM (bucket) chunk Gram: SRA_GRAM_VB=0 (two waves per SIMD) vs 1
# (three) on C5 per-GPU mom_filterL2; then the default-variant C4 filterL2 and
# C4 ex_noregret bench lines under the profiler (gpurun_out/gab2/).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/gab2"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
run() {   # tag env args...
  local tag=$1 envs=$2; shift 2
  eval "$envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d \"$OUTD/$tag\" -o run -- python3 \"$ROOT/bench.py\" --no-cpu --no-host $* > \"$OUTD/$tag.log\" 2>&1" \
    || { echo "trace $tag failed"; exit 1; }
  echo "== $tag"
  python3 "$ROOT/tools/kstats.py" $(find "$OUTD/$tag" -name '*kernel_stats.csv') | grep -E "chunk_gram|wave_solve|noregret_pre"
  tail -1 "$OUTD/$tag.log" | cut -c1-160
}
run mf_vb0 "SRA_GRAM_VB=0" --agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3 --warmup 1
run mf_vb1 "SRA_GRAM_VB=1" --agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3 --warmup 1
run mx_vb1 "SRA_GRAM_VB=1" --agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 3 --warmup 1
run ex_v1 "SRA_GRAM_V=1" --agg ex_noregret --d 1e7 --steps 3 --warmup 1
cd "$ROOT"
SRA_GRAM_VB=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_trace.py tests/test_gpu_shard2.py -x -q --timeout 300 --timeout-method thread \
  > "$OUTD/pytest.log" 2>&1
rc=$?
tail -3 "$OUTD/pytest.log"
exit $rc
