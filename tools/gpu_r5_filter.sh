#!/bin/bash
# Round 5: filter parity (fixtures, decision traces) + solver timing (run from the repo root).
# B: bench lines "tag|bench args" (default: C4 filterL2 and C5 mom_filterL2); NOBENCH=1 skips them.
set -u
mkdir -p gpurun_out
T=${T:-tests/test_gpu_filters.py tests/test_gpu_filter_trace.py}
B=${B:-"bf|--agg filterl2 --d 1e7
bmf|--agg mom_filterl2 --clients 512 --d 1.25e7"}
timeout -k 10 420 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5_pt_filt.log 2>&1
rc=$?
tail -5 gpurun_out/r5_pt_filt.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "${NOBENCH:-}" ] && exit $rc
while IFS='|' read -r tag args; do
  [[ -z "$tag" ]] && continue
  timeout -k 10 200 python bench.py $args --steps 3 --warmup 1 --no-cpu --no-host \
    > gpurun_out/r5_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r5_$tag.log | cut -c1-400
done <<< "$B"
exit $rc
