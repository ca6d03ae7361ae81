#!/bin/bash
# Round 5: filter parity (fixtures, decision traces) + solver timing (run from the repo root).
set -u
mkdir -p gpurun_out
T=${T:-tests/test_gpu_filters.py tests/test_gpu_filter_trace.py}
timeout -k 10 420 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5_pt_filt.log 2>&1
rc=$?
tail -5 gpurun_out/r5_pt_filt.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "${NOBENCH:-}" ] && exit $rc
timeout -k 10 200 python bench.py --agg filterl2 --d 1e7 --steps 3 --warmup 1 --no-cpu --no-host \
  > gpurun_out/r5_bf.log 2>&1 || exit $?
tail -1 gpurun_out/r5_bf.log | cut -c1-400
timeout -k 10 200 python bench.py --agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3 --warmup 1 --no-cpu --no-host \
  > gpurun_out/r5_bmf.log 2>&1 || exit $?
tail -1 gpurun_out/r5_bmf.log | cut -c1-400
exit $rc
