#!/bin/bash
# Filter parity + solver timing on the GPU box (run from the repo root).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_dispatch.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pt_filt.log 2>&1
rc=$?
tail -3 gpurun_out/pt_filt.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/filter_debug.py filterL2_exit synthetic > gpurun_out/filter_debug2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --agg filterl2 --d 1e7 --steps 2 --warmup 1 --no-cpu --no-host \
  > gpurun_out/bf.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --agg ex_noregret --d 1e7 --steps 2 --warmup 1 --no-cpu --no-host \
  > gpurun_out/be.log 2>&1 || exit $?
exit $rc
