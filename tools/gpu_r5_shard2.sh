#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard2.py tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_shard2.log 2>&1
rc=$?
tail -15 gpurun_out/r5_shard2.log
exit $rc
