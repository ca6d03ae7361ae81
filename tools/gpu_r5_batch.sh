#!/bin/bash
# round-5 batch: solver diagnostics, filter parity + benches, first-check sweep, two-rank shard test
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/filter_debug.py filterL2_exit synthetic > gpurun_out/fds.log 2>&1 || exit $?
grep -A8 "mode 0" gpurun_out/fds.log | grep "per\|d=\|checks"
grep "^out\|^want" gpurun_out/fds.log
./tools/gpu_r5_filter.sh || exit $?
./tools/sweep_tmp.sh || exit $?
./tools/gpu_r5_shard2.sh
