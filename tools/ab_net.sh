#!/bin/bash
# A/B of the exact-N trimmed-mean networks: SRA_NET=0 (VOP3 NaN-propagating
# minimum3/maximum3) vs 1 (NaN pre-pass + VOP2 min/max, sorted-4 base blocks)
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_coordwise.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for r in 1 2; do
for n in 128 100; do
  for net in 0 1; do
    SRA_NET=$net timeout -k 10 200 python bench.py --agg trimmedmean --clients $n --steps 20 --warmup 3 --no-cpu --no-host > gpurun_out/b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('N=$n net=$net', r['kernel_ms'], r['frac'])"
  done
done
done
