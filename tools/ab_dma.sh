#!/bin/bash
# A/B of the k-select variants on the GPU box (trimmed mean / median, N=128 and
# 100, d=1e8): LDS-DMA with 2 waves/SIMD (default), 1 wave/SIMD, and the
# one-lane register path.  Each run under its own time limit; stops at the
# first failure.
set -u
OUT=${OUT:-gpurun_out/ab_dma}
mkdir -p "$OUT"
run() { # name env... -- args
  local name=$1; shift
  echo "== $name" | tee -a "$OUT/summary.txt"
  timeout -k 10 240 env "$@" > "$OUT/$name.log" 2>&1 || { echo "FAILED $name rc=$?" | tee -a "$OUT/summary.txt"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('  value %.1f GB/s  kernel %.3f ms  frac %.4f' % (d['value'], r['kernel_ms'], r['frac']))" | tee -a "$OUT/summary.txt"
}
B="python3 bench.py --steps 10 --warmup 2 --no-cpu --no-host"
for agg in trimmedmean median; do
  for n in 128 100; do
    run ${agg}_n${n}_dma2 SRA_DMA_WAVES=2 $B --agg $agg --clients $n
    run ${agg}_n${n}_dma1 SRA_DMA_WAVES=1 $B --agg $agg --clients $n
    run ${agg}_n${n}_reg SRA_SELECT=1 $B --agg $agg --clients $n
  done
done
echo "== done" | tee -a "$OUT/summary.txt"
