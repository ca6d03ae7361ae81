#!/bin/bash
# A/B of the k-select launch variants (trimmed mean N=128 / 100, median N=128,
# d=1e8): register path (block 256 / 768), two-lane path (block 256 / 1024).
set -u
OUT=${OUT:-gpurun_out/ab_select}
mkdir -p "$OUT"
run() { # name env...
  local name=$1; shift
  echo "== $name" | tee -a "$OUT/summary.txt"
  timeout -k 10 240 env "$@" > "$OUT/$name.log" 2>&1 || { echo "FAILED $name rc=$?" | tee -a "$OUT/summary.txt"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('  value %.1f GB/s  kernel %.3f ms  frac %.4f' % (d['value'], r['kernel_ms'], r['frac']))" | tee -a "$OUT/summary.txt"
}
B="python3 bench.py --steps 10 --warmup 2 --no-cpu --no-host"
for cfg in "trimmedmean 128" "trimmedmean 100" "median 128"; do
  set -- $cfg
  agg=$1; n=$2
  run ${agg}_n${n}_reg256 SRA_SELECT=1 SRA_BS=256 $B --agg $agg --clients $n
  run ${agg}_n${n}_reg768 SRA_SELECT=1 SRA_BS=768 $B --agg $agg --clients $n
done
echo "== done" | tee -a "$OUT/summary.txt"
