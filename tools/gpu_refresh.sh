#!/bin/bash
# Refresh the bench lines (CPU port timed beside them) and rocprofv3 kernel stats
# of the non-headline workloads.  Outputs under gpurun_out/refresh/.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/refresh
mkdir -p "$OUT"
export TMPDIR=/tmp
W="krum|--agg krum --d 1e7
mom_krum|--agg mom_krum --clients 512 --d 1.25e7
bulyankrum|--agg bulyankrum --d 1e7
bulyanmedian|--agg bulyanmedian --d 1e7 --steps 3
bulyantrimmedmean|--agg bulyantrimmedmean --d 1e7 --steps 3
filterl2|--agg filterl2 --d 1e7 --steps 3
ex_noregret|--agg ex_noregret --d 1e7 --steps 3
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 3
trimmedmean_n512|--agg trimmedmean --clients 512 --d 1.25e7
median_n512|--agg median --clients 512 --d 1.25e7"
while IFS='|' read -r name args; do
  timeout -k 10 240 python "$R/bench.py" --warmup 1 --no-host --cpu-seconds 8 $args > "$OUT/$name.log" 2>&1 \
    || { echo "bench $name failed rc=$?"; exit 1; }
  echo "bench $name ok"
done <<< "$W"
cd /tmp
while IFS='|' read -r name args; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
    -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host $args > "$OUT/prof_$name.log" 2>&1 \
    || { echo "prof $name failed rc=$?"; exit 1; }
  echo "prof $name ok"
done <<< "$W"
