#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes for the whole-op workloads (filters, Bulyan,
# MoM Krum); collect with: python tools/pmc_traffic.py gpurun_out/pmcw r03pmc
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcw
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
W="${PMCW_LIST:-filterl2|--agg filterl2 --d 1e7
ex_noregret|--agg ex_noregret --d 1e7
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7
bulyankrum|--agg bulyankrum --d 1e7
bulyantrimmedmean|--agg bulyantrimmedmean --d 1e7
mom_krum|--agg mom_krum --clients 512 --d 1.25e7}"
while IFS='|' read -r name args; do
  timeout -k 10 300 python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-host $args > "$OUT/$name.log" 2>&1 \
    || { echo "bench $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc_${name}_$c" -o run \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-host $args > "$OUT/pmc_${name}_$c.log" 2>&1 \
      || { echo "pmc $name $c failed rc=$?"; tail -5 "$OUT/pmc_${name}_$c.log"; exit 1; }
  done
  echo "pmc $name ok"
done <<< "$W"
