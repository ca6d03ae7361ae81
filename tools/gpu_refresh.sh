#!/bin/bash
# Refresh every bench line (CPU port timed beside it) and its rocprofv3 kernel
# stats.  Outputs under gpurun_out/refresh/<name>.log and prof_<name>/.
# usage: bash tools/gpu_refresh.sh [name ...]   (default: all)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/refresh
mkdir -p "$OUT"
export TMPDIR=/tmp
W="default|--agg trimmedmean --steps 20
median|--agg median --steps 20
average|--agg average --steps 20
c2_trimmedmean_d1e6|--agg trimmedmean --d 1e6 --steps 50
trimmedmean_n100|--agg trimmedmean --clients 100 --steps 20
median_n100|--agg median --clients 100 --steps 20
trimmedmean_n512|--agg trimmedmean --clients 512 --d 1.25e7
median_n512|--agg median --clients 512 --d 1.25e7
krum|--agg krum --d 1e7
mom_krum|--agg mom_krum --clients 512 --d 1.25e7
bulyankrum|--agg bulyankrum --d 1e7
bulyanmedian|--agg bulyanmedian --d 1e7 --steps 3
bulyantrimmedmean|--agg bulyantrimmedmean --d 1e7 --steps 3
filterl2|--agg filterl2 --d 1e7 --steps 3
ex_noregret|--agg ex_noregret --d 1e7 --steps 3
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 3"
want=" $* "
while IFS='|' read -r name args; do
  if [ $# -gt 0 ] && [[ "$want" != *" $name "* ]]; then continue; fi
  extra="--no-host"
  [ "$name" = default ] && extra=""
  timeout -k 10 300 python "$R/bench.py" --warmup 2 --cpu-seconds 8 $extra $args > "$OUT/$name.log" 2>&1 \
    || { echo "bench $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "bench $name ok: $(python3 -c "import json;d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['roofline']['frac'])")"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
    -- python3 "$R/bench.py" --warmup 1 --no-cpu --no-host $args > "$OUT/prof_$name.log" 2>&1) \
    || { echo "prof $name failed rc=$?"; exit 1; }
  rm -f "$OUT/prof_$name"/run_kernel_trace.csv "$OUT/prof_$name"/run_agent_info.csv   # keep the stats (<64 MiB back)
  echo "prof $name ok"
done <<< "$W"
