#!/bin/bash
# Round profiling session (run on the GPU box from the repo root):
#   kernel-trace --stats of bench.py per workload (the bench's own defaults:
#   20 timed launches after 3 warmup ones, unless a workload sets --steps), a
#   steady-state summary of the trace (tools/steady_stats.py: the average over
#   the timed launches beside rocprof's all-launch average), then FETCH_SIZE / WRITE_SIZE
#   passes (each its own rocprofv3 run, --kernel-trace only) for the HBM-bound
#   kernels.  Outputs under gpurun_out/$TAG/.  Stops at the first failure.
set -u
TAG=${TAG:-prof_r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
WORKLOADS=${WORKLOADS:-"trimmedmean|--agg trimmedmean
c2_trimmedmean_d1e6|--agg trimmedmean --d 1e6
median|--agg median
average|--agg average
trimmedmean_n100|--agg trimmedmean --clients 100
median_n100|--agg median --clients 100
trimmedmean_n512|--agg trimmedmean --clients 512 --d 1.25e7
median_n512|--agg median --clients 512 --d 1.25e7
krum|--agg krum --d 1e7
mom_krum|--agg mom_krum --clients 512 --d 1.25e7
bulyankrum|--agg bulyankrum --d 1e7
bulyanmedian|--agg bulyanmedian --d 1e7
bulyantrimmedmean|--agg bulyantrimmedmean --d 1e7
filterl2|--agg filterl2 --d 1e7
ex_noregret|--agg ex_noregret --d 1e7
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7"}
PMC_WORKLOADS=${PMC_WORKLOADS:-"trimmedmean median average trimmedmean_n100 trimmedmean_n512 median_n512 krum bulyanmedian bulyantrimmedmean"}
while IFS='|' read -r name args; do
  [[ -z "$name" ]] && continue
  [ -n "${SKIP_TRACE:-}" ] && continue
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/$name" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu --no-host $args > "$OUTD/$name.log" 2>&1 \
    || { echo "trace $name failed rc=$?"; exit 1; }
  steps=$(printf '%s\n' "$args" | sed -n 's/.*--steps \([0-9]*\).*/\1/p')
  tr=$(find "$OUTD/$name" -name '*kernel_trace.csv' | head -1)
  [ -n "$tr" ] && python3 "$ROOT/tools/steady_stats.py" "$tr" "${steps:-20}" > "$OUTD/$name.steady.txt"
  # keep the summaries only (gpurun copies back at most 64 MiB)
  find "$OUTD/$name" -type f ! -name '*kernel_stats.csv' -delete
  echo "trace $name ok"
done <<< "$WORKLOADS"
for name in $PMC_WORKLOADS; do
  args=$(printf '%s\n' "$WORKLOADS" | awk -F'|' -v n="$name" '$1==n{print $2}')
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUTD/pmc_${name}_$ctr" -o run \
      -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-host $args > "$OUTD/pmc_${name}_$ctr.log" 2>&1 \
      || { echo "pmc $name $ctr failed rc=$?"; exit 1; }
    # the counter rows of this library's kernels only
    for f in $(find "$OUTD/pmc_${name}_$ctr" -name '*counter_collection.csv'); do
      python3 -c "import csv,sys; r=list(csv.reader(open(sys.argv[1]))); k=r[0].index('Kernel_Name'); w=csv.writer(open(sys.argv[1],'w',newline='')); w.writerow(r[0]); [w.writerow(x) for x in r[1:] if 'sra::' in x[k]]" "$f"
    done
    find "$OUTD/pmc_${name}_$ctr" -type f ! -name '*counter_collection.csv' -delete
    echo "pmc $name $ctr ok"
  done
done
echo done
