#!/bin/bash
# Round-5 evidence session on the GPU box (from the repo root):
#   PART=trace  kernel-trace --stats + the bench line of every workload
#   PART=pmc    FETCH_SIZE / WRITE_SIZE passes of $PMC_WORKLOADS
# then folds them into profiles/ (kernel stats, bench json, traffic.json) and
# copies what is kept to gpurun_out/keep/ (tools/gpu_pmc_pack.sh).
set -u
export TAG=${TAG:-r05}
export WORKLOADS="default|
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
bulyanmedian|--agg bulyanmedian --d 1e7 --steps 2
bulyantrimmedmean|--agg bulyantrimmedmean --d 1e7 --steps 2
filterl2|--agg filterl2 --d 1e7 --steps 2
ex_noregret|--agg ex_noregret --d 1e7 --steps 2
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7 --steps 2
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 2"
if [ "${PART:-trace}" = "trace" ]; then
  export PMC_WORKLOADS=""
else
  export PMC_WORKLOADS=${PMC_WORKLOADS:-"filterl2 ex_noregret mom_filterl2 mom_ex_noregret bulyankrum bulyanmedian bulyantrimmedmean krum"}
  W2=""
  for n in $PMC_WORKLOADS; do W2="$W2$(printf '%s\n' "$WORKLOADS" | awk -F'|' -v n="$n" '$1==n')"$'\n'; done
  export WORKLOADS="$W2"
  export SKIP_TRACE=1
fi
bash tools/profile_round.sh || exit 1
bash tools/gpu_pmc_pack.sh "$TAG"
