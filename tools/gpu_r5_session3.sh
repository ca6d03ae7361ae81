#!/bin/bash
# Round-5 evidence, part 3: the spectral-filter workloads again after the
# PRO prefetch and the float4 bucket fill (traces + traffic passes).
set -u
export TAG=${TAG:-r05}
export WORKLOADS="filterl2|--agg filterl2 --d 1e7 --steps 2
ex_noregret|--agg ex_noregret --d 1e7 --steps 2
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7 --steps 2
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 2"
export PMC_WORKLOADS="filterl2 ex_noregret mom_filterl2 mom_ex_noregret"
bash tools/profile_round.sh || exit 1
bash tools/gpu_pmc_pack.sh "$TAG"
