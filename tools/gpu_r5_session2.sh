#!/bin/bash
# Round-5 evidence, part 2: traces + FETCH_SIZE / WRITE_SIZE passes of the
# whole-op workloads (filters, Bulyan, Krum family), folded like gpu_r5_session.sh.
set -u
export TAG=${TAG:-r05}
export WORKLOADS="bulyankrum|--agg bulyankrum --d 1e7
bulyanmedian|--agg bulyanmedian --d 1e7 --steps 2
bulyantrimmedmean|--agg bulyantrimmedmean --d 1e7 --steps 2
filterl2|--agg filterl2 --d 1e7 --steps 2
ex_noregret|--agg ex_noregret --d 1e7 --steps 2
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7 --steps 2
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 2
mom_krum|--agg mom_krum --clients 512 --d 1.25e7"
export PMC_WORKLOADS="bulyankrum bulyanmedian bulyantrimmedmean filterl2 ex_noregret mom_filterl2 mom_ex_noregret mom_krum"
bash tools/profile_round.sh || exit 1
bash tools/gpu_pmc_pack.sh "$TAG"
