#!/bin/bash
# Round 3, session a: VALU issue-rate microbenchmarks (1/2/4/8 waves per SIMD)
# and PMC of the spectral-filter solver kernels (one 2000-chunk batch each).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 "$R/tools/ubench/bin/valu_rate" > "$OUT/valu_rate.txt" 2>&1 || { echo "valu_rate failed"; exit 1; }
cat "$OUT/valu_rate.txt"
timeout -k 10 120 "$R/tools/ubench/bin/valu_rate2" > "$OUT/valu_rate2.txt" 2>&1 || { echo "valu_rate2 failed"; exit 1; }
cd /tmp
i=0
for agg in filterl2 ex_noregret; do
  while read -r counters; do
    [[ -z "$counters" ]] && continue
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d "$OUT/pmc_$agg/p$i" -o run \
      -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-host --agg $agg --d 2e6 > "$OUT/pmc_${agg}_$i.log" 2>&1 \
      || { echo "pmc $agg pass $i failed"; tail -3 "$OUT/pmc_${agg}_$i.log"; exit 1; }
    echo "pmc $agg pass $i ok"
  done <<PASSES
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES
PASSES
done
cd "$R"
python3 tools/pmc_summary.py "$OUT/pmc_filterl2" "$OUT/pmc_ex_noregret" > "$OUT/pmc_summary.txt" 2>&1
grep -A30 "solve" "$OUT/pmc_summary.txt" | head -80
echo done
