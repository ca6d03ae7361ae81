#!/bin/bash
# Round-5 closing GPU session: the whole -m gpu suite, smoke and the default
# bench line (logs under gpurun_out/r5f/).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5f
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log"
# kernel stats + bench lines of the four spectral-filter workloads (gpurun_out/r5g/)
W='filterl2|--agg filterl2 --d 1e7 --steps 3 --warmup 1
ex_noregret|--agg ex_noregret --d 1e7 --steps 3 --warmup 1
mom_filterl2|--agg mom_filterl2 --clients 512 --d 1.25e7 --steps 3 --warmup 1
mom_ex_noregret|--agg mom_ex_noregret --clients 512 --d 1.25e7 --steps 3 --warmup 1' TAG=r5g bash tools/gpu_r5_prof.sh
