#!/bin/bash
# Round-4 closing GPU session: the -m gpu files touched by the client-ceiling
# work, then the whole suite, smoke, the default bench line and two N > 512
# bench lines (logs under gpurun_out/r4f/).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4f
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log"
timeout -k 10 300 python -u bench.py --no-cpu --no-host --agg krum --clients 1024 --d 1e6 --byzantine 100 --steps 5 > "$OUT/bench_krum_n1024.log" 2>&1 || { tail -5 "$OUT/bench_krum_n1024.log"; exit 1; }
tail -1 "$OUT/bench_krum_n1024.log"
timeout -k 10 300 python -u bench.py --no-cpu --no-host --agg bulyanmedian --clients 600 --d 1e6 --byzantine 40 --steps 2 --warmup 1 > "$OUT/bench_bulyanmedian_n600.log" 2>&1 || { tail -5 "$OUT/bench_bulyanmedian_n600.log"; exit 1; }
tail -1 "$OUT/bench_bulyanmedian_n600.log"
