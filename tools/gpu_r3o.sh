#!/bin/bash
# Round 3, session o: eigenvector chains from registers: check ubench, filter parity + traces, filterl2 bench.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3o
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R/tools/ubench" && mkdir -p bin && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bin/check_bench check_bench.hip ../../secure-robust-federated-learning_amd/csrc/common.hip > "$OUT/cb_build.log" 2>&1 && timeout -k 10 120 bin/check_bench > "$OUT/check_bench.txt" 2>&1; grep warm "$OUT/check_bench.txt" | tail -4
cd "$R"
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filters.py tests/test_gpu_filter_trace.py tests/test_gpu_dba.py > "$OUT/pytest_filters.log" 2>&1
rc=$?
grep -E "decisions compared|error / bound|passed|failed|FAILED" "$OUT/pytest_filters.log" | tail -14
[[ $rc -gt 1 ]] && { echo "filter pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 200 python -u tools/filter_debug.py filterL2_n128_c4 synthetic > "$OUT/fdebug.log" 2>&1 && grep -E "mode|cycles|d=" "$OUT/fdebug.log" | tail -10
cd /tmp
timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg filterl2 --d 1e7 --steps 3 > "$OUT/fl.log" 2>&1 && echo "filterl2 $(grep '"metric"' "$OUT/fl.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
timeout -k 10 200 python3 "$R/bench.py" --warmup 1 --no-cpu --no-host --agg mom_filterl2 --clients 512 --d 1.25e7 --steps 2 > "$OUT/mfl.log" 2>&1 && echo "mom_filterl2 N=512 d=1.25e7 $(grep '"metric"' "$OUT/mfl.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
