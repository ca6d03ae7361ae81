#!/bin/bash
# Round 3, session c: Lanczos step microbenchmark, then the filter parity tests.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3c
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 120 tools/ubench/bin/lanczos_step > "$OUT/lanczos_step.txt" 2>&1 || { echo "ubench failed"; cat "$OUT/lanczos_step.txt"; exit 1; }
cat "$OUT/lanczos_step.txt"
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filter_trace.py tests/test_gpu_filters.py > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "decisions compared|error .* of max|not compared|passed|failed|FAILED" "$OUT/pytest.log" | tail -30
exit $rc
