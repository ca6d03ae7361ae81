#!/bin/bash
# Round 3, session b: filter decision-trace tests + filter tests + solver step statistics.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3b
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_filter_trace.py tests/test_gpu_filters.py > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|error / bound|agreed|chunk [0-9]+: error|passed|failed" "$OUT/pytest.log" | tail -60
[[ $rc -gt 1 ]] && { echo "pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 200 python -u tools/filter_debug.py filterL2_n128_c4 synthetic > "$OUT/fdebug.log" 2>&1 || { echo "filter_debug failed"; tail -5 "$OUT/fdebug.log"; exit 1; }
tail -25 "$OUT/fdebug.log"
