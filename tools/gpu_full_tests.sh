#!/bin/bash
# the whole -m gpu suite (as the driver runs it), log under gpurun_out/full/
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/full
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
grep -E "PASSED|FAILED|ERROR" "$OUT/pytest.log" | awk '{print $NF}' | sort | uniq -c
exit $rc
