#!/bin/bash
# Round 3, session t: Gram file split -- Krum tests, Krum-family bench refresh.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3t
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_krum.py tests/test_gpu_c3_bulyan.py tests/test_gpu_shard.py > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest: $(grep -E "passed|failed" "$OUT/pytest.log" | tail -1)"
[[ $rc -ne 0 ]] && { grep -E "FAILED|Error" "$OUT/pytest.log" | head; exit $rc; }
bash tools/gpu_refresh.sh krum bulyankrum mom_krum
