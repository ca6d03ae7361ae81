set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bulyan.py tests/test_gpu_dispatch.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_bul.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_bul.log; [ $rc -eq 0 ] || exit $rc
for agg in bulyantrimmedmean bulyanmedian; do
  timeout -k 10 300 python bench.py --agg $agg --d 1e7 --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/bench_$agg.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$agg.log | cut -c1-400
done
timeout -k 10 300 env SRA_BULYAN_ROWLIST=1 python bench.py --agg bulyantrimmedmean --d 1e7 --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/bench_rowlist.log 2>&1 || exit 1
tail -1 gpurun_out/bench_rowlist.log | cut -c1-300
