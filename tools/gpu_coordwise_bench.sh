set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coordwise.py tests/test_gpu_dispatch.py tests/test_gpu_bulyan.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cw.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_cw.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for agg in trimmedmean median; do
  for n in 128 100; do
    timeout -k 10 200 python bench.py --agg $agg --clients $n --steps 20 --warmup 3 --no-cpu --no-host > gpurun_out/b.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$agg N=$n', d['ms_per_step'], r['kernel_ms'], r['frac'])"
  done
done
done
