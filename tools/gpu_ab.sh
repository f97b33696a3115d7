set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pool2x or e2e or update" > gpurun_out/t_pool.log 2>&1
for i in 1 2; do
FSMI_POOL_TORCH=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_old$i.json 2>gpurun_out/ab.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_new$i.json 2>>gpurun_out/ab.err
done
