set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_dt.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "e2e or hiera or cfg2" > gpurun_out/t_e2e.log 2>&1
for i in 1 2; do
FSMI_DT=0 timeout -k 10 200 python -u bench.py > gpurun_out/ab_old$i.json 2>gpurun_out/ab.err
timeout -k 10 200 python -u bench.py > gpurun_out/ab_new$i.json 2>>gpurun_out/ab.err
done
