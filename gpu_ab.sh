set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "halo or e2e_tiny" > gpurun_out/t_halo.log 2>&1
for i in 1 2; do
FSMI_LIB=$GRAFT_REPO_ROOT/foundationstereo_amd/_lib/libfsmi_ab.so timeout -k 10 200 python -u bench.py > gpurun_out/ab_old$i.json 2>gpurun_out/ab.err
timeout -k 10 200 python -u bench.py > gpurun_out/ab_new$i.json 2>>gpurun_out/ab.err
done
