set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "halo or rejects" > gpurun_out/t_halo.log 2>&1
timeout -k 10 600 python -u tools/tune_conv.py --only-cfgs 8 9 --out gpurun_out/fsmi_conv_89.json > gpurun_out/tune89.log 2>&1
for i in 1 2; do
timeout -k 10 200 python -u bench.py > gpurun_out/ab_old$i.json 2>gpurun_out/ab.err
FSMI_TUNE_PATH=gpurun_out/fsmi_conv_89.json timeout -k 10 200 python -u bench.py > gpurun_out/ab_new$i.json 2>>gpurun_out/ab.err
done
