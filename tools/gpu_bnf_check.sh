set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bn_fused.py tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_config_parity.py > gpurun_out/t_bnf.log 2>&1
bash tools/gpu_ab_flag.sh FUSED_BN_FWD
bash tools/gpu_ab_flag.sh FUSED_BN_BWD
