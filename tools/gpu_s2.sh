cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf --tb=short -k "conv and s2" > gpurun_out/s2_tests.log 2>&1 && \
timeout -k 10 200 python tools/gemm_modes.py --modes bf16x3 --only conv --what dgrad > gpurun_out/s2_modes.log 2>&1 && \
bash tools/gpu_run.sh parity
