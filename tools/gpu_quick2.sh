#!/bin/bash
# conv-kernel iteration: conv/op parity tests + per-layer GEMM timings (f32, bf16x6)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "${TESTK:-conv or abi or golden}" > gpurun_out/q2_tests.log 2>&1 || { tail -30 gpurun_out/q2_tests.log; exit 1; }
tail -2 gpurun_out/q2_tests.log
timeout -k 10 300 python tools/gemm_modes.py --modes ${MODES:-f32,bf16x6} --what ${WHAT:-fwd,dgrad,wgrad} > gpurun_out/q2_modes.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/q2_modes.log
