#!/bin/bash
# one-pass LDS InstanceNorm backward: parity tests, microbench vs the closing build, config-3 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k instance_norm > gpurun_out/in_tests.log 2>&1 || { tail -30 gpurun_out/in_tests.log; exit 4; }
tail -2 gpurun_out/in_tests.log
timeout -k 10 300 python tools/norm_bench.py video-style-transfer_amd/vst/libvst_hip.so variants/r5c/video-style-transfer_amd/vst/libvst_hip.so > gpurun_out/in_bench.log 2>&1 || { tail -30 gpurun_out/in_bench.log; exit 5; }
cat gpurun_out/in_bench.log
bash tools/gpu_r05_ab.sh
