#!/bin/bash
# order dependence of test_side_streams_bitwise[adaattn-f16]: after the parity tests, with / without
# the skip-gradient tests before them, and with the skip accumulation off
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $P tests/test_gpu_skipgrad.py tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/ord1.log 2>&1; echo "skip+parity+streams rc=$?"; tail -1 gpurun_out/ord1.log
timeout -k 10 300 $P tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/ord2.log 2>&1; echo "parity+streams rc=$?"; tail -1 gpurun_out/ord2.log
VST_SKIP_ACCUM=0 timeout -k 10 300 $P tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/ord3.log 2>&1; echo "parity+streams skip-off rc=$?"; tail -1 gpurun_out/ord3.log
