#!/bin/bash
# full GPU suite without stopping at the first failure (diagnostics)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf --tb=line > gpurun_out/gpu_tests_all.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests_all.log
tail -40 gpurun_out/gpu_tests_all.log
