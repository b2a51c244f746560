#!/bin/bash
# round-2 GPU pass: full GPU suite (no -x, report every failure), headline bench, f32-policy bench
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf --tb=short > gpurun_out/r02_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r02_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/r02_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gemm f32 --no-cpu-baseline --steps 60 > gpurun_out/r02_bench_f32.log 2>&1 || exit $?
tail -3 gpurun_out/r02_tests.log
