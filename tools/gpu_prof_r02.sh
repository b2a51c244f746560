#!/bin/bash
# round-2 profiling pass: new GPU tests, per-layer GEMM timings per mode, SQ counter passes on the
# bf16x6 conv fwd / wgrad of the residual layer, rocprofv3 kernel stats of the headline bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_adaattn.py tests/test_gpu_abi.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -rf --tb=short > gpurun_out/r02p_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r02p_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/gemm_modes.py --modes f32,bf16x6,bf16x3 > gpurun_out/r02p_modes.log 2>&1 || exit $?
export VST_GEMM_POLICY=bf16x6
for which in fwd wgrad; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/r02p_pmc_${which}_$i -o run -- \
      python3 tools/gemm_one.py $which 5 > gpurun_out/r02p_pmc_${which}_$i.log 2>&1 || { echo "pmc $which $i failed"; exit 3; }
  done
done
unset VST_GEMM_POLICY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02p_prof -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/r02p_prof_bench.log 2>&1 || exit $?
echo done
