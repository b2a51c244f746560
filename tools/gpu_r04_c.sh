#!/bin/bash
# halo vs per-tap conv kernel per layer shape (bf16x6 19/51, fp16 20/52), then SQ counters of one
# VGG conv3 shape under each kernel
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst/libvst_hip.so
BENCH_GEMM_MODES=19,51,20,52 timeout -k 10 300 python tools/gemm_bench.py $L > gpurun_out/r04c_gemm.txt 2>&1 || { cat gpurun_out/r04c_gemm.txt; exit 3; }
cat gpurun_out/r04c_gemm.txt
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  BENCH_ONLY=vgg3_2.fwd BENCH_GEMM_MODES=19,51 timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/r04c_pmc_$i -o run -- \
    python3 tools/gemm_bench.py $L > gpurun_out/r04c_pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail gpurun_out/r04c_pmc_$i.log; exit 4; }
done
echo done
