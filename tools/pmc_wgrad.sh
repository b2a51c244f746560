#!/bin/bash
# SQ / GRBM counter passes over the weight-gradient microbench (tools/wgrad_bench.py) for the shapes
# in BENCH_ONLY and the modes in BENCH_MODES; summary by tools/pmc_busy.py <tag>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-wgrad}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmcb_${tag}_$i -o run -- \
    python3 tools/wgrad_bench.py > gpurun_out/pmcb_${tag}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmcb_${tag}_$i.log; exit 5; }
done
python tools/pmc_busy.py $tag gpurun_out/${tag}_busy.json
