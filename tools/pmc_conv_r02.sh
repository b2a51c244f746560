#!/bin/bash
# SQ / GRBM PMC passes over tools/gemm_one.py for the conv tile variants of the headline step
# (bf16x6 policy): MFMA busy share, issue stalls, effective clock (GRBM_GUI_ACTIVE / 8 / wall).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
export VST_GEMM_POLICY=${VST_GEMM_POLICY:-bf16x6}
for which in ${@:-vgg1 vgg3kb fwd}; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmcc_${which}_$i -o run -- \
      python3 tools/gemm_one.py $which 8 > gpurun_out/pmcc_${which}_$i.log 2>&1 || { echo "pass $which $i failed"; exit 3; }
  done
done
echo "pmc conv done"
