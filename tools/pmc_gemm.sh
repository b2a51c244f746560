#!/bin/bash
# PMC passes (SQ counters) over tools/gemm_one.py for one GEMM flavour; separate runs per pass,
# --kernel-trace only besides --pmc.
set -o pipefail
which=${1:-fwd}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmcg_${which}_$i -o run -- \
    python3 tools/gemm_one.py $which 5 > gpurun_out/pmcg_${which}_$i.log 2>&1 || { echo "pass $i failed"; exit 3; }
done
echo "pmc gemm done"
