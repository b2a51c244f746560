#!/bin/bash
# SQ / GRBM counter passes (one per run, --kernel-trace only) over bench.py's timed steps of the
# headline step: MFMA busy share, wait / issue split, LDS and vector-memory instruction counts per
# GEMM family; summarised by tools/pmc_busy.py --after-marker
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
model=${1:-reconet}
# tag adaattn_c5: the AdaAttN step at BASELINE config 5's shape (B=8, 512x1024)
if [ "$model" = adaattn_c5 ]; then args="--model adaattn --batch 8 --height 512 --width 1024"; else args="--model $model"; fi
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmcb_${model}_$i -o run -- \
    python3 bench.py $args --steps 2 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/pmcb_${model}_$i.log 2>&1 \
    || { echo "pmc pass $i failed"; exit 4; }
done
echo pmc busy done
