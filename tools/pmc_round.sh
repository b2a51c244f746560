#!/bin/bash
# counter passes (one per run, --kernel-trace only, each under its own time limit) over bench.py's
# timed steps: FETCH_SIZE / WRITE_SIZE (HBM traffic, tools/pmc_traffic.py) and two SQ/GRBM sets
# (MFMA busy and instruction mix, tools/pmc_busy.py).  usage: pmc_round.sh <model tag> [traffic|busy|both]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
model=${1:-reconet}
what=${2:-both}
case $model in
  adaattn_c5) args="--model adaattn --batch 8 --height 512 --width 1024" ;;
  reconet_f32) args="--model reconet --gemm f32" ;;
  *) args="--model $model" ;;
esac
if [ "$what" != busy ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${model}_$c -o run -- \
      python3 bench.py $args --steps 2 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/pmc_${model}_$c.log 2>&1 \
      || { echo "pmc $c failed"; exit 4; }
  done
fi
if [ "$what" != traffic ]; then
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmcb_${model}_$i -o run -- \
      python3 bench.py $args --steps 2 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/pmcb_${model}_$i.log 2>&1 \
      || { echo "pmc busy pass $i failed"; exit 5; }
  done
fi
echo pmc $model done
