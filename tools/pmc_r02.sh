#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter block each, --kernel-trace only) over bench.py's timed
# steps; tools/pmc_traffic.py --after-marker summarises them
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
model=${1:-reconet}
# tag adaattn_c5: the AdaAttN step at BASELINE config 5's shape (B=8, 512x1024)
if [ "$model" = adaattn_c5 ]; then args="--model adaattn --batch 8 --height 512 --width 1024"; else args="--model $model"; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${model}_$c -o run -- \
    python3 bench.py $args --steps 2 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/pmc_${model}_$c.log 2>&1 \
    || { echo "pmc $c failed"; exit 4; }
done
echo pmc done
