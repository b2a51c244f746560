#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter block each, --kernel-trace only) over bench.py's timed
# steps; tools/pmc_traffic.py --after-marker summarises them
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
model=${1:-reconet}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${model}_$c -o run -- \
    python3 bench.py --model $model --steps 2 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/pmc_${model}_$c.log 2>&1 \
    || { echo "pmc $c failed"; exit 4; }
done
echo pmc done
