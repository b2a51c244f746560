#!/bin/bash
# rocprofv3 kernel-trace summaries + separate PMC passes (FETCH_SIZE, WRITE_SIZE) for one gpurun call.
# usage: tools/prof_pipeline.sh [reconet|adaattn] [stats|pmc|all]
set -o pipefail
model=${1:-reconet}
what=${2:-all}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
args="--model $model --steps 3 --warmup 1 --no-cpu-baseline --no-vgg19 --gemm ${GEMM:-parity}"
if [ "$what" == "stats" ] || [ "$what" == "all" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$model -o run -- \
    python3 bench.py $args > gpurun_out/prof_$model.log 2>&1 || { echo "stats pass failed rc=$?"; exit 3; }
fi
if [ "$what" == "pmc" ] || [ "$what" == "all" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 500 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${model}_$c -o run -- \
      python3 bench.py --model $model --steps 1 --warmup 1 --no-cpu-baseline --no-vgg19 --gemm ${GEMM:-parity} > gpurun_out/pmc_${model}_$c.log 2>&1 \
      || { echo "pmc $c pass failed rc=$?"; exit 4; }
  done
fi
echo "prof pipeline done"
