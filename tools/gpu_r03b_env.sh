#!/bin/bash
# usage: gpu_r03b_env.sh VAR -- the GPU suite, then the config-5 step with VAR=1 / VAR=0 / VAR=1 /
# VAR=0 (run-time A/B switch of the in-tree build), and the config-4 step once each way
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VAR=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/env_tests.log 2>&1 || exit 4
B5="--model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19"
B4="--model adaattn --steps 30 --prof-steps 0 --no-cpu-baseline --no-vgg19"
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  env $VAR=$v timeout -k 10 300 python bench.py $B5 > gpurun_out/env5_${v}_$i.json 2> gpurun_out/env5_$i.err || exit 5
done
for v in 1 0; do
  env $VAR=$v timeout -k 10 300 python bench.py $B4 > gpurun_out/env4_$v.json 2> gpurun_out/env4_$v.err || exit 6
done
echo ok
