#!/bin/bash
# usage: gpu_ab_wg.sh "VAR=v,VAR2=v2" "VAR=w" ... -- per environment setting (in the order given, so
# A/B/A orders are possible): weight-gradient microbench, the GPU suite, and the headline step
# (no CPU baseline / VGG19 sub-metric)
cd $GRAFT_REPO_ROOT
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=$(echo "$cfg" | tr ',' ' ')
  tag=$(echo "$cfg" | tr ',=' '_-')
  env $envs timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/wg_${i}_$tag.log 2>&1 || exit 3
  env $envs timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wg_tests_${i}_$tag.log 2>&1 || exit 4
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-vgg19 --steps 100 > gpurun_out/wg_bench_${i}_$tag.json 2>/dev/null || exit 5
done
echo ok
