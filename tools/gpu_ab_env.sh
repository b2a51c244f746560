#!/bin/bash
# A/B of a Python-layer switch (vst/ops.py VST_* variables) on one box, interleaved:
#   tools/gpu_ab_env.sh TAG VAR "BENCH ARGS" VALUE1 VALUE2 ...   -> gpurun_out/ab_TAG_<rep>_<value>.json
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; VAR=$2; ARGS=$3; shift 3
for rep in 1 2; do
  for v in "$@"; do
    out=gpurun_out/ab_${TAG}_${rep}_${v}.json
    env $VAR=$v timeout -k 10 300 python bench.py $ARGS > $out 2> ${out%.json}.err
    rc=$?; case $rc in 0) ;; *) echo "bench rc=$rc ($VAR=$v)"; exit 9;; esac
    python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('$rep $VAR=$v', round(d['value'],2), round(d['ms_per_step'],2))"
  done
done
