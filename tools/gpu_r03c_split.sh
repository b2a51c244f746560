#!/bin/bash
# GPU suite on the in-tree build, then config 5 with the VGG19 slice-boundary split off / on (A/B/A/B)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/split_tests.log 2>&1 || { tail -40 gpurun_out/split_tests.log; exit 4; }
tail -2 gpurun_out/split_tests.log
for i in 1 2; do
  for v in 0 1; do
    VST_FEATURE_SPLIT=$v timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/split${v}_$i.json 2>/dev/null || exit 5
    python -c "import json;d=json.load(open('gpurun_out/split${v}_$i.json'));print('c5 split=$v', round(d['ms_per_step'],2))"
  done
done
echo done
