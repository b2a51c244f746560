#!/bin/bash
# rocprofv3 kernel summary of the config-5 step (AdaAttN, B=8, 512x1024, f16 policy)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p5_prof -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/p5_prof.log 2>&1 || exit 6
python tools/prof_summary.py gpurun_out/p5_prof 10 -shapes > gpurun_out/p5_summary.txt 2>&1
echo done
