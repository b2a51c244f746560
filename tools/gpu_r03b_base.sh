#!/bin/bash
# session-2 baseline of round 3: config-5 and config-3 rocprofv3 kernel summaries on HEAD
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b5_prof -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/b5_prof.log 2>&1 || exit 6
python tools/prof_summary.py gpurun_out/b5_prof 12 -shapes > gpurun_out/b5_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b3_prof -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/b3_prof.log 2>&1 || exit 8
python tools/prof_summary.py gpurun_out/b3_prof 30 -shapes > gpurun_out/b3_summary.txt 2>&1
echo done
