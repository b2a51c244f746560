#!/bin/bash
# per-kernel rocprofv3 summaries of the config-3 step: round-4 tree vs HEAD (side streams off), plus
# HEAD with the row-tiled weight gradient and with one replayed input batch
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0
(cd variants/r4 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/r05h_p4 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05h_p4.log 2>&1) || exit 3
python tools/prof_summary.py gpurun_out/r05h_p4 12 -shapes > gpurun_out/r05h_r4_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05h_p5 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r05h_p5.log 2>&1 || exit 4
python tools/prof_summary.py gpurun_out/r05h_p5 12 -shapes > gpurun_out/r05h_head_summary.txt 2>&1
head -50 gpurun_out/r05h_r4_summary.txt
echo ====
head -50 gpurun_out/r05h_head_summary.txt
rm -rf gpurun_out/r05h_p4 gpurun_out/r05h_p5
