#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_ddp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k_tests.log 2>&1 || { tail -40 gpurun_out/r05k_tests.log; exit 3; }
tail -1 gpurun_out/r05k_tests.log
for i in 1 2; do
  (cd variants/r4 && timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05k_r4_$i.json 2>/dev/null) || exit 5
  python tools/show_bench.py gpurun_out/r05k_r4_$i.json | head -1
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05k_head_$i.json 2> gpurun_out/r05k_head.err || exit 6
  python tools/show_bench.py gpurun_out/r05k_head_$i.json | head -1
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 --replay-input > gpurun_out/r05k_replay_$i.json 2> gpurun_out/r05k_head.err || exit 6
  python tools/show_bench.py gpurun_out/r05k_replay_$i.json | head -1
done
export VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05k_p5 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r05k_p5.log 2>&1 || exit 4
python tools/prof_summary.py gpurun_out/r05k_p5 12 -shapes > gpurun_out/r05k_head_summary.txt 2>&1
grep -E "total|warp|wgrad_halo|family" gpurun_out/r05k_head_summary.txt
rm -rf gpurun_out/r05k_p5
