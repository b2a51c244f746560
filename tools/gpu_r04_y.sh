#!/bin/bash
# 3 vs 4 waves/SIMD for the single-product one-buffer halo tiles (libsminw3 vs default): config-5
# steps A/B/A/B on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=video-style-transfer_amd/vst/variants
for i in 1 2; do
  for v in default sminw3; do
    if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
    VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04y_c5_${v}_$i.json 2>/dev/null || exit 6
    echo "$v"; python tools/show_bench.py gpurun_out/r04y_c5_${v}_$i.json | head -1
  done
done
echo done
