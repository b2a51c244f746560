#!/bin/bash
# 192-row layers on the 2x2 one-buffer halo block: halo tests; the bf16x6 residual padded-grid data
# gradient on the halo kernel (default) vs per-tap (libpadout_pertap), config-3 steps A/B/A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=video-style-transfer_amd/vst/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04s_tests.log 2>&1 || { tail -30 gpurun_out/r04s_tests.log; exit 3; }
tail -1 gpurun_out/r04s_tests.log
for i in 1 2; do
  for v in default padout_pertap; do
    if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
    VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --steps 60 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04s_c3_${v}_$i.json 2>/dev/null || exit 7
    echo "$v"; python tools/show_bench.py gpurun_out/r04s_c3_${v}_$i.json | head -1
  done
done
echo done
