#!/bin/bash
# depth-2 prefetch (VST_PF2) for the single-/two-term conv GEMMs: correctness (conv unit tests in
# every mode), the f16 NaN locator, then the config-5 step main / PF2=0 / main / PF2=0 on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "conv_fwd_bwd" > gpurun_out/r03_pf2_tests.log 2>&1 || exit 3
timeout -k 10 200 python tools/nan_diag.py > gpurun_out/r03_nan.log 2>&1 || exit 4
L=video-style-transfer_amd/vst/libvst_hip.so
cp $L /tmp/libvst_main.so || exit 2
i=0
for lib in /tmp/libvst_main.so variants/libvst_pf0.so /tmp/libvst_main.so variants/libvst_pf0.so; do
  i=$((i+1))
  cp $lib $L || exit 2
  timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 --gemm bf16 > gpurun_out/r03_pf2_ab_$i.json 2>/dev/null || { cp /tmp/libvst_main.so $L; exit 5; }
done
cp /tmp/libvst_main.so $L
echo done
