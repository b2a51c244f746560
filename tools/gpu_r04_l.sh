#!/bin/bash
# halo split-K: tests (bitwise unsplit vs per-tap, split vs unsplit / fp64), the layer shapes on the
# default build (split-K + bf16x6 padded-grid dgrad on the halo kernel) vs libnosplit (round-4 state)
# vs libsplit_pertap (split-K, padded-grid dgrad per-tap); config-4 and config-3 steps on each
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
V=$L/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_parity.py tests/test_gpu_adaattn.py -k 'not reduced_policy and not midsize' -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04l_tests.log 2>&1 || { tail -30 gpurun_out/r04l_tests.log; exit 3; }
tail -1 gpurun_out/r04l_tests.log
for v in default nosplit split_pertap; do
  if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
  VST_LIB_PATH=$LP timeout -k 10 300 python -u -m pytest tests/test_gpu_adaattn.py -k 'reduced_policy or midsize' -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04l_policy_$v.log 2>&1
  echo "$v rc=$?"; grep "policy: loss\|step: loss\|own-norm worst\|passed\|failed" gpurun_out/r04l_policy_$v.log
done
BENCH_ONLY=res,aa4 BENCH_GEMM_MODES=19,20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $V/libnosplit.so $V/libsplit_pertap.so > gpurun_out/r04l_gemm.txt 2>&1 || { cat gpurun_out/r04l_gemm.txt; exit 4; }
cat gpurun_out/r04l_gemm.txt
for v in default nosplit split_pertap; do
  if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
  VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --model adaattn --steps 30 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04l_c4_$v.json 2>/dev/null || exit 6
  echo "$v"; python tools/show_bench.py gpurun_out/r04l_c4_$v.json | head -1
  VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --steps 60 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04l_c3_$v.json 2>/dev/null || exit 7
  echo "$v"; python tools/show_bench.py gpurun_out/r04l_c3_$v.json | head -1
done
echo done
