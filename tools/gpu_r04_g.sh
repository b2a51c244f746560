#!/bin/bash
# halo block-shape variants (default / a: 2x4 one-buffer everywhere / b: 4x2 one-buffer for 128- and
# 256-row layers / c: one-buffer tiles at 3 waves per SIMD), the new GPU tests (HIP data-parallel
# step, AdaAttN API blocks, decoder K order), and the config-5 parity measurements
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_ONLY=vgg,res BENCH_GEMM_MODES=19,20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $L/variants/liba.so $L/variants/libb.so $L/variants/libc.so > gpurun_out/r04g_gemm.txt 2>&1 || { cat gpurun_out/r04g_gemm.txt; exit 3; }
cat gpurun_out/r04g_gemm.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_adaattn_api.py tests/test_gpu_halo.py tests/test_gpu_adaattn.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04g_tests.log 2>&1 || { tail -40 gpurun_out/r04g_tests.log; exit 4; }
tail -2 gpurun_out/r04g_tests.log
timeout -k 10 600 python -u tools/f16_parity_diag.py f16 bf16 > gpurun_out/r04g_f16diag.json 2> gpurun_out/r04g_f16diag.err || { tail -20 gpurun_out/r04g_f16diag.err; exit 5; }
cat gpurun_out/r04g_f16diag.json
echo done
