#!/bin/bash
# bf16x6 halo weight gradient on 32-column strips: tests; config 3 with the residual layers on it (A/B/A/B); config 4
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_halo.py tests/test_gpu_streams.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k3_t.log 2>&1 || { tail -30 gpurun_out/r05k3_t.log; exit 2; }
tail -1 gpurun_out/r05k3_t.log
for r in 1 0 1 0; do
  VST_WGRAD_HALO_RES=$r timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05k3_c3_$r.json 2>/dev/null || exit 5
  echo "halo_res=$r"; python tools/show_bench.py gpurun_out/r05k3_c3_$r.json | head -3
done
timeout -k 10 400 python bench.py --model adaattn --steps 40 --no-cpu-baseline --no-vgg19 > gpurun_out/r05k3_aa4.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r05k3_aa4.json | head -3
