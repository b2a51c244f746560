#!/bin/bash
# GPU tests (stop at first failure) + bench per GEMM policy; usage: tools/gpu_run.sh [policies...]
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf --tb=line > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -8
pols=${@:-parity}
for p in $pols; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --gemm $p > gpurun_out/bench_$p.log 2>&1 || { echo "bench $p failed"; tail -5 gpurun_out/bench_$p.log; exit 2; }
  grep -v amdgpu.ids gpurun_out/bench_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; v=d.get('north_star_vgg19',{}); print('$p', 'value %.1f ms %.1f conv %.1f TF peak %.0f frac %.3f' % (d['value'], d['ms_per_step'], r['achieved'], r['peak'], r['frac']), 'vgg19 %.1f TF wall %.1f' % (v.get('conv_tflops',0), v.get('wall_tflops',0)), {k: round(x['tflops'],1) for k, x in r['by_mode'].items()})"
done
