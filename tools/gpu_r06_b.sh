#!/bin/bash
# round-6 check of the stream / scratch diagnosis and the ATen-free step: full GPU suite, the f16
# reproducibility run with scratch poisoning on HEAD and on the reverted SkipGrad build
# (variants/skip), and a short rocprofv3 kernel summary of the config-3 step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
chk() { case $1 in 124|137|134|139) echo "fatal rc=$1 at $2"; exit 9;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf --tb=short > gpurun_out/r06b_tests.log 2>&1; rc=$?; echo "suite rc=$rc"; chk $rc suite
grep -E "FAILED|passed|failed" gpurun_out/r06b_tests.log | tail -12
timeout -k 10 400 python -u tools/f16_repro.py 4 gpurun_out/r06_f16_repro_head_poison.json --poison-scratch > gpurun_out/r06_f16_repro_head_poison.log 2>&1; rc=$?; echo "head poison rc=$rc"; chk $rc head-poison
grep differ gpurun_out/r06_f16_repro_head_poison.log | cut -c1-220
(cd variants/skip && timeout -k 10 400 python -u tools/f16_repro.py 4 ../../gpurun_out/r06_f16_repro_skip_poison.json --poison-scratch > ../../gpurun_out/r06_f16_repro_skip_poison.log 2>&1); rc=$?; echo "skip poison rc=$rc"; chk $rc skip-poison
grep differ gpurun_out/r06_f16_repro_skip_poison.log | cut -c1-220
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06b_prof3 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r06b_prof3.log 2>&1; rc=$?; echo "prof rc=$rc"; chk $rc prof
python tools/prof_summary.py gpurun_out/r06b_prof3 12 -shapes > gpurun_out/r06b_kernel_summary.txt 2>&1; cp gpurun_out/r06b_prof3/run_kernel_stats.csv gpurun_out/r06b_kernel_stats.csv; rm -rf gpurun_out/r06b_prof3
head -3 gpurun_out/r06b_kernel_summary.txt; grep -c native gpurun_out/r06b_kernel_stats.csv
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err; rc=$?; echo "bench rc=$rc"; chk $rc bench
python tools/show_bench.py gpurun_out/r06b_bench.json | head -2
echo done
