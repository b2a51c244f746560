#!/bin/bash
# round-6 diagnosis of the round-5 side-stream difference: the stream tests (with
# the delay-injected and NaN-poisoned variants) and tools/f16_repro.py on this tree and on the reverted
# SkipGrad build checked out and built under variants/skip (git worktree of b160d7c + the test hooks);
# pass --poison-scratch as $1 to fill the private (scratch) slots with NaN before every run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
chk() { case $1 in 124|137|134|139) echo "fatal rc=$1 at $2"; exit 9;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_streams_head.log 2>&1; rc=$?; echo "head streams rc=$rc"; chk $rc head-streams
grep -E "PASS|FAIL" gpurun_out/r06_streams_head.log | cut -c1-150
timeout -k 10 400 python -u tools/f16_repro.py 8 gpurun_out/r06_f16_repro_head.json $1 > gpurun_out/r06_f16_repro_head.log 2>&1; rc=$?; echo "head repro rc=$rc"; chk $rc head-repro
grep differ gpurun_out/r06_f16_repro_head.log | cut -c1-200
cd variants/skip
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > ../../gpurun_out/r06_streams_skip.log 2>&1; rc=$?; echo "skip streams rc=$rc"; chk $rc skip-streams
grep -E "PASS|FAIL" ../../gpurun_out/r06_streams_skip.log | cut -c1-150
timeout -k 10 400 python -u tools/f16_repro.py 8 ../../gpurun_out/r06_f16_repro_skip.json $1 > ../../gpurun_out/r06_f16_repro_skip.log 2>&1; rc=$?; echo "skip repro rc=$rc"; chk $rc skip-repro
grep differ ../../gpurun_out/r06_f16_repro_skip.log | cut -c1-200
echo done
