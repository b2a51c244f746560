#!/bin/bash
# rest of the round-5 counter set (the reconet traffic pass is in; busy passes re-summarised)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_r05.sh adaattn_c5 both || exit 5
python tools/pmc_traffic.py adaattn_c5 gpurun_out/r05_traffic_adaattn_c5.json --after-marker > /dev/null && \
python tools/pmc_busy.py adaattn_c5 gpurun_out/r05_mfma_busy_adaattn_c5.json || exit 6
bash tools/pmc_r05.sh reconet_f32 traffic || exit 7
python tools/pmc_traffic.py reconet_f32 gpurun_out/r05_traffic_reconet_f32.json --after-marker > /dev/null || exit 8
bash tools/pmc_r05.sh adaattn traffic || exit 9
python tools/pmc_traffic.py adaattn gpurun_out/r05_traffic_adaattn.json --after-marker > /dev/null || exit 10
rm -rf gpurun_out/pmc_* gpurun_out/pmcb_*
echo done
