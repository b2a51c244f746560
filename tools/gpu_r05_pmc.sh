#!/bin/bash
# round-5 counter set: HBM traffic (FETCH/WRITE) of the headline (bf16x6), strict
# f32, config-4 and config-5 steps; SQ/GRBM MFMA-busy passes of the headline and config-5 steps.
# Summaries go to gpurun_out/r05_traffic_*.json / r05_mfma_busy_*.json (copied into profiles/).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_r05.sh reconet both || exit 3
python tools/pmc_traffic.py reconet gpurun_out/r05_traffic_reconet.json --after-marker > /dev/null && \
python tools/pmc_busy.py reconet gpurun_out/r05_mfma_busy_reconet.json || exit 4
bash tools/pmc_r05.sh adaattn_c5 both || exit 5
python tools/pmc_traffic.py adaattn_c5 gpurun_out/r05_traffic_adaattn_c5.json --after-marker > /dev/null && \
python tools/pmc_busy.py adaattn_c5 gpurun_out/r05_mfma_busy_adaattn_c5.json || exit 6
bash tools/pmc_r05.sh reconet_f32 traffic || exit 7
python tools/pmc_traffic.py reconet_f32 gpurun_out/r05_traffic_reconet_f32.json --after-marker > /dev/null || exit 8
bash tools/pmc_r05.sh adaattn traffic || exit 9
python tools/pmc_traffic.py adaattn gpurun_out/r05_traffic_adaattn.json --after-marker > /dev/null || exit 10
rm -rf gpurun_out/pmc_* gpurun_out/pmcb_*
echo done
