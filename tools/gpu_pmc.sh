#!/bin/bash
# round counter set: HBM traffic (FETCH/WRITE) and the SQ/GRBM MFMA-busy passes of the headline (config 3) and
# config-5 steps -> gpurun_out/r06_traffic_*.json, r06_mfma_busy_*.json (copied into profiles/)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_round.sh reconet both || exit 3
python tools/pmc_traffic.py reconet gpurun_out/r06_traffic_reconet.json --after-marker > /dev/null && \
python tools/pmc_busy.py reconet gpurun_out/r06_mfma_busy_reconet.json || exit 4
bash tools/pmc_round.sh adaattn_c5 both || exit 5
python tools/pmc_traffic.py adaattn_c5 gpurun_out/r06_traffic_adaattn_c5.json --after-marker > /dev/null && \
python tools/pmc_busy.py adaattn_c5 gpurun_out/r06_mfma_busy_adaattn_c5.json || exit 6
rm -rf gpurun_out/pmc_* gpurun_out/pmcb_*
echo done
