#!/bin/bash
# diagnostic: counters of k_forward in the timing harness (GPU box), one rocprofv3 pass per group
cd "$(dirname "$0")/.." || exit 2
set -e
export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude -Inypc-yacht-auction_amd/csrc \
   tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_p -w
mkdir -p gpurun_out/pmc
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F32" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --kernel-include-regex k_forward --pmc $grp -d gpurun_out/pmc/g$i -o g$i --output-format csv -- /tmp/abl_p ${1:-3480} || echo "group $i failed"
done
