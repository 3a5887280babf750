#!/bin/bash
# Encoder PMC pass (MFMA busy, LDS bank conflicts, clock) on the 16-window encoder chunk
# (profiles/enc_pmc.py): one counter group per run, kernel trace only; writes
# gpurun_out/enc_pmc.json (profiles/pmc_summary.py).  Copy it to profiles/<round>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/enc_pmc -o run \
  --output-format csv -- python3 $R/profiles/enc_pmc.py > $R/gpurun_out/enc_pmc.log 2>&1 || exit 1
cd $R && python3 profiles/pmc_summary.py gpurun_out/enc_pmc "k_gemm_256<1," "k_gemm_256<2," "k_gemm_256<8," "k_gemm_256<4," k_attn_enc k_gemm_tile k_layernorm \
  > gpurun_out/enc_pmc.json
