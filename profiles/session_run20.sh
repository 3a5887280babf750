#!/bin/bash
# library GEMM (hipBLASLt via torch.matmul) vs k_gemm_256 at the encoder shapes, same box
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./whisper.coreml_amd/tools/gemm_bench 20 7 > gpurun_out/gemm_ours_${tag}.txt 2>&1 || exit 2
timeout -k 10 300 python3 -u profiles/gemm_lib_compare.py > gpurun_out/gemm_lib_${tag}.txt 2>&1 || exit 3
cat gpurun_out/gemm_ours_${tag}.txt gpurun_out/gemm_lib_${tag}.txt
