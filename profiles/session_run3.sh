#!/bin/bash
# edge microbenchmark (flat / per-XCD hand-off) + GPU suite + step profile + default bench
#   profiles/session_run3.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 180 ./whisper.coreml_amd/tools/edge_bench 64 20 > gpurun_out/edge_bench_${tag}.txt 2>&1 || { cat gpurun_out/edge_bench_${tag}.txt; exit 5; }
cat gpurun_out/edge_bench_${tag}.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_${tag}.log 2>&1 || { tail -30 gpurun_out/gpu_tests_${tag}.log; exit 1; }
tail -3 gpurun_out/gpu_tests_${tag}.log
bash profiles/profile_step.sh w20_${tag} --windows 20 --steps 16 --encode 4 || exit 2
head -3 gpurun_out/step_w20_${tag}_plain.txt
grep -E 'attn_enc|xattn|gemm_256' gpurun_out/step_w20_${tag}_summary.txt
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || exit 4
cat gpurun_out/bench_${tag}.json
