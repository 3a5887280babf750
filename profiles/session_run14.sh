#!/bin/bash
# the batch-invariance test first, then the GPU suite and the default bench
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batch.py -k batch_invariance -x -q -s --timeout 280 --timeout-method thread \
  > gpurun_out/inv_${tag}.log 2>&1 || { tail -30 gpurun_out/inv_${tag}.log; exit 1; }
tail -3 gpurun_out/inv_${tag}.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_${tag}.log 2>&1 || { tail -30 gpurun_out/gpu_tests_${tag}.log; exit 2; }
tail -3 gpurun_out/gpu_tests_${tag}.log
bash profiles/profile_step.sh w20_${tag} --windows 20 --steps 16 || exit 3
head -3 gpurun_out/step_w20_${tag}_plain.txt
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || exit 4
cat gpurun_out/bench_${tag}.json
