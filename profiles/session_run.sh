#!/bin/bash
# one GPU-box session: GPU suite, graph-mode step profiles (20 windows, 1 window), default bench
#   profiles/session_run.sh <tag> [tests|notests]
set -o pipefail
tag=$1; mode=${2:-tests}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$mode" = tests ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_${tag}.log 2>&1 || { tail -30 gpurun_out/gpu_tests_${tag}.log; exit 1; }
  tail -3 gpurun_out/gpu_tests_${tag}.log
fi
bash profiles/profile_step.sh w20_${tag} --windows 20 --steps 16 || exit 2
bash profiles/profile_step.sh w1_${tag} --windows 1 --steps 32 || exit 3
head -3 gpurun_out/step_w20_${tag}_plain.txt gpurun_out/step_w1_${tag}_plain.txt
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || exit 4
cat gpurun_out/bench_${tag}.json
