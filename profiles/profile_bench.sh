#!/bin/bash
# rocprofv3 kernel profiles of bench.py on the GPU box (run from the repo root):
#   profiles/profile_bench.sh <tag> [bench args...]
# eager mode (the tuning library with WHISPER_HIP_EAGER=1: the step kernels launched directly;
# the shipped library reads no environment) and graph mode (the shipped library);
# summaries land in gpurun_out/prof_<tag>_{eager,graph}/
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out
mkdir -p $out
WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_${tag}_eager -o run -- \
  python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 "$@" > $out/prof_${tag}_eager.log 2>&1
echo "eager rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_${tag}_graph -o run -- \
  python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 "$@" > $out/prof_${tag}_graph.log 2>&1
echo "graph rc=$?"
