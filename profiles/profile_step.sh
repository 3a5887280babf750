#!/bin/bash
# graph-mode kernel profile of the decoder step: profiles/profile_step.sh <tag> [step_profile.py args]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 profiles/step_profile.py "$@" > gpurun_out/step_${tag}_plain.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step_${tag} -o run -- \
  python3 profiles/step_profile.py "$@" > gpurun_out/step_${tag}_prof.log 2>&1 || exit 2
python3 profiles/summarize_db.py $(ls gpurun_out/prof_step_${tag}/*/run_results.db gpurun_out/prof_step_${tag}/run_results.db 2>/dev/null | head -1) 40 gpurun_out/step_${tag}_kernel_stats.csv > gpurun_out/step_${tag}_summary.txt
