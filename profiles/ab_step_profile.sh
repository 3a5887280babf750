#!/bin/bash
# graph-mode step profiles of a tuning-build switch, one run per value:
#   profiles/ab_step_profile.sh <tag> <VAR> <windows> <v1> [<v2> ...]
# (the tuning library, WHISPER_HIP_LIB; summaries in gpurun_out/abprof_<tag>_<VAR>_<v>.txt)
set -o pipefail
tag=$1; var=$2; win=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in "$@"; do
  d=gpurun_out/abprof_${tag}_${var}_${v}
  env $var=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- \
    python3 profiles/step_profile.py --windows $win > ${d}.log 2>&1 || exit 2
  db=$(ls $d/*/run_results.db $d/run_results.db 2>/dev/null | head -1)
  python3 profiles/summarize_db.py $db 30 > ${d}.txt || exit 3
  echo "== $var=$v"; cat ${d}.txt
done
