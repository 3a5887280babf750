#!/bin/bash
# step graph along a fixed-work 20-window decode (profiles/ancestry_probe.py) for each value
# of a tuning-build switch: profiles/ctx_ab.sh <VAR> <v1> [<v2> ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TUNE=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
var=$1; shift
for v in "$@"; do
  echo "== $var=$v"
  env WHISPER_HIP_LIB=$TUNE $var=$v timeout -k 10 300 python3 -u profiles/ancestry_probe.py large-v3 20 \
    > gpurun_out/ctx_${var}_$v.txt 2>&1 || { tail -5 gpurun_out/ctx_${var}_$v.txt; exit 2; }
  grep -v "^W" gpurun_out/ctx_${var}_$v.txt
done
