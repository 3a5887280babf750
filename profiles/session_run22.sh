#!/bin/bash
# encoder attention K/V prefetch depth A/B (tuning build: WHISPER_HIP_ENC_PF=1 = round-3 form, 2 = new)
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
out=gpurun_out/enc_pf_${tag}.txt
: > $out
for rep in 1 2; do
  for pf in 1 2; do
    for w in 1 20; do
      echo -n "PF=$pf " >> $out
      WHISPER_HIP_ENC_PF=$pf timeout -k 10 200 python3 -u profiles/enc_chunk_probe.py --model large-v3 --windows $w --reps 5 >> $out 2>&1 || exit 2
    done
  done
done
cat $out
