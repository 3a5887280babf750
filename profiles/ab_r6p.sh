# Round 6 (p): phase marks of the single-window cross-attention with the split query (QV 6,
# WHISPER_HIP_XQP1=2) and with the shipped form (0): where the in-kernel exchange's time goes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in 2 0; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 200 python profiles/xattn_trace.py 1 > gpurun_out/xtp_$v.txt 2>&1 || exit 1
done
