# Round 6 (j): the 100-row token selection with 8 slices per row (WHISPER_HIP_LP_NS=8: 800
# workgroups, one round) vs the shipped 16 (1600, three rounds), chain traces, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for v in 16 8; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_LP_NS=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctj_${v}_$rep.txt 2>&1 || exit 1
  done
done
