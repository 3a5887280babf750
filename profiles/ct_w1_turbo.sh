# Round 6: the one-window turbo step (config 2's latency path) priced per launch by chain_trace.py,
# at 0 and 150 replayed steps, shipped defaults on the tuning build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for adv in 0 150; do
  CT_MODEL=turbo WHISPER_HIP_LIB=$N timeout -k 10 150 python profiles/chain_trace.py 1 10 $adv > gpurun_out/ct_w1_turbo_$adv.txt 2>&1 || exit 2
done
