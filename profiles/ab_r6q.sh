# Round 6 (q): the coalesced-K self-attention's threshold (WHISPER_HIP_SA_KCO_MIN: cached keys from
# which it runs; shipped 64) at 0 / 60 / 150 replayed steps, 20 windows, tuning build, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for adv in 0 60 150; do
  for v in 0 64 128 off; do
    case $v in off) E="WHISPER_HIP_SA_KCO=0";; *) E="WHISPER_HIP_SA_KCO_MIN=$v";; esac
    env $E WHISPER_HIP_LIB=$N timeout -k 10 150 python profiles/chain_trace.py 20 8 $adv > gpurun_out/ctq_${v}_$adv.txt 2>&1 || exit 2
  done
done
