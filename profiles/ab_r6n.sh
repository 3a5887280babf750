# Round 6 (n): the cross K / V pull (k_kv_pull, WHISPER_HIP_XKV_PF) on a high-priority stream
# (WHISPER_HIP_XKV_PRIO=1) vs normal priority vs off: chain traces, one box, tuning build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for v in 0 p n; do
    case $v in 0) E="WHISPER_HIP_XKV_PF=0";; p) E="WHISPER_HIP_XKV_PF=256 WHISPER_HIP_XKV_PRIO=1";; n) E="WHISPER_HIP_XKV_PF=256";; esac
    env $E WHISPER_HIP_LIB=$N timeout -k 10 150 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctn_${v}_$rep.txt 2>&1 || exit 2
  done
done
