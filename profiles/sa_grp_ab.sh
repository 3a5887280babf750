set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TUNE=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in ${@:-1 0}; do
  echo "== SA_GRP=$v"
  WHISPER_HIP_LIB=$TUNE WHISPER_HIP_SA_GRP=$v timeout -k 10 300 python3 -u profiles/ancestry_probe.py large-v3 20 > gpurun_out/anc_sa$v.txt 2>&1 || { tail -5 gpurun_out/anc_sa$v.txt; exit 2; }
  grep -v "^W" gpurun_out/anc_sa$v.txt
done
