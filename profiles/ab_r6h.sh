# Round 6 (h): the in-kernel query projection's load orders 2 / 4 / 5 (wh_kernels.hip
# xq_project: 4 = W_q first, ahead of the metadata round trip; 5 = 4 with the two tiles'
# K / V after the projection), phase marks and chain traces, one box (tuning lib); LAST:
# the late-context self-attention traffic in eager mode (profiles/sa_traffic.py, 100 steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in 2 4 5; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQV=$v timeout -k 10 120 python profiles/xattn_trace.py 20,15,2 > gpurun_out/xth_${v}.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in 2 4 5; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQV=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/cth_${v}_$rep.txt 2>&1 || exit 1
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp
WHISPER_HIP_LIB=$N timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_self_attn_qkv -d $R/gpurun_out/sa_f -o run --output-format csv -- \
  python3 $R/profiles/sa_traffic.py run > $R/gpurun_out/sa_f7.log 2>&1 || exit 6
WHISPER_HIP_LIB=$N timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_self_attn_qkv -d $R/gpurun_out/sa_w -o run --output-format csv -- \
  python3 $R/profiles/sa_traffic.py run > $R/gpurun_out/sa_w7.log 2>&1 || exit 7
cd $R && python3 profiles/sa_traffic.py parse gpurun_out/sa_f gpurun_out/sa_w > gpurun_out/sa_traffic.json
