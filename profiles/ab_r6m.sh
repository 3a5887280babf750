# Round 6 (m): probe — each layer's cross K / V pulled through the memory side (Infinity Cache)
# on a second stream beside the layer chain (k_kv_pull, tuning WHISPER_HIP_XKV_PF=<workgroups>)
# vs off (k_kv_pull by LDS-DMA, 256-thread workgroups): chain traces at 0 / 150 replayed steps, then config-3 lines, alternated, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for adv in 0 150; do
    for v in 0 128 256; do
      WHISPER_HIP_LIB=$N WHISPER_HIP_XKV_PF=$v timeout -k 10 150 python profiles/chain_trace.py 20 8 $adv > gpurun_out/ctm_${v}_${adv}_$rep.txt 2>&1 || exit 2
    done
  done
done
for v in 128 0; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XKV_PF=$v timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/m_c3_$v.json 2>gpurun_out/m_c3_$v.err || exit 3
done
