# Round 6 (f): (1) fewer split-K slices for the 100-row projections now that the slabs are
# fp16: chain traces with WHISPER_HIP_PROJ_FORCE pinning, per (N, K), a
# tiling of profiles/../wh_proj.hip CFGS — out / cross-out z 8 -> 4 (1280:1280:1), fc2 z 16 -> 8
# (1280:5120:5, 1280:5120:6), fc1 z 4 -> 2 (5120:1280:5); (2) the PMC traffic passes of the
# final kernels (profiles/pmc_pass.sh); (3) LAST (it crashed rocprofv3 in round 5): the
# late-context self-attention traffic, restructured (profiles/sa_traffic.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for f in none 1280:1280:1 1280:5120:5 1280:5120:6 5120:1280:5; do
    t=${f//:/_}
    if [ $f = none ]; then
      WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctf_${t}_$rep.txt 2>&1 || exit 1
    else
      WHISPER_HIP_LIB=$N WHISPER_HIP_PROJ_FORCE=$f timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctf_${t}_$rep.txt 2>&1 || exit 1
    fi
  done
done
bash profiles/pmc_pass.sh || exit 5
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_self_attn_qkv -d $R/gpurun_out/sa_f -o run --output-format csv -- \
  python3 $R/profiles/sa_traffic.py run > $R/gpurun_out/sa_f6.log 2>&1 || exit 6
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_self_attn_qkv -d $R/gpurun_out/sa_w -o run --output-format csv -- \
  python3 $R/profiles/sa_traffic.py run > $R/gpurun_out/sa_w6.log 2>&1 || exit 7
cd $R && python3 profiles/sa_traffic.py parse gpurun_out/sa_f gpurun_out/sa_w > gpurun_out/sa_traffic.json
