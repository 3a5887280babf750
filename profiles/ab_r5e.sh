# Round 5 A/B (e): k_xattn_seg's merge reads its pairs' window metadata from LDS (kept at the
# query staging) instead of a vector global load + vmcnt(0) ahead of the merge
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
P=$PWD/whisper.coreml_amd/lib/libwhisper_hip_prev_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/xattn_trace.py 20,1 > gpurun_out/xte_prev_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/xattn_trace.py 20,1 > gpurun_out/xte_new_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/cte_prev_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/cte_new_$rep.txt 2>&1 || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_models.py tests/test_gpu_tail.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_e.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_e.json 2> gpurun_out/cfg3_e.err || exit 3
