# Round 5 A/B (g): the vocabulary kernels' logit stores as one 16-B write-through store per
# lane (WHISPER_HIP_V2P_WIDE=1: k_vocab_2p at 100 rows, k_vocab1 at one window) vs 4 x 4-B
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_WIDE=0 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctg_0_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_WIDE=1 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctg_1_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_WIDE=0 timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctg1w_0_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_WIDE=1 timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctg1w_1_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_WIDE=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_tail.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_g.txt 2>&1 || exit 2
