# Round 5 A/B (n): k_vocab_2p's epilogue through LDS (WHISPER_HIP_V2P_TR=1: one 1-KB row
# segment per store instruction) vs per-lane 16-B stores of 16 rows x 64 B (=0), tuning lib
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_TR=0 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctn_0_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_TR=1 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctn_1_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$N WHISPER_HIP_V2P_TR=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_n.txt 2>&1 || exit 2
