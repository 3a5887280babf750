# Round 5 A/B (b): scalar prologues (32-bit range splits, one round trip of window metadata in
# k_xattn_seg, 32-bit k_reduce_store indexing) and the row-major cross-attention partials
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
P=$PWD/whisper.coreml_amd/lib/libwhisper_hip_prev_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctb_prev_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctb_new_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/xattn_trace.py > gpurun_out/xtb_prev.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/xattn_trace.py > gpurun_out/xtb_new.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctb_new_w1.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_tail.py tests/test_gpu_micro.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_b.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_b.json 2> gpurun_out/cfg3_b.err || exit 3
