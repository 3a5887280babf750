# Round 5 A/B (c): LDS-only barriers in the selection / window merge (no store drain at
# each barrier) and the history row loaded with the logits in k_logit_part
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
P=$PWD/whisper.coreml_amd/lib/libwhisper_hip_prev_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctc_prev_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctc_new_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctc_prev_w1_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctc_new_w1_$rep.txt 2>&1 || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_tail.py tests/test_gpu_beam_options.py tests/test_gpu_models.py tests/test_gpu_resume.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_c.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_c.json 2> gpurun_out/cfg3_c.err || exit 3
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --model turbo --seconds 30 > gpurun_out/cfg2_c.json 2> gpurun_out/cfg2_c.err || exit 4
