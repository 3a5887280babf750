# Round 5 A/B (f): single-window issue-side fixes — k_proj1's QKV epilogue coordinates in the
# first round trip; k_xattn_seg (few windows) issues its first tile after ONE scalar batch;
# k_self_attn issues its query row with the row tables (a per-lane vector load into LDS)
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
P=$PWD/whisper.coreml_amd/lib/libwhisper_hip_prev_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctf_prev_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctf_new_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/xattn_trace.py 1 > gpurun_out/xtf_prev.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/xattn_trace.py 1 > gpurun_out/xtf_new.txt 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_models.py tests/test_gpu_tail.py tests/test_gpu_micro.py tests/test_gpu_resume.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_f.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/cfg2_f.json 2> gpurun_out/cfg2_f.err || exit 4
