"""Encoder-only workload for PMC passes on the encoder GEMMs / attention.

large-v3 fp16, one 16-window encoder chunk, encoded twice (the second pass is the one
to read).  Usage on the GPU box (one counter group per run, no trace domains):

  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \\
      SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/enc_pmc -o run \\
      --output-format csv -- python3 profiles/enc_pmc.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))
    import whisper
    from whisper import synthetic as S
    dims = S.MODEL_DIMS["large-v3"]
    model = whisper.Whisper(whisper.ModelDimensions(**dims), "large-v3", device=0, dtype="fp16",
                            max_windows=16, max_group=5)
    model.load_state_dict(S.synthetic_state_dict(dims, 0))
    audio = S.synthetic_audio(480.0, seed=1000)
    model.ctx.log_mel(audio, padding=480000, n_mels=dims["n_mels"], normalize=True)
    for _ in range(2):
        model.ctx.encode([3000 * i for i in range(16)], [3000] * 16)
    model.ctx.sync()
    model.close()
    print("ok")


if __name__ == "__main__":
    main()
