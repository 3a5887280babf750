"""A device-loop decode resumed after other work on the same context.

The step graph's input rows (x_d, row_pos) are written by the previous update's merge, so
anything else that runs rows through those buffers between two wh_decode_steps chunks — a
first pass for word alignment (wh_align_batch), prefill logits (wh_prefill_logits), a
timing stage — must not change the decode: the next chunk re-embeds every row from the
decode state first (wh_runtime.hip rows_dirty).  Checked on the micro model in fp32: a
decode of three windows (split-K k_proj layers) and of one window (k_proj1 layers) cut
into chunks with alignment / prefill work between them gives exactly the tokens,
log-probabilities and candidates of the same decode run in one call.  The interleaved first
passes use encoder slot 3, outside the decode batch: a first pass writes its window slot's
self-KV rows (as the reference's alignment pass does after that window's decode), so it
may run on a finished or idle slot, not on one still decoding."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def micro32():
    import whisper
    m = whisper.load_model("micro", device=0, dtype="fp32", max_windows=4, max_group=5, synthetic=True)
    yield m
    m.close()


def _setup(m, n):
    import whisper
    from whisper import synthetic as S
    from whisper.audio import N_FRAMES
    from whisper.decoding import DecodingTask
    mels = []
    for s in range(4):
        audio = S.synthetic_audio(30.0, seed=700 + s)
        mel = whisper.log_mel_spectrogram(audio, m.dims.n_mels, padding=whisper.audio.N_SAMPLES)
        mels.append(whisper.pad_or_trim(mel[:, :3000], 3000))
    m.ctx.mel_write(np.concatenate(mels, axis=1))
    m.ctx.encode([i * N_FRAMES for i in range(4)], [N_FRAMES] * 4)  # slots 0..3
    # fixed work (EOT suppressed: no early stop) so every chunk boundary falls inside a
    # live decode
    from whisper.tokenizer import get_tokenizer
    eot = get_tokenizer(m.is_multilingual, num_languages=m.num_languages, language="en", task="transcribe").eot
    return DecodingTask(m, whisper.DecodingOptions(language="en", beam_size=5, sample_len=96,
                                                   suppress_tokens=f"-1,{eot}"))


def _read(m, task, n):
    out = []
    for i in range(n):
        r = m.ctx.decode_read(i, task.n_group)
        out.append((r["tokens"].copy(), r["sum_logprobs"].copy(), r["length"], r["fin_len"].copy(),
                    r["fin_score"].copy()))
    return out


@pytest.mark.parametrize("n", [3, 1])
def test_decode_resumes_after_alignment_and_prefill(micro32, n):
    from whisper.timing import _alignment_head_ids
    from whisper.tokenizer import get_tokenizer
    m = micro32
    task = _setup(m, n)
    init = [task.initial_tokens] * n
    m.ctx.decode_begin(task.wh_opts(), init, [task.sot_index] * n)
    m.ctx.decode_steps(task.sample_len)
    ref = _read(m, task, n)

    tok = get_tokenizer(m.is_multilingual, num_languages=m.num_languages, language="en", task="transcribe")
    heads = _alignment_head_ids(m)
    seq = [*tok.sot_sequence, tok.no_timestamps, *range(100, 140), tok.eot]
    m.ctx.decode_begin(task.wh_opts(), init, [task.sot_index] * n)
    done = m.ctx.decode_steps(9)
    assert done < n, "the decode must still be live at the first cut"
    m.ctx.align_batch([3], [seq], len(tok.sot_sequence), [3000], heads)   # a first pass through x_d
    m.ctx.decode_steps(17)
    m.ctx.prefill_logits(3, list(task.initial_tokens) + list(range(200, 230)))  # another one
    m.ctx.time_stage(2, 1)  # the six projections of every layer on the current rows
    m.ctx.decode_steps(task.sample_len)
    got = _read(m, task, n)
    for w in range(n):
        for a, b, what in zip(got[w], ref[w], ("tokens", "sum_logprobs", "length", "fin_len", "fin_score")):
            np.testing.assert_array_equal(a, b, err_msg=f"window {w}: {what} changed by the interleaved work")
