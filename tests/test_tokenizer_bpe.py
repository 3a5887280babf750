"""BPE text encoding / decoding (reference tests/test_tokenizer.py) with the rank
files the reference's tokenizer loads ({gpt2,multilingual}.tiktoken, data the
reference ships in whisper/assets and this package ships in whisper/assets), and
text prompts end to end (decoding.py:614-640, transcribe.py:243-244)."""
import os

import numpy as np
import pytest


@pytest.fixture(autouse=True)
def bpe_tables(monkeypatch):
    from whisper import tokenizer as T
    monkeypatch.delenv("WHISPER_TIKTOKEN_DIR", raising=False)
    T._rank_file.cache_clear()
    T._encoder.cache_clear()
    yield
    T._rank_file.cache_clear()
    T._encoder.cache_clear()


@pytest.mark.parametrize("multilingual", [True, False])
def test_tokenizer(multilingual):
    # reference tests/test_tokenizer.py:6-11
    from whisper.tokenizer import get_tokenizer
    tokenizer = get_tokenizer(multilingual=multilingual)
    assert tokenizer.sot in tokenizer.sot_sequence
    assert len(tokenizer.all_language_codes) == len(tokenizer.all_language_tokens)
    assert all(c < tokenizer.timestamp_begin for c in tokenizer.all_language_tokens)


def test_multilingual_tokenizer():
    # reference tests/test_tokenizer.py:14-25
    from whisper.tokenizer import get_tokenizer
    gpt2_tokenizer = get_tokenizer(multilingual=False)
    multilingual_tokenizer = get_tokenizer(multilingual=True)
    text = "다람쥐 헌 쳇바퀴에 타고파"
    gpt2_tokens = gpt2_tokenizer.encode(text)
    multilingual_tokens = multilingual_tokenizer.encode(text)
    assert gpt2_tokenizer.decode(gpt2_tokens) == text
    assert multilingual_tokenizer.decode(multilingual_tokens) == text
    assert len(gpt2_tokens) > len(multilingual_tokens)


def test_split_on_unicode():
    # reference tests/test_tokenizer.py:28-34
    from whisper.tokenizer import get_tokenizer
    multilingual_tokenizer = get_tokenizer(multilingual=True)
    tokens = [8404, 871, 287, 6, 246, 526, 3210, 20378]
    words, word_tokens = multilingual_tokenizer.split_tokens_on_unicode(tokens)
    assert words == [" elle", " est", " l", "'", "�", "é", "rit", "oire"]
    assert word_tokens == [[8404], [871], [287], [6], [246], [526], [3210], [20378]]


def test_known_ids_and_round_trips():
    from whisper.tokenizer import get_tokenizer
    ml = get_tokenizer(multilingual=True)
    # ids of the reference tokenizer (SURVEY.md §8c probe 1)
    assert ml.encode(" And so my fellow Americans") == [400, 370, 452, 7177, 6280]
    for text in ["", " ", "Hello, world!  It's 3:15 p.m.\n", "naïve café — ünïcödé", "   leading spaces",
                 "tab\there", "数字 123 456"]:
        for tok in (ml, get_tokenizer(multilingual=False)):
            ids = tok.encode(text)
            assert all(0 <= i < tok.eot for i in ids)
            assert tok.decode(ids) == text
    assert ml.encode(" ") == ml.encode_blank()


def test_text_needs_rank_file(monkeypatch, tmp_path):
    """A directory without the rank files: encode and decode fail loudly (no silent "")."""
    from whisper import tokenizer as T
    monkeypatch.setenv("WHISPER_TIKTOKEN_DIR", str(tmp_path))
    T._rank_file.cache_clear()
    T._encoder.cache_clear()
    tok = T.get_tokenizer(multilingual=True)
    with pytest.raises(RuntimeError):
        tok.encode("x")
    with pytest.raises(RuntimeError):
        tok.decode([400])


def test_split_to_word_tokens_spaces_and_punctuation():
    """split_tokens_on_spaces semantics (tokenizer.py:313-327): a piece starts a word
    when it is special, begins with a space or is punctuation."""
    from whisper.tokenizer import get_tokenizer
    ml = get_tokenizer(multilingual=True, language="en")
    ids = ml.encode(" Hello, wonderful world!") + [ml.eot]
    words, groups = ml.split_to_word_tokens(ids)
    assert "".join(words[:-1]) == " Hello, wonderful world!"
    assert words[0] == " Hello" and words[1] == "," and words[-1] == "<|endoftext|>"
    assert [t for g in groups for t in g] == ids


@pytest.mark.gpu
def test_text_prompt_decode_matches_oracle():
    """DecodingOptions(prompt=str, prefix=str) on the micro model (fp32) gives the
    oracle's tokens with the prompt/prefix encoded as " " + text.strip()."""
    import whisper
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    from whisper.tokenizer import get_tokenizer
    dims = S.MODEL_DIMS["micro"]
    sd = S.synthetic_state_dict(dims, 0)
    m = whisper.Whisper(whisper.ModelDimensions(**dims), "micro", device=0, dtype="fp32", max_windows=1,
                        max_group=5)
    m.load_state_dict(sd)
    audio = S.synthetic_audio(30.0, seed=3)
    mel = whisper.pad_or_trim(whisper.log_mel_spectrogram(audio, dims["n_mels"], padding=whisper.audio.N_SAMPLES)
                              [:, :3000], 3000)
    prompt, prefix = "  The quick brown fox. ", "Jumps"
    try:
        res = whisper.decode(m, mel, whisper.DecodingOptions(language="en", prompt=prompt, prefix=prefix,
                                                             sample_len=32))
    finally:
        m.close()
    tok = get_tokenizer(multilingual=dims["n_vocab"] >= 51865, language="en", task="transcribe")
    om = R.OracleWhisper(dims, sd)
    ref_mel = R.pad_or_trim(R.log_mel_spectrogram(audio, dims["n_mels"], padding=R.N_SAMPLES)[:, :3000])
    ref = R.decode(om, ref_mel, R.Options(prompt=tok.encode(" " + prompt.strip()),
                                          prefix=tok.encode(" " + prefix.strip()), sample_len=32))
    np.testing.assert_array_equal(np.asarray(res.tokens), np.asarray(ref.tokens))
