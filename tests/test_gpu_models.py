"""HIP path vs the reference at the official model dimensions (tiny.en, turbo,
large-v3), seeded synthetic weights regenerated on the box (whisper/synthetic.py,
checksum pinned to the golden).

Bars:
  * fp32 context: greedy and beam-5 token sequences identical to the reference
    CPU path for all 224 steps (fixed work: EOT suppressed), avg_logprob within
    1e-3;
  * fp16 context (production): first-step logits within 2% of the logit range
    (max abs error over the reference top-64 / (max - min) of those values),
    identical top-1, and >= 4 of the reference top-5 in our top-5; free-running
    greedy equal through the decisive prefix (every step whose reference margin
    exceeds twice the teacher-forced fp16 bound of test_gpu_batch.py).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, record_margin

pytestmark = pytest.mark.gpu

MODELS = ["tiny.en", "turbo", "large-v3"]


def _golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def _model(name, dtype):
    from conftest import full_model
    return full_model(name, dtype)


def _window(name):
    from conftest import golden_window
    return golden_window(name)


@pytest.mark.parametrize("dtype", ["fp16", "fp32"])
@pytest.mark.parametrize("name", MODELS)
def test_first_step_logits(name, dtype):
    g = _golden(name)
    m = _model(name, dtype)
    m.ctx.mel_write(_window(name))
    m.ctx.encode([0], [3000])
    rn = np.linalg.norm(m.ctx.audio_features(0).astype(np.float64), axis=1)
    np.testing.assert_allclose(rn, g["xa_rownorm"], rtol=2e-3 if dtype == "fp32" else 2e-2)
    logits, _ = m.ctx.prefill_logits(0, list(g["sot_sequence"]))
    row = logits[-1]
    topi, topv = g["first_last_topi"], g["first_last_topv"]
    rng = float(topv.max() - topv.min())
    err = float(np.abs(row[topi] - topv).max())
    print(f"{name} {dtype}: top-64 max abs err {err:.3e} (range {rng:.2f})")
    bound = 1e-3 if dtype == "fp32" else 0.02
    record_margin("first_step_logits", model=name, dtype=dtype, worst_rel=err / rng, tau=bound,
                  frac_of_tau=err / rng / bound, top1_equal=bool(int(np.argmax(row)) == int(topi[0])))
    assert err < (1e-3 * rng if dtype == "fp32" else 0.02 * rng)
    assert int(np.argmax(row)) == int(topi[0])
    assert len(set(np.argsort(-row)[:5]) & set(topi[:5])) >= 4
    assert int(np.argmax(logits[0])) == int(g["first_sot_topi"][0])


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("kind", ["greedy_fixed", "beam_fixed"])
def test_fp32_tokens_exact(name, kind):
    import whisper
    g = _golden(name)
    m = _model(name, "fp32")
    eot = 50257 if m.is_multilingual else 50256
    opts = dict(language="en", suppress_tokens=f"-1,{eot}")
    if kind.startswith("beam"):
        opts["beam_size"] = 5
    res = whisper.decode(m, _window(name), whisper.DecodingOptions(**opts))
    np.testing.assert_array_equal(np.asarray(res.tokens), g[f"{kind}_tokens"])
    assert res.avg_logprob == pytest.approx(float(g[f"{kind}_avg_logprob"]), abs=1e-3)


NATURAL = [(n, k) for n in MODELS for k in ("greedy", "greedy_prompt", "greedy_notime")] + [("tiny.en", "beam")]


def _natural_options(kind):
    """The reference runs behind the natural goldens (oracle/gen_golden.py model_goldens):
    EOT allowed, timestamps on unless `notime`, a 40-token prompt for `prompt`."""
    opts = dict(language="en")
    if kind == "greedy_prompt":
        opts["prompt"] = list(range(1000, 1040))
    if kind == "greedy_notime":
        opts["without_timestamps"] = True
    if kind == "beam":
        opts["beam_size"] = 5
    return opts


@pytest.mark.parametrize("name,kind", NATURAL)
def test_fp32_natural_tokens_exact(name, kind):
    """Natural decoding (EOT may win, decoding.py:707-737) at real dims, fp32: tokens equal
    the reference's, including the prompt prefill at real width (<|startofprev|> + 40
    tokens + sot sequence, decoding.py:628-638) and the no-timestamp sot sequence."""
    import whisper
    g = _golden(name)
    m = _model(name, "fp32")
    res = whisper.decode(m, _window(name), whisper.DecodingOptions(**_natural_options(kind)))
    np.testing.assert_array_equal(np.asarray(res.tokens), g[f"{kind}_tokens"])
    assert res.avg_logprob == pytest.approx(float(g[f"{kind}_avg_logprob"]), abs=1e-3)
    assert res.no_speech_prob == pytest.approx(float(g[f"{kind}_no_speech_prob"]), abs=1e-4)


@pytest.mark.parametrize("dtype", ["fp16", "fp32"])
@pytest.mark.parametrize("name", MODELS)
def test_prompt_prefill_logits(name, dtype):
    """First pass over a 44-token prompted sequence: the last row's logits against the
    reference's top-64 (same bars as test_first_step_logits)."""
    g = _golden(name)
    m = _model(name, dtype)
    m.ctx.mel_write(_window(name))
    m.ctx.encode([0], [3000])
    logits, _ = m.ctx.prefill_logits(0, [int(t) for t in g["prompt_tokens"]])
    row = logits[-1]
    topi, topv = g["prompt_last_topi"], g["prompt_last_topv"]
    rng = float(topv.max() - topv.min())
    err = float(np.abs(row[topi] - topv).max())
    print(f"{name} {dtype}: prompt prefill top-64 max abs err {err:.3e} (range {rng:.2f})")
    bound = 1e-3 if dtype == "fp32" else 0.02
    record_margin("prompt_prefill_logits", model=name, dtype=dtype, worst_rel=err / rng, tau=bound,
                  frac_of_tau=err / rng / bound, top1_equal=bool(int(np.argmax(row)) == int(topi[0])))
    assert err < (1e-3 * rng if dtype == "fp32" else 0.02 * rng)
    assert int(np.argmax(row)) == int(topi[0])


@pytest.mark.parametrize("name", MODELS)
def test_fp16_natural_greedy_agreement(name):
    """fp16 natural greedy equals the reference through every step whose post-filter top-2
    margin (recorded by the reference run, greedy_margins) exceeds twice the fp16
    teacher-forced bound, taken in absolute terms as TAU * the median top-32 range of
    the reference's steps."""
    import whisper
    from test_gpu_batch import TAU, _steps
    g = _golden(name)
    m = _model(name, "fp16")
    res = whisper.decode(m, _window(name), whisper.DecodingOptions(language="en"))
    got, ref = np.asarray(res.tokens), g["greedy_tokens"]
    topv = _steps(name)["tf_greedy_fixed_topv"][:, 0]
    eps = TAU["fp16"] * float(np.median(topv[:, 0] - topv[:, -1]))
    margins = g["greedy_margins"]
    close = margins <= 2 * eps
    need = int(np.argmax(close)) if close.any() else len(margins)
    n = min(len(got), len(ref))
    agree = int(np.argmax(got[:n] != ref[:n])) if np.any(got[:n] != ref[:n]) else n
    print(f"{name} fp16 natural greedy agreement {agree}/{len(ref)} (decisive prefix {need})")
    record_margin("fp16_natural_greedy", model=name, dtype="fp16", agree_steps=agree, ref_steps=int(len(ref)),
                  decisive_prefix=need, tokens_equal=bool(len(got) == len(ref) and np.array_equal(got, ref)))
    assert agree >= min(need, len(ref))
    if need >= len(margins):
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("name", MODELS)
def test_fp16_greedy_agreement(name):
    """fp16 greedy (free running, fixed work) equals the reference through every step
    whose reference top-2 margin exceeds twice the teacher-forced fp16 logit bound
    (test_gpu_batch.TAU): up to there no choice can flip."""
    import whisper
    from test_gpu_batch import TAU, decisive_prefix
    g = _golden(name)
    m = _model(name, "fp16")
    eot = 50257 if m.is_multilingual else 50256
    res = whisper.decode(m, _window(name), whisper.DecodingOptions(language="en", suppress_tokens=f"-1,{eot}"))
    got, ref = np.asarray(res.tokens), g["greedy_fixed_tokens"]
    n = min(len(got), len(ref))
    agree = int(np.argmax(got[:n] != ref[:n])) if np.any(got[:n] != ref[:n]) else n
    need = min(decisive_prefix(name, "greedy_fixed", TAU["fp16"]), len(ref))
    print(f"{name} fp16 greedy agreement {agree}/{len(ref)} (decisive prefix {need}); avg_logprob "
          f"{res.avg_logprob:.4f} vs {float(g['greedy_fixed_avg_logprob']):.4f}")
    record_margin("fp16_fixed_greedy", model=name, dtype="fp16", agree_steps=agree, ref_steps=int(len(ref)),
                  decisive_prefix=need, avg_logprob_diff=abs(float(res.avg_logprob) - float(g["greedy_fixed_avg_logprob"])))
    assert len(got) == len(ref)
    assert agree >= need
