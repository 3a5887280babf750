"""The single-window fp16 token tail of the step graph against the reference's own host
decode loop on the same logits.

The graph path (`whisper.decode` -> decode_steps, one window) runs k_vocab1 (the final
LayerNorm + vocabulary projection: a workgroup's columns reduced over its 8 K-eighths in
wave order), then k_logit_part with the window's candidate merge folded in (round 4);
the tuning build's WHISPER_HIP_VOCAB_SEL=1 runs all three as one launch (k_vocab_sel),
with the same vocabulary arithmetic.  The per-step ABI (wh_prefill / wh_step /
wh_reorder_kv through HipInference) runs the same decoder layers and k_vocab1, so both
paths see bit-identical logits every step; `oracle.ref_whisper.decode` applies the
reference's filters, log-softmax and GreedyDecoder / BeamSearchDecoder updates to them
on the CPU (decoding.py:304-409, 450-532).  The graph path must choose the same tokens;
its log-probabilities are normalised in another summation order, so avg_logprob agrees
to float rounding.  Large-v3 and turbo (K 1280, the width k_vocab1 serves).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    ("large-v3", "beam_fixed"),
    ("large-v3", "greedy_fixed"),
    ("large-v3", "greedy_natural"),
    ("turbo", "beam_fixed"),
]


def _options(kind, eot):
    opts = {}
    if kind.endswith("fixed"):
        opts["suppress_tokens"] = f"-1,{eot}"
    if kind.startswith("beam"):
        opts["beam_size"] = 5
    return opts


@pytest.mark.parametrize("name,kind", CASES)
def test_fused_tail_equals_reference_host_loop(name, kind):
    import whisper
    from conftest import full_model, golden_window
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    from whisper.inference import HipInference

    m = full_model(name, "fp16")
    dims = S.MODEL_DIMS[name]
    st = R.SpecialTokens.for_model(dims)
    opts = _options(kind, st.eot)
    mel = golden_window(name)

    # graph path: decode_steps on one window (the fused tail every step)
    kern = m.ctx.step_kernels(1, opts.get("beam_size", 1))  # names the tail the graph runs
    got = whisper.decode(m, mel, whisper.DecodingOptions(language="en", **opts))

    # the reference's host loop over the per-step ABI, same window
    m.ctx.mel_write(mel)
    m.ctx.encode([0], [3000])
    inf = HipInference(m, len(st.sot_sequence), group=opts.get("beam_size", 1), sot_index=0)

    class _Shell:
        pass
    shell = _Shell()
    shell.dims = dims
    ref = R.decode(shell, None, R.Options(**opts), st, inference=inf)

    a, b = np.asarray(got.tokens), np.asarray(ref.tokens)
    print(f"{name} fp16 {kind}: {len(a)} tokens (host loop {len(b)}), avg_logprob {got.avg_logprob:.6f} vs "
          f"{ref.avg_logprob:.6f}; step kernels {kern}")
    np.testing.assert_array_equal(a, b)
    assert got.avg_logprob == pytest.approx(ref.avg_logprob, abs=1e-4)
