import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "whisper.coreml_amd")
for p in (PKG_ROOT, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# Every GPU run records each tolerance test's measured margin (worst relative error, where
# it was, top-1 agreement, the bound it is held to) as one JSON line here, so a change that
# ate most of a tolerance shows up even while the suite stays green (DESIGN.md §2;
# profiles/summarize_margins.py folds a run's lines into profiles/<round>/fp16_margins.json).
MARGIN_LOG = os.environ.get("WH_MARGIN_LOG", os.path.join(REPO, "gpurun_out", "margins.jsonl"))


def record_margin(test, **fields):
    import json
    os.makedirs(os.path.dirname(MARGIN_LOG), exist_ok=True)
    rec = {"test": test}
    rec.update({k: (float(v) if hasattr(v, "dtype") and v.shape == () else v) for k, v in fields.items()})
    with open(MARGIN_LOG, "a") as f:
        f.write(json.dumps(rec) + "\n")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


# ---------------------------------------------------------------- full-size models
# One HIP context at a time (large-v3 fp32 at 20 windows holds ~25 GB of KV caches);
# the seeded synthetic state dict of the last model is kept on the host so that
# contexts of other dtypes / capacities reload it without regenerating it.
_SD = {}
_CTX = {}


def full_model(name, dtype, max_windows=20, max_group=5):
    """whisper.Whisper with the golden file's seeded weights (checksum pinned)."""
    import numpy as np

    import whisper
    from whisper import synthetic as S
    key = (name, dtype, max_windows, max_group)
    if key in _CTX:
        return _CTX[key]
    for k in list(_CTX):
        _CTX.pop(k).close()
    if name not in _SD:
        _SD.clear()
        g = np.load(os.path.join(GOLDEN, f"{name}.npz"))
        sd = S.synthetic_state_dict(S.MODEL_DIMS[name], int(g["seed"]))
        assert S.state_dict_checksum(sd) == pytest.approx(float(g["weights_checksum"]), rel=1e-12)
        _SD[name] = sd
    m = whisper.Whisper(whisper.ModelDimensions(**S.MODEL_DIMS[name]), name, device=0, dtype=dtype,
                        max_windows=max_windows, max_group=max_group)
    m.load_state_dict(_SD[name])
    if name in whisper._ALIGNMENT_HEADS:
        m.set_alignment_heads(whisper._ALIGNMENT_HEADS[name])
    _CTX[key] = m
    return m


def golden_window(name, audio_seed=None):
    """The reference's 30 s window of seeded audio (log-mel on the GPU, pad_or_trim)."""
    import numpy as np

    import whisper
    from whisper import synthetic as S
    if audio_seed is None:
        audio_seed = int(np.load(os.path.join(GOLDEN, f"{name}.npz"))["audio_seed"])
    audio = S.synthetic_audio(30.0, seed=int(audio_seed))
    mel = whisper.log_mel_spectrogram(audio, S.MODEL_DIMS[name]["n_mels"], padding=whisper.audio.N_SAMPLES)
    return whisper.pad_or_trim(mel[:, :3000], 3000)
