"""The C-ABI library loads without a GPU and exports every symbol that
include/whisper_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "whisper_hip.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int)\s+(wh_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    for must in ("wh_create", "wh_destroy", "wh_load_tensor", "wh_finalize", "wh_log_mel", "wh_encode",
                 "wh_decode_begin", "wh_decode_steps", "wh_decode_read", "wh_prefill_logits", "wh_last_error",
                 "wh_prefill", "wh_step", "wh_reorder_kv", "wh_decode_begin_slots"):
        assert must in names


def test_library_exports_all_declared_symbols():
    from whisper import backend_hip
    path = backend_hip.lib_path()
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python shim binds exactly the declared surface
    assert set(backend_hip._EXPORTS) <= set(_declared())
    lib.wh_version.restype = ctypes.c_int
    assert lib.wh_version() >= 1


def test_create_fails_loudly_without_gpu():
    import whisper
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    with pytest.raises(whisper.HipBackendError):
        whisper.load_model("micro", device=0, synthetic=True)


def test_load_model_without_checkpoint_raises(tmp_path):
    """No silent random weights: a missing checkpoint raises unless synthetic=True."""
    import whisper
    with pytest.raises(RuntimeError, match="not found"):
        whisper.load_model("large-v3", device=0, download_root=str(tmp_path))


def test_context_refuses_self_kv_over_2gib_before_loading():
    """One layer's self-KV cache must stay under 2 GiB (32-bit buffer offsets in the
    self-attention kernels): the wrapper refuses a larger max_windows with the limit in the
    message, before touching the library; bench.py clamps to the same limit."""
    import pytest
    from whisper import synthetic as S
    from whisper.backend_hip import HipContext, max_windows_limit
    d = S.MODEL_DIMS["large-v3"]
    assert max_windows_limit(d, "fp32", 5) == 187 and max_windows_limit(d, "fp16", 5) == 374
    assert (max_windows_limit(d, "fp32", 5) + 1) * 5 * 448 * 1280 * 4 >= (1 << 31) - 4096
    with pytest.raises(ValueError, match="at most 187 windows"):
        HipContext(d, dtype="fp32", max_windows=200, max_group=5)
