"""ctypes shim into libwhisper_hip.so — the role whisper/coreml.py:19-244 plays for
the reference's CoreML library, bound to the C ABI of include/whisper_hip.h.

Differences from the reference shim, on purpose:
  * the library owns a *context* (not process globals, coreml.mm:18-23) and every
    call returns a status that is turned into ``HipBackendError`` here (the
    reference's void calls only NSLog failures, coreml.mm:54-56);
  * there is no CPU fallback: if the library or a HIP device is missing, every
    entry point raises.  The product path never computes on the host.
"""

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_uint64, c_void_p
from typing import Optional, Sequence

import numpy as np

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(os.path.dirname(_PKG_DIR), "lib", "libwhisper_hip.so")

WH_F32 = 0
WH_F16 = 1


class HipBackendError(RuntimeError):
    pass


class WhDims(ctypes.Structure):
    _fields_ = [(k, c_int) for k in ("n_mels", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer",
                                     "n_vocab", "n_text_ctx", "n_text_state", "n_text_head", "n_text_layer")]


class WhDecodeOpts(ctypes.Structure):
    _fields_ = [("group", c_int), ("beam", c_int), ("patience", c_float), ("temperature", c_float),
                ("sample_len", c_int), ("suppress_blank", c_int), ("timestamps", c_int), ("max_initial", c_int),
                ("eot", c_int), ("no_speech", c_int), ("no_timestamps", c_int), ("timestamp_begin", c_int),
                ("blank", c_int * 4), ("n_blank", c_int), ("suppress", POINTER(c_int)), ("n_suppress", c_int),
                ("seed", c_uint64), ("max_candidates", c_int)]


_lib = None
_EXPORTS = {
    # name: (restype, argtypes)
    "wh_last_error": (c_char_p, []),
    "wh_version": (c_int, []),
    "wh_create": (c_int, [c_int, POINTER(WhDims), c_int, c_int, c_int, POINTER(c_void_p)]),
    "wh_destroy": (c_int, [c_void_p]),
    "wh_load_tensor": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "wh_finalize": (c_int, [c_void_p]),
    "wh_set_mel_filters": (c_int, [c_void_p, c_int, c_void_p]),
    "wh_log_mel": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int, c_int, POINTER(c_int64)]),
    "wh_log_mel_frames": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int, c_int64, c_int64, c_int,
                                  POINTER(c_int64)]),
    "wh_audio_upload": (c_int, [c_void_p, c_void_p, c_int64]),
    "wh_mel_max": (c_int, [c_void_p, POINTER(c_float)]),
    "wh_mel_normalize": (c_int, [c_void_p, c_float]),
    "wh_mel_read": (c_int, [c_void_p, c_void_p, c_int64, c_int64]),
    "wh_mel_write": (c_int, [c_void_p, c_void_p, c_int64]),
    "wh_encode": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "wh_read_audio_features": (c_int, [c_void_p, c_int, c_void_p]),
    "wh_read_cross_kv": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "wh_decode_begin": (c_int, [c_void_p, c_int, POINTER(WhDecodeOpts), c_void_p, c_void_p, c_int, c_void_p]),
    "wh_decode_begin_slots": (c_int, [c_void_p, c_int, c_void_p, POINTER(WhDecodeOpts), c_void_p, c_void_p, c_int,
                                      c_void_p]),
    "wh_decode_steps": (c_int, [c_void_p, c_int, POINTER(c_int)]),
    "wh_decode_read": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "wh_decode_maxc": (c_int, [c_void_p]),
    "wh_prefill": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "wh_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "wh_reorder_kv": (c_int, [c_void_p, c_void_p]),
    "wh_prefill_logits": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "wh_align": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                         POINTER(c_int)]),
    "wh_align_batch": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                               c_int, c_void_p, c_void_p, c_void_p]),
    "wh_dtw": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, POINTER(c_int)]),
    "wh_stats": (c_int, [c_void_p, POINTER(c_double), c_int]),
    "wh_sync": (c_int, [c_void_p]),
    "wh_time_stage": (c_int, [c_void_p, c_int, c_int, POINTER(c_double)]),
    "wh_step_kernels": (c_int, [c_void_p, c_int, c_int, ctypes.c_char_p, c_int]),
    "wh_token_ms": (c_int, [c_void_p, c_void_p, c_int, POINTER(c_int), c_int]),
    "wh_flac_info": (c_int, [c_void_p, c_int64, POINTER(c_int), POINTER(c_int), POINTER(c_int), POINTER(c_int64)]),
    "wh_flac_decode": (c_int, [c_void_p, c_int64, c_void_p, c_int64, POINTER(c_int64)]),
    "wh_flac_last_error": (c_char_p, []),
}


def lib_path() -> str:
    return os.environ.get("WHISPER_HIP_LIB", _DEFAULT_LIB)


def load_library(path: Optional[str] = None):
    """Load libwhisper_hip.so (raises if absent: no silent fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or lib_path()
    if not os.path.exists(p):
        raise HipBackendError(f"libwhisper_hip.so not found at {p}; build it with `make -C whisper.coreml_amd`")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(c_void_p)


def decode_flac(data: bytes):
    """FLAC bytes -> (int32 samples [frames][channels], sample_rate, bits_per_sample),
    decoded by the library's host FLAC reader (wh_flac_decode; bit-exact)."""
    lib = load_library()
    buf = np.frombuffer(data, np.uint8)
    rate, ch, bps, total = c_int(), c_int(), c_int(), c_int64()
    rc = lib.wh_flac_info(_ptr(buf), len(buf), ctypes.byref(rate), ctypes.byref(ch), ctypes.byref(bps),
                          ctypes.byref(total))
    if rc != 0:
        raise HipBackendError(f"wh_flac_info failed ({rc}): {lib.wh_flac_last_error().decode(errors='replace')}")
    # STREAMINFO may leave the total unknown (0): size the output from the byte count
    # (a FLAC frame cannot carry more samples than a 1-bit-per-sample verbatim one)
    cap = total.value if total.value > 0 else len(buf) * 8
    out = np.empty((cap, ch.value), np.int32)
    n = c_int64()
    rc = lib.wh_flac_decode(_ptr(buf), len(buf), _ptr(out), cap, ctypes.byref(n))
    if rc != 0:
        raise HipBackendError(f"wh_flac_decode failed ({rc}): {lib.wh_flac_last_error().decode(errors='replace')}")
    return out[: n.value], rate.value, bps.value


class DeviceAudio:
    """Audio already resident in a context's HBM (``HipContext.audio_upload``);
    ``transcribe`` then starts from device memory (no host-to-device copy)."""

    def __init__(self, ctx, n_samples: int):
        self.ctx = ctx
        self.n_samples = n_samples


def max_windows_limit(dims: dict, dtype: str, max_group: int) -> int:
    """Largest max_windows a context can hold: the self-attention kernels address one
    layer's self-K / V cache ([windows][max_group][n_text_ctx][n]) with 32-bit byte offsets,
    so it must stay under 2 GiB (wh_runtime.hip init refuses larger caches)."""
    elem = 2 if dtype == "fp16" else 4
    per_window = int(max_group) * int(dims["n_text_ctx"]) * int(dims["n_text_state"]) * elem
    return max(0, ((1 << 31) - 4096 - 1) // per_window)


class HipContext:
    """One libwhisper_hip context = one model on one GPU (per process)."""

    def __init__(self, dims: dict, device: int = 0, dtype: str = "fp16", max_windows: int = 8, max_group: int = 5):
        lim = max_windows_limit(dims, dtype, max_group)
        if max_windows > lim:
            raise ValueError(f"max_windows={max_windows} with max_group={max_group} in {dtype}: one layer's self-KV cache "
                             f"would exceed 2 GiB (32-bit offsets in the self-attention kernels); at most {lim} windows")
        self.lib = load_library()
        self.dims = dict(dims)
        self.dtype = dtype
        self.device = device
        self.max_windows = max_windows
        self.max_group = max_group
        d = WhDims(**{k: int(dims[k]) for k, _ in WhDims._fields_})
        h = c_void_p()
        code = {"fp16": WH_F16, "fp32": WH_F32}[dtype]
        self._check(self.lib.wh_create(device, ctypes.byref(d), code, max_windows, max_group, ctypes.byref(h)),
                    "wh_create")
        self.h = h

    # -- errors
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.wh_last_error().decode(errors="replace")
            raise HipBackendError(f"{what} failed ({rc}): {msg}")

    def close(self):
        """Release the context; raises HipBackendError if a HIP release failed (wh_destroy
        reports it instead of leaving the error pending for the next context)."""
        if getattr(self, "h", None):
            rc = self.lib.wh_destroy(self.h)
            # -1: refused (other contexts still read this one's weights), the context is
            # intact: keep the handle so close() can be retried once they are gone.  Any
            # other code: the context is released (a non-zero code reports a failed release)
            if rc != -1:
                self.h = None
            self._check(rc, "wh_destroy")

    def __del__(self):
        try:
            self.close()
        except HipBackendError as e:  # no raising from a finalizer: report it
            import warnings
            warnings.warn(str(e), RuntimeWarning)
        except Exception:
            pass

    # -- weights
    def load_tensor(self, name: str, value: np.ndarray):
        v = np.ascontiguousarray(value, dtype=np.float32)
        shape = (c_int64 * max(v.ndim, 1))(*v.shape)
        self._check(self.lib.wh_load_tensor(self.h, name.encode(), _ptr(v), shape, v.ndim), f"load {name}")

    def finalize(self):
        self._check(self.lib.wh_finalize(self.h), "wh_finalize")

    def set_mel_filters(self, n_mels: int, filters: np.ndarray):
        f = np.ascontiguousarray(filters, dtype=np.float32)
        assert f.shape == (n_mels, 201)
        self._check(self.lib.wh_set_mel_filters(self.h, n_mels, _ptr(f)), "wh_set_mel_filters")

    # -- mel
    def log_mel(self, audio: np.ndarray, n_mels: int, padding: int = 0, normalize: bool = True) -> int:
        a = np.ascontiguousarray(audio, dtype=np.float32)
        nf = c_int64()
        self._check(self.lib.wh_log_mel(self.h, _ptr(a), a.shape[0], int(padding), n_mels, int(normalize),
                                        ctypes.byref(nf)), "wh_log_mel")
        return nf.value

    def audio_upload(self, audio: np.ndarray) -> "DeviceAudio":
        a = np.ascontiguousarray(audio, dtype=np.float32)
        self._check(self.lib.wh_audio_upload(self.h, _ptr(a), a.shape[0]), "wh_audio_upload")
        return DeviceAudio(self, a.shape[0])

    def log_mel_resident(self, n_samples: int, n_mels: int, padding: int = 0, normalize: bool = True) -> int:
        nf = c_int64()
        self._check(self.lib.wh_log_mel(self.h, None, n_samples, int(padding), n_mels, int(normalize),
                                        ctypes.byref(nf)), "wh_log_mel")
        return nf.value

    def log_mel_frames(self, audio: Optional[np.ndarray], n_samples: int, n_mels: int, frame0: int, count: int,
                       padding: int = 0, normalize: bool = True) -> int:
        """Frames [frame0, frame0+count) of the padded file's log-mel (audio None: the
        resident buffer).  Returns the whole file's frame count."""
        a = None if audio is None else np.ascontiguousarray(audio, dtype=np.float32)
        tot = c_int64()
        self._check(self.lib.wh_log_mel_frames(self.h, None if a is None else _ptr(a), int(n_samples), int(padding),
                                               n_mels, int(frame0), int(count), int(normalize), ctypes.byref(tot)),
                    "wh_log_mel_frames")
        return tot.value

    def mel_max(self) -> float:
        g = c_float()
        self._check(self.lib.wh_mel_max(self.h, ctypes.byref(g)), "wh_mel_max")
        return g.value

    def mel_normalize(self, gmax: float):
        self._check(self.lib.wh_mel_normalize(self.h, float(gmax)), "wh_mel_normalize")

    def mel_read(self, n_mels: int, frame0: int, n_frames: int) -> np.ndarray:
        out = np.empty((n_mels, n_frames), dtype=np.float32)
        self._check(self.lib.wh_mel_read(self.h, _ptr(out), frame0, n_frames), "wh_mel_read")
        return out

    def mel_write(self, mel: np.ndarray):
        m = np.ascontiguousarray(mel, dtype=np.float32)
        self._check(self.lib.wh_mel_write(self.h, _ptr(m), m.shape[1]), "wh_mel_write")

    # -- encoder
    def encode(self, seeks: Sequence[int], segs: Sequence[int]):
        s = np.asarray(seeks, dtype=np.int64)
        g = np.asarray(segs, dtype=np.int32)
        self._check(self.lib.wh_encode(self.h, len(s), _ptr(s), _ptr(g)), "wh_encode")

    def audio_features(self, slot: int) -> np.ndarray:
        out = np.empty((self.dims["n_audio_ctx"], self.dims["n_audio_state"]), dtype=np.float32)
        self._check(self.lib.wh_read_audio_features(self.h, slot, _ptr(out)), "wh_read_audio_features")
        return out

    def cross_kv(self, slot: int, layer: int):
        H = self.dims["n_text_head"]
        k = np.empty((H, self.dims["n_audio_ctx"], 64), dtype=np.float32)
        v = np.empty_like(k)
        self._check(self.lib.wh_read_cross_kv(self.h, slot, layer, _ptr(k), _ptr(v)), "wh_read_cross_kv")
        return k, v

    # -- decoding
    def decode_begin(self, opts: WhDecodeOpts, init_tokens: Sequence[Sequence[int]], sot_index: Sequence[int],
                     slots: Optional[Sequence[int]] = None):
        """Decode window w = init_tokens[w] over encoder slot slots[w] (default w)."""
        n = len(init_tokens)
        mx = max(len(t) for t in init_tokens)
        arr = np.zeros((n, mx), dtype=np.int32)
        for i, t in enumerate(init_tokens):
            arr[i, :len(t)] = t
        nin = np.asarray([len(t) for t in init_tokens], dtype=np.int32)
        si = np.asarray(sot_index, dtype=np.int32)
        if slots is None:
            self._check(self.lib.wh_decode_begin(self.h, n, ctypes.byref(opts), _ptr(arr), _ptr(nin), mx, _ptr(si)),
                        "wh_decode_begin")
        else:
            sl = np.ascontiguousarray(slots, dtype=np.int32)
            assert len(sl) == n
            self._check(self.lib.wh_decode_begin_slots(self.h, n, _ptr(sl), ctypes.byref(opts), _ptr(arr), _ptr(nin),
                                                       mx, _ptr(si)), "wh_decode_begin_slots")

    def decode_steps(self, max_steps: int) -> int:
        nd = c_int()
        self._check(self.lib.wh_decode_steps(self.h, int(max_steps), ctypes.byref(nd)), "wh_decode_steps")
        return nd.value

    def decode_read(self, slot: int, group: int):
        hctx = self.dims["n_text_ctx"] + 1
        maxc = max(1, self.lib.wh_decode_maxc(self.h))
        toks = np.zeros((group, hctx), dtype=np.int32)
        slp = np.zeros(group, dtype=np.float32)
        ln = np.zeros(1, dtype=np.int32)
        fn = np.zeros(1, dtype=np.int32)
        ftok = np.zeros((maxc, hctx), dtype=np.int32)
        flen = np.zeros(maxc, dtype=np.int32)
        fsc = np.zeros(maxc, dtype=np.float32)
        nsp = np.zeros(1, dtype=np.float32)
        self._check(self.lib.wh_decode_read(self.h, slot, _ptr(toks), _ptr(slp), _ptr(ln), _ptr(fn), _ptr(ftok),
                                            _ptr(flen), _ptr(fsc), _ptr(nsp)), "wh_decode_read")
        n = int(fn[0])
        return dict(tokens=toks, sum_logprobs=slp, length=int(ln[0]), fin_tokens=ftok[:n], fin_len=flen[:n],
                    fin_score=fsc[:n], no_speech_prob=float(nsp[0]))

    # -- per-step boundary (decoder256Predict / decoder1Predict / rearrange_mkv roles)
    def prefill(self, init_tokens: Sequence[Sequence[int]], group: int, sot_index: Sequence[int],
                logits: bool = True):
        """wh_prefill: first pass of each window's initial tokens (windows = slots
        0..n-1); returns [n][2][V] logits at (sot_index, last) or None."""
        n = len(init_tokens)
        mx = max(len(t) for t in init_tokens)
        arr = np.zeros((n, mx), dtype=np.int32)
        for i, t in enumerate(init_tokens):
            arr[i, :len(t)] = t
        nin = np.asarray([len(t) for t in init_tokens], dtype=np.int32)
        si = np.asarray(sot_index, dtype=np.int32)
        out = np.empty((n, 2, self.dims["n_vocab"]), dtype=np.float32) if logits else None
        self._check(self.lib.wh_prefill(self.h, n, int(group), _ptr(arr), _ptr(nin), mx, _ptr(si),
                                        _ptr(out) if out is not None else None), "wh_prefill")
        return out

    def step(self, tokens: Sequence[int], text_offsets: Optional[Sequence[int]] = None, logits: bool = True):
        """wh_step: rows append ``tokens`` and run one decoder step; [rows][V] logits."""
        t = np.ascontiguousarray(tokens, dtype=np.int32)
        off = None if text_offsets is None else np.ascontiguousarray(text_offsets, dtype=np.int32)
        out = np.empty((len(t), self.dims["n_vocab"]), dtype=np.float32) if logits else None
        self._check(self.lib.wh_step(self.h, _ptr(t), _ptr(off) if off is not None else None,
                                     _ptr(out) if out is not None else None), "wh_step")
        return out

    def reorder_kv(self, source_rows: Sequence[int]):
        """wh_reorder_kv: row r continues row source_rows[r] (same window)."""
        s = np.ascontiguousarray(source_rows, dtype=np.int32)
        self._check(self.lib.wh_reorder_kv(self.h, _ptr(s)), "wh_reorder_kv")

    def prefill_logits(self, slot: int, tokens: Sequence[int], align_heads: Sequence[int] = ()):
        t = np.asarray(tokens, dtype=np.int32)
        V = self.dims["n_vocab"]
        lg = np.empty((len(t), V), dtype=np.float32)
        ah = np.asarray(align_heads, dtype=np.int32)
        qk = np.empty((len(ah), len(t), self.dims["n_audio_ctx"]), dtype=np.float32) if len(ah) else None
        self._check(self.lib.wh_prefill_logits(self.h, slot, _ptr(t), len(t), _ptr(lg),
                                               _ptr(ah) if len(ah) else None, len(ah),
                                               _ptr(qk) if qk is not None else None), "wh_prefill_logits")
        return lg, qk

    def align(self, slot: int, tokens: Sequence[int], n_sot: int, num_frames: int, align_heads: Sequence[int],
              medfilt_width: int = 7):
        """find_alignment's device half (timing.py:163-231): returns (text_token_probs [T],
        text_indices, time_indices) of dtw(-matrix)."""
        return self.align_batch([slot], [tokens], n_sot, [num_frames], align_heads, medfilt_width)[0]

    def align_batch(self, slots: Sequence[int], token_lists: Sequence[Sequence[int]], n_sot: int,
                    num_frames: Sequence[int], align_heads: Sequence[int], medfilt_width: int = 7):
        """wh_align_batch: one (probs, text_indices, time_indices) per window."""
        n = len(slots)
        toks = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.int32) for t in token_lists]))
        ntok = np.asarray([len(t) for t in token_lists], dtype=np.int32)
        nfr = np.asarray(num_frames, dtype=np.int32)
        sl = np.asarray(slots, dtype=np.int32)
        ah = np.ascontiguousarray(align_heads, dtype=np.int32)
        T = ntok - n_sot - 2
        widths = (T + 1) + nfr // 2
        probs = np.zeros(max(int(T.sum()), 1), dtype=np.float32)
        paths = np.zeros(max(int(2 * widths.sum()), 1), dtype=np.int32)
        plens = np.zeros(n, dtype=np.int32)
        self._check(self.lib.wh_align_batch(self.h, n, _ptr(sl), _ptr(toks), _ptr(ntok), n_sot, _ptr(nfr), _ptr(ah),
                                            len(ah), medfilt_width, _ptr(probs), _ptr(paths), _ptr(plens)),
                    "wh_align_batch")
        out, po, qo = [], 0, 0
        for w in range(n):
            L, W = int(plens[w]), int(widths[w])
            path = paths[qo:qo + 2 * W].reshape(2, W)
            out.append((probs[po:po + T[w]].copy(), path[0, :L].copy(), path[1, :L].copy()))
            po += int(T[w])
            qo += 2 * W
        return out

    def dtw(self, x: np.ndarray) -> np.ndarray:
        """timing.dtw(x) on the GPU: [2][path length] (text indices, time indices)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        N, M = x.shape
        path = np.zeros((2, N + M), dtype=np.int32)
        n = c_int(0)
        self._check(self.lib.wh_dtw(self.h, _ptr(x), N, M, _ptr(path), ctypes.byref(n)), "wh_dtw")
        return path[:, :n.value].copy()

    def stats(self) -> dict:
        out = (c_double * 8)()
        self._check(self.lib.wh_stats(self.h, out, 8), "wh_stats")
        keys = ["mel_ms", "encode_ms", "prefill_ms", "steps_ms", "steps", "encode_windows"]
        return {k: out[i] for i, k in enumerate(keys)}

    def sync(self):
        self._check(self.lib.wh_sync(self.h), "wh_sync")

    def token_ms(self, reset: bool = False) -> np.ndarray:
        """Per-token wall ms of each decode_steps chunk since the last reset."""
        n = c_int(0)
        self._check(self.lib.wh_token_ms(self.h, None, 0, ctypes.byref(n), 0), "wh_token_ms")
        out = np.zeros(max(n.value, 1), np.float32)
        self._check(self.lib.wh_token_ms(self.h, _ptr(out), n.value, ctypes.byref(n), int(reset)), "wh_token_ms")
        return out[:n.value]

    def step_kernels(self, n_win: int, group: int) -> dict:
        """The kernels the decoder step runs for this batch shape (wh_step_kernels):
        {"proj", "xattn", "self_attn", "tail"}."""
        buf = ctypes.create_string_buffer(256)
        n = self.lib.wh_step_kernels(self.h, n_win, group, buf, 256)
        self._check(0 if n >= 0 else n, "wh_step_kernels")
        return dict(kv.split("=", 1) for kv in buf.value.decode().split(","))

    def time_stage(self, what: int, iters: int) -> float:
        ms = c_double()
        self._check(self.lib.wh_time_stage(self.h, what, iters, ctypes.byref(ms)), "wh_time_stage")
        return ms.value
