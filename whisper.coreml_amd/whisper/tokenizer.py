"""Token-id side of the reference tokenizer (whisper/tokenizer.py:132-395).

The hot path needs only ids: special tokens (laid out after the base BPE ranks
exactly as ``get_encoding`` does, tokenizer.py:331-363), the SuppressTokens
``-1`` set (``non_speech_tokens``, tokenizer.py:253-284) and ``encode(" ")``.
Those facts ship as data in assets/specials.json (exported from the reference
tokenizer by oracle/gen_golden.py).  Text needs the BPE rank files
(``multilingual.tiktoken`` / ``gpt2.tiktoken``, data the reference ships in
whisper/assets): they ship in assets/ too, WHISPER_TIKTOKEN_DIR overrides the
directory, and ``decode`` / ``encode`` raise when a file is missing.  ``encode`` is
tiktoken's byte-level BPE restated (tiktoken is a Rust dependency of the reference,
unpinned in requirements.txt; tokenizer.py:331-363 builds the Encoding): the text is
split by the encoding's regex, each piece's UTF-8 bytes are merged pairwise, lowest
merged rank first, until no adjacent pair is a token.
"""

import base64
import json
import os
import string
from dataclasses import dataclass, field
from functools import lru_cache
from typing import Dict, List, Optional, Tuple

_ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


@lru_cache(maxsize=None)
def _specials():
    with open(os.path.join(_ASSETS, "specials.json")) as f:
        return json.load(f)


LANGUAGES: Dict[str, str] = {c: n for c, n in _specials()["languages"]}
TO_LANGUAGE_CODE: Dict[str, str] = {**{n: c for c, n in LANGUAGES.items()}, **_specials()["to_language_code"]}


_RANK_OVERRIDE: Dict[str, Dict[int, bytes]] = {}


def set_token_bytes(encoding_name: str, table: Optional[Dict[int, bytes]]):
    """Install (or with None remove) an id -> bytes table for `encoding_name` in place
    of the BPE rank file (tests ship the few ids their fixtures decode)."""
    if table is None:
        _RANK_OVERRIDE.pop(encoding_name, None)
    else:
        _RANK_OVERRIDE[encoding_name] = dict(table)


def _ranks(name: str) -> Optional[Dict[int, bytes]]:
    if name in _RANK_OVERRIDE:
        return _RANK_OVERRIDE[name]
    return _rank_file(name)


@lru_cache(maxsize=None)
def _rank_file(name: str) -> Optional[Dict[int, bytes]]:
    """BPE ranks of `name` from WHISPER_TIKTOKEN_DIR if set, else the package assets
    (the reference ships the same two files in whisper/assets, tokenizer.py:332-336)."""
    d = os.environ.get("WHISPER_TIKTOKEN_DIR") or _ASSETS
    p = os.path.join(d, f"{name}.tiktoken")
    if not os.path.exists(p):
        return None
    out = {}
    with open(p) as f:
        for line in f:
            if line.strip():
                tok, rank = line.split()
                out[int(rank)] = base64.b64decode(tok)
    return out


# tokenizer.py:345-346 (both encodings use the GPT-2 split pattern)
_PAT = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


@lru_cache(maxsize=None)
def _encoder(name: str):
    ranks = _rank_file(name)
    if ranks is None:
        return None
    import regex
    return {b: r for r, b in ranks.items()}, regex.compile(_PAT)


def _bpe(piece: bytes, rank: Dict[bytes, int]) -> List[int]:
    if piece in rank:
        return [rank[piece]]
    parts = [piece[i:i + 1] for i in range(len(piece))]
    while len(parts) > 1:
        best, bi = None, -1
        for i in range(len(parts) - 1):
            r = rank.get(parts[i] + parts[i + 1])
            if r is not None and (best is None or r < best):
                best, bi = r, i
        if bi < 0:
            break
        parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
    return [rank[p] for p in parts]


@dataclass
class Tokenizer:
    encoding_name: str
    num_languages: int
    language: Optional[str] = None
    task: Optional[str] = None
    sot_sequence: Tuple[int, ...] = ()
    special_tokens: Dict[str, int] = field(default_factory=dict)

    def __post_init__(self):
        v = _specials()["vocab"][f"{self.encoding_name}_{self.num_languages}"]
        self._v = v
        base = v["n_base"]
        names = ["<|endoftext|>", "<|startoftranscript|>"]
        names += [f"<|{c}|>" for c in list(LANGUAGES)[: self.num_languages]]
        names += ["<|translate|>", "<|transcribe|>", "<|startoflm|>", "<|startofprev|>", "<|nospeech|>",
                  "<|notimestamps|>"]
        names += [f"<|{i * 0.02:.2f}|>" for i in range(1501)]
        self.special_tokens = {s: base + i for i, s in enumerate(names)}
        self.n_vocab = base + len(names)
        seq = [self.sot]
        if self.language is not None:
            seq.append(self.sot + 1 + list(LANGUAGES).index(self.language))
        if self.task is not None:
            seq.append(self.transcribe if self.task == "transcribe" else self.translate)
        self.sot_sequence = tuple(seq)

    # special ids (tokenizer.py:172-212)
    @property
    def eot(self) -> int:
        return self.special_tokens["<|endoftext|>"]

    @property
    def transcribe(self) -> int:
        return self.special_tokens["<|transcribe|>"]

    @property
    def translate(self) -> int:
        return self.special_tokens["<|translate|>"]

    @property
    def sot(self) -> int:
        return self.special_tokens["<|startoftranscript|>"]

    @property
    def sot_lm(self) -> int:
        return self.special_tokens["<|startoflm|>"]

    @property
    def sot_prev(self) -> int:
        return self.special_tokens["<|startofprev|>"]

    @property
    def no_speech(self) -> int:
        return self.special_tokens["<|nospeech|>"]

    @property
    def no_timestamps(self) -> int:
        return self.special_tokens["<|notimestamps|>"]

    @property
    def timestamp_begin(self) -> int:
        return self.special_tokens["<|0.00|>"]

    @property
    def language_token(self) -> int:
        if self.language is None:
            raise ValueError("This tokenizer does not have language token configured")
        return self.special_tokens[f"<|{self.language}|>"]

    @property
    def all_language_tokens(self) -> Tuple[int, ...]:
        return tuple(self.special_tokens[f"<|{c}|>"] for c in list(LANGUAGES)[: self.num_languages])

    @property
    def all_language_codes(self) -> Tuple[str, ...]:
        return tuple(list(LANGUAGES)[: self.num_languages])

    @property
    def sot_sequence_including_notimestamps(self) -> Tuple[int, ...]:
        return tuple(list(self.sot_sequence) + [self.no_timestamps])

    @property
    def non_speech_tokens(self) -> Tuple[int, ...]:
        return tuple(self._v["non_speech_tokens"])

    @property
    def whitespace_tokens(self) -> Tuple[int, ...]:
        return tuple(self._v["whitespace_tokens"])

    def encode_blank(self) -> List[int]:
        """tokenizer.encode(" ") used by SuppressBlank (decoding.py:457)."""
        return list(self._v["blank"])

    def is_blank_text(self, tokens: List[int]) -> bool:
        """True when decode(tokens).strip() == "" (transcribe.py:494-499)."""
        ws = set(self._v["whitespace_tokens"])
        return all(t in ws for t in tokens if t < self.eot)

    def encode(self, text: str) -> List[int]:
        """tokenizer.py:148-149 (``encoding.encode(text)``: plain text, no specials)."""
        enc = _encoder(self.encoding_name)
        if enc is None:
            raise RuntimeError(f"encode needs the BPE rank file {self.encoding_name}.tiktoken "
                               "(whisper/assets or WHISPER_TIKTOKEN_DIR)")
        rank, pat = enc
        out: List[int] = []
        for piece in pat.findall(text):
            out.extend(_bpe(piece.encode("utf-8"), rank))
        return out

    def decode(self, token_ids: List[int]) -> str:
        ranks = _ranks(self.encoding_name)
        if ranks is None:
            raise RuntimeError(f"decode needs the BPE rank file {self.encoding_name}.tiktoken "
                               "(whisper/assets or WHISPER_TIKTOKEN_DIR)")
        b = b"".join(ranks[t] for t in token_ids if t < self.timestamp_begin and t in ranks)
        return b.decode("utf-8", errors="replace")

    def decode_with_timestamps(self, token_ids: List[int]) -> str:
        ranks = _ranks(self.encoding_name) or {}
        inv = self._special_bytes()
        return b"".join(ranks[t] if t in ranks else inv.get(t, b"") for t in token_ids).decode("utf-8", errors="replace")

    def _special_bytes(self) -> Dict[int, bytes]:
        inv = self.__dict__.get("_inv_special")
        if inv is None:
            inv = {v: k.encode() for k, v in self.special_tokens.items()}
            self.__dict__["_inv_special"] = inv
        return inv

    # word splitting for word-level timestamps (tokenizer.py:277-327)
    def split_to_word_tokens(self, tokens: List[int]):
        """(words, word_tokens).  Tokens are first grouped into UTF-8-complete pieces;
        for space-delimited languages a piece then starts a new word if it is a special
        token, begins with a space, is punctuation, or is the first piece; otherwise it
        extends the previous word."""
        if _ranks(self.encoding_name) is None:
            raise RuntimeError("word timestamps need the BPE rank file "
                               f"{self.encoding_name}.tiktoken (whisper/assets or WHISPER_TIKTOKEN_DIR)")
        pieces = self._utf8_pieces(tokens)
        if self.language in {"zh", "ja", "th", "lo", "my", "yue"}:
            return [p for p, _ in pieces], [ids for _, ids in pieces]
        words: List[str] = []
        ids: List[List[int]] = []
        for text, group in pieces:
            if not words or group[0] >= self.eot or text.startswith(" ") or text.strip() in string.punctuation:
                words.append(text)
                ids.append(list(group))
            else:
                words[-1] += text
                ids[-1].extend(group)
        return words, ids

    def split_tokens_on_unicode(self, tokens: List[int]):
        pieces = self._utf8_pieces(tokens)
        return [p for p, _ in pieces], [ids for _, ids in pieces]

    def split_tokens_on_spaces(self, tokens: List[int]):
        return self.split_to_word_tokens(tokens)

    def _utf8_pieces(self, tokens: List[int]) -> List[Tuple[str, List[int]]]:
        """Consecutive tokens whose bytes decode together (tokenizer.py:286-311): a
        piece ends at the first token after which its text has no U+FFFD, or after
        which its first U+FFFD is also present at that place of the whole text (bytes
        that no following token completes)."""
        raw = [self._token_bytes(t) for t in tokens]
        whole = b"".join(raw).decode("utf-8", errors="replace")
        out: List[Tuple[str, List[int]]] = []
        begin, chars = 0, 0
        for stop in range(1, len(tokens) + 1):
            text = b"".join(raw[begin:stop]).decode("utf-8", errors="replace")
            bad = text.find("\ufffd")
            if bad < 0 or whole[chars + bad] == "\ufffd":
                out.append((text, list(tokens[begin:stop])))
                begin, chars = stop, chars + len(text)
        return out

    def _token_bytes(self, t: int) -> bytes:
        ranks = _ranks(self.encoding_name) or {}
        return ranks[t] if t in ranks else self._special_bytes().get(t, b"")


@lru_cache(maxsize=None)
def get_tokenizer(multilingual: bool, *, num_languages: int = 99, language: Optional[str] = None,
                  task: Optional[str] = None) -> Tokenizer:
    """tokenizer.py:367-395."""
    if language is not None:
        language = language.lower()
        if language not in LANGUAGES:
            if language in TO_LANGUAGE_CODE:
                language = TO_LANGUAGE_CODE[language]
            else:
                raise ValueError(f"Unsupported language: {language}")
    if multilingual:
        name = "multilingual"
        language = language or "en"
        task = task or "transcribe"
    else:
        name = "gpt2"
        language = None
        task = None
    return Tokenizer(name, num_languages, language, task)
