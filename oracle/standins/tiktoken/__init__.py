"""Stand-in for the absent `tiktoken` package (golden generation only).

tiktoken (Rust, unpinned in reference requirements.txt:6) is a byte-pair
encoder: the text is split by the regex `pat_str`, each piece is encoded as
bytes and adjacent byte-strings are merged lowest-rank-first while the merged
string is in `mergeable_ranks`.  This restates that published algorithm so the
reference's tokenizer (whisper/tokenizer.py:132-363) can run here.  It only
decides the ids of special/suppressed tokens and of text; it is not on the
hot path.  Verified: " And so my fellow Americans" -> [400, 370, 452, 7177, 6280]
(SURVEY.md §8(c)).
"""

import regex


class Encoding:
    def __init__(self, name, explicit_n_vocab=None, pat_str="", mergeable_ranks=None,
                 special_tokens=None):
        self.name = name
        self.n_vocab = explicit_n_vocab
        self._pat = regex.compile(pat_str)
        self._ranks = dict(mergeable_ranks or {})
        self._special = dict(special_tokens or {})
        self._decoder = {v: k for k, v in self._ranks.items()}
        for s, i in self._special.items():
            self._decoder[i] = s.encode("utf-8")

    @property
    def special_tokens_set(self):
        return set(self._special.keys())

    @property
    def eot_token(self):
        return self._special["<|endoftext|>"]

    def encode_single_token(self, text):
        if isinstance(text, str) and text in self._special:
            return self._special[text]
        b = text.encode("utf-8") if isinstance(text, str) else text
        return self._ranks[b]

    def _bpe(self, piece: bytes):
        if piece in self._ranks:
            return [self._ranks[piece]]
        parts = [bytes([c]) for c in piece]
        while len(parts) > 1:
            best, best_i = None, -1
            for i in range(len(parts) - 1):
                r = self._ranks.get(parts[i] + parts[i + 1])
                if r is not None and (best is None or r < best):
                    best, best_i = r, i
            if best is None:
                break
            parts = parts[:best_i] + [parts[best_i] + parts[best_i + 1]] + parts[best_i + 2:]
        return [self._ranks[p] for p in parts]

    def encode(self, text, allowed_special=(), disallowed_special=()):
        out = []
        for piece in self._pat.findall(text):
            out.extend(self._bpe(piece.encode("utf-8")))
        return out

    def decode_bytes(self, tokens):
        return b"".join(self._decoder[t] for t in tokens)

    def decode(self, tokens, errors="replace"):
        return self.decode_bytes(tokens).decode("utf-8", errors=errors)
