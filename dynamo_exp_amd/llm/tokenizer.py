"""Tokenizers and incremental detokenization.

* `HFTokenizer` wraps a HuggingFace `tokenizer.json` via the `tokenizers`
  library (reference lib/llm/src/tokenizers/hf.rs).
* `SyntheticTokenizer` is a deterministic byte-level tokenizer used for
  random-init models when no tokenizer files exist offline (bench / tests).
* `DecodeStream` detokenizes incrementally with a bounded window
  (prefix_offset/read_offset), fixing the reference's O(n^2) re-decode of the
  whole sequence every step (lib/llm/src/tokenizers.rs:211-233).
"""
from __future__ import annotations

import json
import os
from typing import Iterable


class Tokenizer:
    eos_token_ids: list[int] = []
    bos_token_id: int | None = None
    bos_token: str = ""
    eos_token: str = ""
    vocab_size: int = 0

    def encode(self, text: str, add_special_tokens: bool = False) -> list[int]:
        raise NotImplementedError

    def decode(self, ids: Iterable[int], skip_special_tokens: bool = True) -> str:
        raise NotImplementedError

    def decode_stream(self, prompt_ids: list[int] | None = None, skip_special_tokens: bool = True) -> "DecodeStream":
        return DecodeStream(self, prompt_ids or [], skip_special_tokens)


class HFTokenizer(Tokenizer):
    def __init__(self, path: str):
        from tokenizers import Tokenizer as _T

        tj = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
        self.tk = _T.from_file(tj)
        self.vocab_size = self.tk.get_vocab_size(with_added_tokens=True)
        cfg = {}
        d = os.path.dirname(tj)
        tc = os.path.join(d, "tokenizer_config.json")
        if os.path.exists(tc):
            with open(tc) as f:
                cfg = json.load(f)
        self.config = cfg

        def tok_str(v):
            return v.get("content") if isinstance(v, dict) else v

        self.bos_token = tok_str(cfg.get("bos_token")) or ""
        self.eos_token = tok_str(cfg.get("eos_token")) or ""
        self.bos_token_id = self.tk.token_to_id(self.bos_token) if self.bos_token else None
        eid = self.tk.token_to_id(self.eos_token) if self.eos_token else None
        self.eos_token_ids = [eid] if eid is not None else []
        gen = os.path.join(d, "generation_config.json")
        if os.path.exists(gen):
            with open(gen) as f:
                g = json.load(f)
            e = g.get("eos_token_id")
            if e is not None:
                self.eos_token_ids = list(dict.fromkeys((e if isinstance(e, list) else [e]) + self.eos_token_ids))

    def encode(self, text: str, add_special_tokens: bool = False) -> list[int]:
        return self.tk.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        return self.tk.decode(list(ids), skip_special_tokens=skip_special_tokens)

    @property
    def chat_template(self) -> str | None:
        t = self.config.get("chat_template")
        if isinstance(t, list):  # named templates
            for e in t:
                if e.get("name") == "default":
                    return e.get("template")
            return t[0].get("template") if t else None
        return t


class SyntheticTokenizer(Tokenizer):
    """Byte-level: ids 0..255 are raw bytes; a few special tokens; every other
    id decodes to a short pseudo-word so random-init generations are printable."""

    SPECIALS = {"<|begin_of_text|>": 0, "<|end_of_text|>": 1, "<|eot_id|>": 2, "<|start_header_id|>": 3,
                "<|end_header_id|>": 4}

    def __init__(self, vocab_size: int = 128256, bos_token_id: int = 128000, eos_token_ids: list[int] | None = None):
        self.vocab_size = vocab_size
        self.offset = 256  # bytes live at [offset, offset+256)
        self.bos_token_id = bos_token_id if bos_token_id < vocab_size else 0
        self.eos_token_ids = list(eos_token_ids or [min(vocab_size - 1, 128001)])
        self.bos_token = "<|begin_of_text|>"
        self.eos_token = "<|end_of_text|>"
        self.special_ids = {self.bos_token_id: self.bos_token}
        for e in self.eos_token_ids:
            self.special_ids[e] = self.eos_token
        self.special_ids.setdefault(2, "<|eot_id|>")
        self._sp_text = {v: k for k, v in self.special_ids.items()}

    def encode(self, text: str, add_special_tokens: bool = False) -> list[int]:
        ids = [self.bos_token_id] if add_special_tokens else []
        i = 0
        # special tokens embedded in text (chat templates)
        while i < len(text):
            if text[i] == "<":
                hit = next((s for s in self._sp_text if text.startswith(s, i)), None)
                if hit:
                    ids.append(self._sp_text[hit])
                    i += len(hit)
                    continue
            j = text.find("<", i + 1)
            j = len(text) if j < 0 else j
            ids.extend(self.offset + b for b in text[i:j].encode("utf-8"))
            i = j
        return ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        out = bytearray()
        for t in ids:
            t = int(t)
            if t in self.special_ids:
                if not skip_special_tokens:
                    out += self.special_ids[t].encode()
            elif self.offset <= t < self.offset + 256:
                out.append(t - self.offset)
            else:
                out += f" w{t}".encode()
        return out.decode("utf-8", errors="replace")


class DecodeStream:
    """Incremental detokenizer: emits only complete (non-replacement-char)
    text; each step decodes a bounded window, so cost is O(1) in length."""

    def __init__(self, tok: Tokenizer, prompt_ids: list[int], skip_special_tokens: bool = True):
        self.tok = tok
        self.skip = skip_special_tokens
        self.ids: list[int] = list(prompt_ids[-6:])
        self.prefix_offset = 0
        self.read_offset = len(self.ids)
        # byte-level synthetic tokenizer: incremental UTF-8 over the pending
        # bytes only (no window re-decodes; it serves the random-init presets
        # the benchmarks stream)
        self._bytes = bytearray() if isinstance(tok, SyntheticTokenizer) else None

    def _step_bytes(self, t: int) -> str | None:
        tok = self.tok
        if t in tok.special_ids:
            text = "" if self.skip else tok.special_ids[t]
        elif tok.offset <= t < tok.offset + 256:
            self._bytes.append(t - tok.offset)
            try:
                text = self._bytes.decode("utf-8")
            except UnicodeDecodeError as e:
                if e.reason == "unexpected end of data" and len(self._bytes) < 4:
                    return None  # an incomplete multi-byte character: wait for its next byte
                text = self._bytes.decode("utf-8", errors="replace")
            self._bytes.clear()
            return text or None
        else:
            text = f" w{t}"
        if self._bytes:  # a dangling partial character ends here
            text = self._bytes.decode("utf-8", errors="replace") + text
            self._bytes.clear()
        return text or None

    def step(self, token_id: int) -> str | None:
        if self._bytes is not None:
            return self._step_bytes(int(token_id))
        self.ids.append(int(token_id))
        prefix_text = self.tok.decode(self.ids[self.prefix_offset:self.read_offset], self.skip)
        new_text = self.tok.decode(self.ids[self.prefix_offset:], self.skip)
        if len(new_text) > len(prefix_text) and not new_text.endswith("�"):
            delta = new_text[len(prefix_text):]
            self.prefix_offset = self.read_offset
            self.read_offset = len(self.ids)
            if self.prefix_offset > 64:  # keep the window bounded
                cut = self.prefix_offset - 6
                self.ids = self.ids[cut:]
                self.prefix_offset -= cut
                self.read_offset -= cut
            return delta
        return None


def load_tokenizer(path: str | None, vocab_size: int = 128256, bos: int = 128000,
                   eos: list[int] | None = None) -> Tokenizer:
    if path and os.path.exists(os.path.join(path, "tokenizer.json")):
        return HFTokenizer(path)
    return SyntheticTokenizer(vocab_size, bos, eos)
