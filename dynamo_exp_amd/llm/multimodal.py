"""Multimodal serving helpers (reference examples/multimodal: EncodeWorker
returns image features, the worker feeds them to the engine as
`multi_modal_data`).

* `make_vision_encoder(model_cfg, path)` -- CLIP tower + projector for a
  LLaVA config (safetensors from a checkpoint dir, else random init);
* `encode_urls(encoder, urls)` -> ([n_images * tokens_per_image, hidden], hash)
  where the hash covers the raw image bytes (prefix-cache identity);
* `encode_features` / `decode_features`: bf16 bytes + shape over the
  request plane (msgpack bin, no JSON float lists).
"""
from __future__ import annotations

import io
import os

import torch

from ..kv.hashing import xxh3_64
from ..models.vision import VisionEncoder, load_image


def make_vision_encoder(model_cfg, path: str | None, device: str = "cuda") -> VisionEncoder:
    if not model_cfg.vision:
        raise ValueError(f"{model_cfg.name} has no vision tower")
    enc = VisionEncoder(model_cfg.vision, model_cfg.hidden_size, device=device)
    if path and os.path.isdir(path) and any(f.endswith(".safetensors") for f in os.listdir(path)):
        return enc.load_safetensors(path)
    return enc.random_init(0)


def _image_bytes_hash(images) -> int:
    h = 0
    for im in images:
        buf = io.BytesIO()
        im.convert("RGB").save(buf, format="PNG")
        h = xxh3_64(buf.getvalue(), h)
    return h


def encode_urls(encoder: VisionEncoder, urls: list[str]) -> tuple[torch.Tensor, int]:
    images = [load_image(u) for u in urls]
    feats = encoder.encode_images(images)
    return feats.reshape(-1, feats.shape[-1]), _image_bytes_hash(images)


def encode_features(feats: torch.Tensor, h: int) -> dict:
    f = feats.detach().to(torch.bfloat16).contiguous().cpu()
    return {"features": f.view(torch.int16).numpy().tobytes(), "shape": list(f.shape), "hash": int(h)}


def decode_features(msg: dict, device) -> torch.Tensor:
    t = torch.frombuffer(bytearray(msg["features"]), dtype=torch.int16).view(torch.bfloat16)
    return t.view(*msg["shape"]).to(device)
