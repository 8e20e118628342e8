"""EncodeWorker (reference examples/multimodal/components/encode_worker.py):
image URL(s) -> CLIP tower + projector features, returned as bf16 bytes."""
import asyncio

import torch

from dynamo_exp_amd.llm.multimodal import encode_features, encode_urls, make_vision_encoder
from dynamo_exp_amd.models.config import get_config
from dynamo_exp_amd.sdk import ServiceConfig, async_on_start, dynamo_endpoint, service


@service(dynamo={"namespace": "dynamo"}, resources={"gpu": 1})
class EncodeWorker:
    @async_on_start
    async def async_init(self):
        cfg = ServiceConfig.get_instance()
        model = cfg.get("EncodeWorker", {}).get("model") or cfg.get("Common", {}).get("model", "llava-1.5-7b")
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        self.encoder = await asyncio.to_thread(make_vision_encoder, get_config(model), model, dev)

    @dynamo_endpoint()
    async def encode(self, request: dict):
        feats, h = await asyncio.to_thread(encode_urls, self.encoder, request["image_urls"])
        yield encode_features(feats, h)
