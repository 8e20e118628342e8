"""Model configurations (Llama family) and presets.

Presets cover the BASELINE.json configs: Llama-3-8B, Llama-3-70B and
DeepSeek-R1-Distill-Llama-8B (Llama-3.1-8B architecture), plus tiny test
models.  ``ModelConfig.from_hf_dir`` reads a HuggingFace ``config.json`` so a
local checkpoint directory (config + tokenizer, optional safetensors) works.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field

LLAMA3_ROPE_SCALING = {
    "rope_type": "llama3",
    "factor": 8.0,
    "low_freq_factor": 1.0,
    "high_freq_factor": 4.0,
    "original_max_position_embeddings": 8192,
}


@dataclass
class ModelConfig:
    name: str = "llama"
    architecture: str = "LlamaForCausalLM"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    bos_token_id: int = 128000
    eos_token_id: list[int] = field(default_factory=lambda: [128001, 128009])
    # multimodal (LLaVA): CLIP vision tower + projector config, image placeholder id
    vision: dict | None = None
    image_token_id: int | None = None

    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    def num_params(self) -> int:
        h, f, v, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_hidden_layers
        per_layer = h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * f + 2 * h
        return L * per_layer + v * h * (1 if self.tie_word_embeddings else 2) + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.num_hidden_layers * 2 * self.kv_size * dtype_bytes

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def from_hf_dir(cls, path: str) -> "ModelConfig":
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        vision = image_tok = None
        if "text_config" in c:  # LLaVA-style composite config
            vc = c.get("vision_config") or {}
            vision = dict(CLIP_L_336)
            vision.update({k: vc[k] for k in ("image_size", "patch_size", "hidden_size", "num_hidden_layers",
                                               "num_attention_heads", "intermediate_size", "layer_norm_eps")
                           if k in vc})
            vision["feature_layer"] = c.get("vision_feature_layer", -2)
            image_tok = c.get("image_token_index", 32000)
            c = {**c["text_config"], "architectures": c.get("architectures")}
            c.setdefault("vocab_size", 32064)
        heads = c["num_attention_heads"]
        eos = c.get("eos_token_id", 2)
        cfg = cls(
            name=os.path.basename(os.path.normpath(path)),
            architecture=(c.get("architectures") or ["LlamaForCausalLM"])[0],
            vocab_size=c["vocab_size"],
            hidden_size=c["hidden_size"],
            intermediate_size=c["intermediate_size"],
            num_hidden_layers=c["num_hidden_layers"],
            num_attention_heads=heads,
            num_key_value_heads=c.get("num_key_value_heads", heads),
            head_dim=c.get("head_dim", c["hidden_size"] // heads),
            rms_norm_eps=c.get("rms_norm_eps", 1e-5),
            rope_theta=c.get("rope_theta", 10000.0),
            rope_scaling=c.get("rope_scaling"),
            max_position_embeddings=c.get("max_position_embeddings", 8192),
            tie_word_embeddings=c.get("tie_word_embeddings", False),
            bos_token_id=c.get("bos_token_id", 1) or 1,
            eos_token_id=eos if isinstance(eos, list) else [eos],
            vision=vision,
            image_token_id=image_tok,
        )
        return cfg

    def write_hf_config(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        d = {
            "architectures": [self.architecture],
            "model_type": "llama",
            "vocab_size": self.vocab_size,
            "hidden_size": self.hidden_size,
            "intermediate_size": self.intermediate_size,
            "num_hidden_layers": self.num_hidden_layers,
            "num_attention_heads": self.num_attention_heads,
            "num_key_value_heads": self.num_key_value_heads,
            "head_dim": self.head_dim,
            "rms_norm_eps": self.rms_norm_eps,
            "rope_theta": self.rope_theta,
            "rope_scaling": self.rope_scaling,
            "max_position_embeddings": self.max_position_embeddings,
            "tie_word_embeddings": self.tie_word_embeddings,
            "bos_token_id": self.bos_token_id,
            "eos_token_id": self.eos_token_id,
            "torch_dtype": "bfloat16",
        }
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(d, f, indent=2)


# CLIP ViT-L/14 at 336 px, the LLaVA-1.5 vision tower; features from the
# second-to-last layer, CLS dropped, projected by a 2-layer GELU MLP
CLIP_L_336 = {
    "image_size": 336, "patch_size": 14, "hidden_size": 1024, "num_hidden_layers": 24, "num_attention_heads": 16,
    "intermediate_size": 4096, "layer_norm_eps": 1e-5, "feature_layer": -2,
}

PRESETS: dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig(name="Llama-3-8B", rope_theta=500000.0, rope_scaling=None, max_position_embeddings=8192),
    "llama3.1-8b": ModelConfig(name="Llama-3.1-8B", rope_scaling=dict(LLAMA3_ROPE_SCALING), max_position_embeddings=131072),
    "deepseek-r1-distill-llama-8b": ModelConfig(
        name="DeepSeek-R1-Distill-Llama-8B", rope_scaling=dict(LLAMA3_ROPE_SCALING), max_position_embeddings=131072,
        eos_token_id=[128001],
    ),
    "llama3-70b": ModelConfig(
        name="Llama-3-70B", hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
        num_key_value_heads=8, rope_scaling=None, max_position_embeddings=8192,
    ),
    "llama3.1-70b": ModelConfig(
        name="Llama-3.1-70B", hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
        num_key_value_heads=8, rope_scaling=dict(LLAMA3_ROPE_SCALING), max_position_embeddings=131072,
    ),
    "llama2-7b": ModelConfig(
        name="Llama-2-7B", vocab_size=32000, intermediate_size=11008, num_key_value_heads=32, rope_theta=10000.0,
        max_position_embeddings=4096, bos_token_id=1, eos_token_id=[2],
    ),
    "llava-1.5-7b": ModelConfig(
        name="llava-1.5-7b", architecture="LlavaForConditionalGeneration", vocab_size=32064, intermediate_size=11008,
        num_key_value_heads=32, rope_theta=10000.0, max_position_embeddings=4096, bos_token_id=1, eos_token_id=[2],
        vision=dict(CLIP_L_336), image_token_id=32000,
    ),
    # tiny models for CI / smoke (GQA 4 like Llama-3; head_dim 128 as the kernels require)
    "tiny": ModelConfig(
        name="tiny-llama", vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
        num_attention_heads=4, num_key_value_heads=1, head_dim=128, max_position_embeddings=4096,
        bos_token_id=1, eos_token_id=[2],
    ),
    "tiny-llava": ModelConfig(
        name="tiny-llava", architecture="LlavaForConditionalGeneration", vocab_size=512, hidden_size=256,
        intermediate_size=512, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=1, head_dim=128,
        max_position_embeddings=4096, bos_token_id=1, eos_token_id=[2], image_token_id=500,
        vision={"image_size": 56, "patch_size": 14, "hidden_size": 64, "num_hidden_layers": 3, "num_attention_heads": 4,
                "intermediate_size": 128, "layer_norm_eps": 1e-5, "feature_layer": -2},
    ),
    "small": ModelConfig(
        name="small-llama", vocab_size=32000, hidden_size=1024, intermediate_size=2816, num_hidden_layers=4,
        num_attention_heads=8, num_key_value_heads=2, head_dim=128, max_position_embeddings=8192,
        bos_token_id=1, eos_token_id=[2],
    ),
}


def get_config(name_or_path: str) -> ModelConfig:
    """A preset, an HF directory, or `<preset>@<layers>`: the preset's
    architecture truncated to its first <layers> decoder layers (one-GPU
    rehearsals of a big model's TP / transfer mechanics at its real layer
    shapes; never a throughput number for the full model)."""
    if "@" in name_or_path and not os.path.isdir(name_or_path):
        base, n = name_or_path.rsplit("@", 1)
        cfg = get_config(base)
        layers = int(n)
        if not 1 <= layers <= cfg.num_hidden_layers:
            raise ValueError(f"{name_or_path!r}: layer count must be 1..{cfg.num_hidden_layers}")
        return dataclasses.replace(cfg, num_hidden_layers=layers,
                                   name=f"{cfg.name} ({layers} of {cfg.num_hidden_layers} layers)")
    if name_or_path in PRESETS:
        return dataclasses.replace(PRESETS[name_or_path])
    if os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "config.json")):
        return ModelConfig.from_hf_dir(name_or_path)
    key = name_or_path.lower().replace("meta-llama/", "").replace("meta-", "")
    for k in PRESETS:
        if k.replace(".", "").replace("-", "") in key.replace(".", "").replace("-", "").replace("_", ""):
            return dataclasses.replace(PRESETS[k])
    raise ValueError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")
