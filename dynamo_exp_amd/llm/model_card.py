"""Model Deployment Card (MDC) and LocalModel registration.

The MDC describes how to talk to a model: display/service name, model config,
tokenizer and prompt-formatter files and context mixins, plus a checksum
(`mdcsum`).  Workers publish it so frontends can build the preprocessing
pipeline without local model files: file contents go to the control plane's
blob store (bucket `mdc`, TTL 5 min like the reference's NATS object store,
lib/llm/src/model_card.rs:30, model/model.rs:233-281) and the card itself to
the KV store.  `attach()` registers a ModelEntry under the endpoint's lease
(local_model.rs:124-163) for the HTTP frontend's model watcher.
"""
from __future__ import annotations

import hashlib
import json
import os
import tempfile
import time
from dataclasses import asdict, dataclass, field
from typing import Any

from ..models.config import ModelConfig, get_config

BUCKET = "mdc"
BUCKET_TTL = 300.0
MODELS_PREFIX = "models/"
MDC_PREFIX = "mdc/"

MODEL_TYPES = ("chat", "completion", "backend")


@dataclass
class ModelDeploymentCard:
    display_name: str
    service_name: str
    model_info: dict[str, Any] = field(default_factory=dict)  # config.json
    tokenizer_files: dict[str, str] = field(default_factory=dict)  # name -> local path or blob:// ref
    prompt_context: list[str] = field(default_factory=list)  # e.g. ["llama3_date_time"]
    kv_block_size: int = 64
    context_length: int = 8192
    revision: int = 0
    last_published: float = 0.0

    def mdcsum(self) -> str:
        d = asdict(self)
        d.pop("last_published", None)
        return hashlib.sha256(json.dumps(d, sort_keys=True).encode()).hexdigest()[:16]

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s: str | bytes) -> "ModelDeploymentCard":
        return cls(**json.loads(s))

    @property
    def slug(self) -> str:
        return "".join(c if c.isalnum() or c in "-_" else "_" for c in self.service_name.lower())

    # ----------------------------------------------------------- construction
    @classmethod
    def load(cls, model: str, name: str | None = None, block_size: int = 64) -> "ModelDeploymentCard":
        """From an HF directory (config + tokenizer files) or a preset name."""
        files = {}
        if os.path.isdir(model):
            cfg = ModelConfig.from_hf_dir(model)
            for f in ("config.json", "tokenizer.json", "tokenizer_config.json", "generation_config.json"):
                p = os.path.join(model, f)
                if os.path.exists(p):
                    files[f] = p
            info = json.load(open(os.path.join(model, "config.json")))
        else:
            cfg = get_config(model)
            info = cfg.to_dict()
        disp = name or (os.path.basename(os.path.normpath(model)) if os.path.isdir(model) else cfg.name)
        return cls(display_name=disp, service_name=disp, model_info=info, tokenizer_files=files,
                   kv_block_size=block_size, context_length=cfg.max_position_embeddings,
                   prompt_context=["llama3_date_time"] if "llama" in cfg.architecture.lower() else [])

    def model_config(self) -> ModelConfig:
        if "architectures" in self.model_info:
            d = tempfile.mkdtemp(prefix="dx_mdc_cfg_")
            with open(os.path.join(d, "config.json"), "w") as f:
                json.dump(self.model_info, f)
            return ModelConfig.from_hf_dir(d)
        return ModelConfig.from_dict(self.model_info)

    def local_dir(self) -> str | None:
        """Directory holding the tokenizer files, if local."""
        for p in self.tokenizer_files.values():
            if not p.startswith("blob://") and os.path.exists(p):
                return os.path.dirname(p)
        return None

    # ----------------------------------------------------------- blob store
    async def move_to_blob_store(self, cp) -> "ModelDeploymentCard":
        out = dict(self.tokenizer_files)
        for name, path in self.tokenizer_files.items():
            if path.startswith("blob://"):
                continue
            with open(path, "rb") as f:
                await cp.blob_put(BUCKET, f"{self.slug}/{name}", f.read(), ttl=BUCKET_TTL)
            out[name] = f"blob://{BUCKET}/{self.slug}/{name}"
        self.tokenizer_files = out
        return self

    async def move_from_blob_store(self, cp, dest: str | None = None) -> "ModelDeploymentCard":
        dest = dest or tempfile.mkdtemp(prefix=f"dx_mdc_{self.slug}_")
        out = dict(self.tokenizer_files)
        for name, ref in self.tokenizer_files.items():
            if not ref.startswith("blob://"):
                continue
            _, _, rest = ref.partition("blob://")
            bucket, _, key = rest.partition("/")
            data = await cp.blob_get(bucket, key)
            if data is None:
                raise FileNotFoundError(f"{ref} expired or missing")
            p = os.path.join(dest, name)
            with open(p, "wb") as f:
                f.write(data)
            out[name] = p
        self.tokenizer_files = out
        return self


@dataclass
class ModelEntry:
    """Frontend-visible registration: model name -> serving endpoint."""

    name: str
    endpoint: str  # "ns/component/endpoint"
    model_type: str  # chat | completion | backend
    mdc_key: str | None = None
    router_mode: str = "round_robin"  # round_robin | random | kv
    kv_block_size: int = 64

    def to_json(self) -> bytes:
        return json.dumps(asdict(self)).encode()

    @classmethod
    def from_json(cls, b: bytes) -> "ModelEntry":
        return cls(**json.loads(b))


def model_key(model_type: str, name: str, lease_id: int = 0) -> str:
    """`models/{type}/{name}:{lease}` (one entry per serving instance)."""
    return f"{MODELS_PREFIX}{model_type}/{name}:{lease_id:x}"


async def attach(drt, endpoint, card: ModelDeploymentCard, model_type: str = "backend", router_mode: str = "round_robin",
                 lease=None) -> ModelEntry:
    """Publish the card + a ModelEntry bound to the endpoint's lease."""
    assert model_type in MODEL_TYPES
    cp = drt.cp
    lease = lease or drt.primary_lease
    lid = lease.id if lease else 0
    await card.move_to_blob_store(cp)
    card.last_published = time.time()
    mdc_key = f"{MDC_PREFIX}{card.slug}"
    await cp.put(mdc_key, card.to_json().encode())
    entry = ModelEntry(card.display_name, endpoint.path, model_type, mdc_key, router_mode, card.kv_block_size)
    await cp.put(model_key(model_type, card.display_name, lid), entry.to_json(), lease=lid if lease else None)
    return entry
