"""LLaVA-style vision encoder: CLIP ViT tower + 2-layer GELU projector
(reference examples/multimodal/components/encode_worker.py:40-82, which runs
HF `LlavaForConditionalGeneration.vision_tower` + `multi_modal_projector`).

Image -> [num_patches, text_hidden] embeddings that replace the image
placeholder tokens of the prompt.  Pre-LN ViT:
    x = patch_embed(img) (+ CLS) + pos;  x = pre_ln(x)
    per layer: x += attn(ln1(x)) (bidirectional, biased q/k/v/o);  x += fc2(quick_gelu(fc1(ln2(x))))
features = hidden state of layer `feature_layer` (-2) without CLS, then
    linear_2(gelu(linear_1(features))).
GEMMs run on hipBLASLt (torch.matmul in bf16); the 577-token bidirectional
attention (ViT-L: 16 heads x 577^2, head dim 64) runs on the prefill
attention HIP kernel in its non-causal mode (head dim zero-padded to 128);
DX_VISION_HIP_ATTN=0 (or a CPU device) keeps two batched GEMMs around an
fp32 softmax.
"""
from __future__ import annotations

import glob
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def preprocess_image(img, size: int) -> torch.Tensor:
    """PIL image -> [3, size, size] float32 (CLIPImageProcessor: shortest side
    resize, bicubic; center crop; scale; normalize)."""
    from PIL import Image

    img = img.convert("RGB")
    w, h = img.size
    s = size / min(w, h)
    img = img.resize((max(size, round(w * s)), max(size, round(h * s))), Image.BICUBIC)
    w, h = img.size
    left, top = (w - size) // 2, (h - size) // 2
    img = img.crop((left, top, left + size, top + size))
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = (a - np.array(CLIP_MEAN, dtype=np.float32)) / np.array(CLIP_STD, dtype=np.float32)
    return torch.from_numpy(a.transpose(2, 0, 1).copy())


def load_image(src: str):
    """Local path or data: URL (no network access in this deployment)."""
    import base64
    import io

    from PIL import Image

    if src.startswith("data:"):
        payload = src.split(",", 1)[1]
        return Image.open(io.BytesIO(base64.b64decode(payload)))
    if src.startswith("file://"):
        src = src[7:]
    if src.startswith("http://") or src.startswith("https://"):
        raise ValueError("remote image URLs are not fetched; pass a local path or a data: URL")
    return Image.open(src)


class VisionEncoder:
    def __init__(self, vcfg: dict, text_hidden: int, device="cuda", dtype=torch.bfloat16):
        self.c = vcfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.text_hidden = text_hidden
        self.H = vcfg["hidden_size"]
        self.heads = vcfg["num_attention_heads"]
        self.P = vcfg["patch_size"]
        self.n_patches = (vcfg["image_size"] // self.P) ** 2
        self.eps = vcfg.get("layer_norm_eps", 1e-5)
        self.feature_layer = vcfg.get("feature_layer", -2)
        self.w: dict[str, torch.Tensor] = {}
        self.layers: list[dict] = []

    @property
    def num_image_tokens(self) -> int:
        return self.n_patches

    # ------------------------------------------------------------------ weights
    def random_init(self, seed: int = 0) -> "VisionEncoder":
        g = torch.Generator().manual_seed(seed + 7919)
        H, I, P = self.H, self.c["intermediate_size"], self.P

        def rn(*shape, std=0.02):
            return (torch.randn(*shape, generator=g) * std).to(self.dtype).to(self.device)

        def ones(n):
            return torch.ones(n, dtype=self.dtype, device=self.device)

        def zeros(n):
            return torch.zeros(n, dtype=self.dtype, device=self.device)

        self.w = dict(patch=rn(H, 3 * P * P), cls=rn(H), pos=rn(self.n_patches + 1, H), pre_ln_w=ones(H),
                      pre_ln_b=zeros(H), proj1_w=rn(self.text_hidden, H), proj1_b=zeros(self.text_hidden),
                      proj2_w=rn(self.text_hidden, self.text_hidden), proj2_b=zeros(self.text_hidden))
        self.layers = []
        for _ in range(self.c["num_hidden_layers"]):
            self.layers.append(dict(ln1_w=ones(H), ln1_b=zeros(H), qkv_w=rn(3 * H, H), qkv_b=zeros(3 * H),
                                    o_w=rn(H, H), o_b=zeros(H), ln2_w=ones(H), ln2_b=zeros(H), fc1_w=rn(I, H),
                                    fc1_b=zeros(I), fc2_w=rn(H, I), fc2_b=zeros(H)))
        return self

    def load_safetensors(self, path: str) -> "VisionEncoder":
        """HF LLaVA checkpoint (vision_tower.vision_model.* / multi_modal_projector.*)."""
        from safetensors import safe_open

        t = {}
        for f in sorted(glob.glob(os.path.join(path, "*.safetensors"))):
            with safe_open(f, framework="pt") as sf:
                for k in sf.keys():
                    if k.startswith("vision_tower.") or k.startswith("multi_modal_projector."):
                        t[k] = sf.get_tensor(k)
        d = lambda x: x.to(self.dtype).to(self.device)  # noqa: E731
        vp = "vision_tower.vision_model."
        H, P = self.H, self.P
        self.w = dict(
            patch=d(t[vp + "embeddings.patch_embedding.weight"].reshape(H, 3 * P * P)),
            cls=d(t[vp + "embeddings.class_embedding"]), pos=d(t[vp + "embeddings.position_embedding.weight"]),
            pre_ln_w=d(t[vp + "pre_layrnorm.weight"]), pre_ln_b=d(t[vp + "pre_layrnorm.bias"]),
            proj1_w=d(t["multi_modal_projector.linear_1.weight"]), proj1_b=d(t["multi_modal_projector.linear_1.bias"]),
            proj2_w=d(t["multi_modal_projector.linear_2.weight"]), proj2_b=d(t["multi_modal_projector.linear_2.bias"]))
        self.layers = []
        for i in range(self.c["num_hidden_layers"]):
            p = f"{vp}encoder.layers.{i}."
            a = p + "self_attn."
            self.layers.append(dict(
                ln1_w=d(t[p + "layer_norm1.weight"]), ln1_b=d(t[p + "layer_norm1.bias"]),
                qkv_w=d(torch.cat([t[a + f"{n}_proj.weight"] for n in "qkv"])),
                qkv_b=d(torch.cat([t[a + f"{n}_proj.bias"] for n in "qkv"])),
                o_w=d(t[a + "out_proj.weight"]), o_b=d(t[a + "out_proj.bias"]),
                ln2_w=d(t[p + "layer_norm2.weight"]), ln2_b=d(t[p + "layer_norm2.bias"]),
                fc1_w=d(t[p + "mlp.fc1.weight"]), fc1_b=d(t[p + "mlp.fc1.bias"]),
                fc2_w=d(t[p + "mlp.fc2.weight"]), fc2_b=d(t[p + "mlp.fc2.bias"])))
        return self

    # ------------------------------------------------------------------ forward
    def _hip_attn(self, hd: int) -> bool:
        return (self.device.type == "cuda" and self.dtype == torch.bfloat16 and hd <= 128 and hd % 8 == 0
                and os.environ.get("DX_VISION_HIP_ATTN", "1") != "0")

    def _attn_plan(self, N: int, T: int, nh: int, hd: int) -> dict:
        """Per-forward state of the HIP attention path: the block table, cu /
        ctx lengths and the kernel's work list depend only on (N, T), so they
        are built once per encode (host-side, one H2D each) instead of once
        per layer; the zero-padded q / K / V buffers are allocated once too
        and only their live columns are overwritten per layer."""
        from .. import ops

        D, BS = 128, 64
        nb = -(-T // BS)
        dev, dt = self.device, self.dtype
        work = ops.prefill_work_list([T] * N, [T] * N, nh, nh)
        return {"nb": nb, "D": D, "BS": BS,
                "q": torch.zeros((N * T, nh, D), device=dev, dtype=dt),
                "kv": torch.zeros((2, N, nb, nh, BS, D), device=dev, dtype=dt),
                "src": torch.zeros((N, nb * BS, nh, hd), device=dev, dtype=dt),
                "bt": torch.arange(N * nb, dtype=torch.int32).view(N, nb).to(dev, non_blocking=True),
                "cu": torch.arange(0, N * T + 1, T, dtype=torch.int32).to(dev, non_blocking=True),
                "ctx": torch.full((N,), T, dtype=torch.int32).to(dev, non_blocking=True),
                "work": torch.tensor(work, dtype=torch.int32).to(dev, non_blocking=True)}

    def _attention_hip(self, qkv: torch.Tensor, scale: float, plan: dict | None = None) -> torch.Tensor:
        """Bidirectional attention of every image's T tokens on the prefill
        attention kernel (csrc/kernels/attn_prefill.hip, causal=0): q/k/v are
        zero-padded to the kernel's head dim 128 (the padding adds nothing to
        q.k and yields zero output columns) and K/V laid out as a 64-token
        paged cache with one block table row per image.  qkv: [N, T, 3, nh, hd]
        -> [N * T, nh, hd]."""
        from .. import ops

        N, T, _, nh, hd = qkv.shape
        if plan is None:
            plan = self._attn_plan(N, T, nh, hd)
        nb, D, BS = plan["nb"], plan["D"], plan["BS"]
        q, kv, src = plan["q"], plan["kv"], plan["src"]
        q[:, :, :hd] = qkv[:, :, 0].reshape(N * T, nh, hd)
        for i in (0, 1):  # [N, T, nh, hd] -> blocks [N, nb, nh, BS, hd]; padding rows stay zero
            src[:, :T] = qkv[:, :, 1 + i]
            kv[i, ..., :hd] = src.view(N, nb, BS, nh, hd).transpose(2, 3)
        kc, vc = kv[0].view(N * nb, nh, BS, D), kv[1].view(N * nb, nh, BS, D)
        out = torch.empty_like(q)
        ops.prefill_attention(q, kc, vc, plan["bt"], plan["cu"], plan["ctx"], scale, out, work=plan["work"],
                              causal=False)
        return out[:, :, :hd]

    def _ln(self, x, w, b):
        return F.layer_norm(x.float(), (self.H,), w.float(), b.float(), self.eps).to(self.dtype)

    @torch.inference_mode()
    def encode(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [N, 3, S, S] float -> [N, n_patches, text_hidden] (dtype)."""
        N = pixels.shape[0]
        P, H, nh = self.P, self.H, self.heads
        x = pixels.to(self.device, torch.float32)
        patches = F.unfold(x, kernel_size=P, stride=P).transpose(1, 2)  # [N, np, 3*P*P] (c, kh, kw order)
        h = torch.matmul(patches.to(self.dtype), self.w["patch"].t())
        cls = self.w["cls"].view(1, 1, H).expand(N, 1, H)
        h = torch.cat([cls, h], 1) + self.w["pos"].unsqueeze(0)
        h = self._ln(h, self.w["pre_ln_w"], self.w["pre_ln_b"])
        n_layers = len(self.layers)
        stop = self.feature_layer % (n_layers + 1)  # hidden_states index: 0 = embeddings
        T = h.shape[1]
        hd = H // nh
        scale = 1.0 / math.sqrt(hd)
        plan = self._attn_plan(N, T, nh, hd) if self._hip_attn(hd) else None
        for li in range(stop):
            L = self.layers[li]
            y = self._ln(h, L["ln1_w"], L["ln1_b"])
            qkv = torch.addmm(L["qkv_b"], y.view(N * T, H), L["qkv_w"].t()).view(N, T, 3, nh, hd)
            if self._hip_attn(hd):
                a = self._attention_hip(qkv, scale, plan).reshape(N * T, H)
            else:
                q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))  # [N, nh, T, hd]
                s = torch.matmul(q, k.transpose(-1, -2)).float() * scale
                p = torch.softmax(s, dim=-1).to(self.dtype)
                a = torch.matmul(p, v).transpose(1, 2).reshape(N * T, H)
            h = h + torch.addmm(L["o_b"], a, L["o_w"].t()).view(N, T, H)
            y = self._ln(h, L["ln2_w"], L["ln2_b"]).view(N * T, H)
            f = torch.addmm(L["fc1_b"], y, L["fc1_w"].t())
            f = (f.float() * torch.sigmoid(1.702 * f.float())).to(self.dtype)  # quick_gelu
            h = h + torch.addmm(L["fc2_b"], f, L["fc2_w"].t()).view(N, T, H)
        feats = h[:, 1:].reshape(N * (T - 1), H)  # drop CLS
        z = torch.addmm(self.w["proj1_b"], feats, self.w["proj1_w"].t())
        z = F.gelu(z.float()).to(self.dtype)
        z = torch.addmm(self.w["proj2_b"], z, self.w["proj2_w"].t())
        return z.view(N, T - 1, self.text_hidden)

    def encode_images(self, images: list) -> torch.Tensor:
        px = torch.stack([preprocess_image(im, self.c["image_size"]) for im in images])
        return self.encode(px)
