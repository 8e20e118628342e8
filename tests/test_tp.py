"""Tensor parallelism on CPU (gloo, world 2): sharded model logits equal the
unsharded model's, and the SPMD replicated engines stay in lockstep."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from dynamo_exp_amd.models.config import get_config
from dynamo_exp_amd.models.llama import AttnMeta, LlamaForCausalLM, TPGroup


def _logits(model, ids):
    cfg = model.cfg
    bs, nb = 16, 32
    T = ids.numel()
    kv = torch.zeros(cfg.num_hidden_layers, 2, nb, model.n_kv, bs, model.head_dim, dtype=torch.bfloat16)
    caches = [(kv[i, 0], kv[i, 1]) for i in range(cfg.num_hidden_layers)]
    bt = torch.arange(0, (T + bs - 1) // bs, dtype=torch.int32).view(1, -1)
    pos = torch.arange(T)
    meta = AttnMeta(True, pos, bt[0].long()[pos // bs] * bs + pos % bs, bt, torch.tensor([T], dtype=torch.int32),
                    logits_idx=torch.tensor([T - 1]), cu_seqlens_q=torch.tensor([0, T], dtype=torch.int32))
    return model.compute_logits(model.forward(ids, meta, caches)).float()


def _worker(rank, world, port, q):
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    cfg = get_config("small")
    full = LlamaForCausalLM(cfg, device="cpu").random_init(11)
    shard = LlamaForCausalLM(cfg, device="cpu", tp=TPGroup(dist.group.WORLD, rank, world)).load_shard_from(full)
    ids = torch.arange(40, 140)
    lg = _logits(shard, ids)
    if rank == 0:
        ref = _logits(full, ids)
        q.put(((lg - ref).abs().max().item(), ref.abs().max().item()))
    dist.destroy_process_group()


def test_tp2_logits_match():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29561
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    err, scale = q.get(timeout=240)
    [p.join(60) for p in ps]
    assert err < 0.03 * scale + 0.05, (err, scale)
