"""FP8 (e4m3fn w8a8) serving path: quantisation kernels vs the fp32 PyTorch
reference, fp8 GEMM, and the fp8 model against the bf16 model."""
import os

import pytest
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams
from dynamo_exp_amd.models.config import get_config
from dynamo_exp_amd.models.llama import AttnMeta, LlamaForCausalLM
from dynamo_exp_amd.ops import reference as ref


def _dequant(q, s):
    return q.float() * s.float()


# GPU vs CPU encodings of the same row may differ by one e4m3 step where the
# two scales differ in the last bit: at the top binade one step is 32/448 of
# the row maximum
TOL = 0.08


def test_quant_reference_roundtrip():
    y = torch.randn(7, 4096) * torch.linspace(0.01, 10, 7).view(-1, 1)
    q, s = ref.quant_fp8_rows(y)
    assert q.dtype == torch.float8_e4m3fn and s.shape == (7, 1)
    assert q.float().abs().amax(dim=1).max() <= 448
    rel = (_dequant(q, s) - y).abs().max() / y.abs().max()
    assert rel < 0.07  # e4m3: 3 mantissa bits


def _run(model, ids, dev):
    cfg = model.cfg
    bs, T = 16, ids.shape[0]
    nb = (T + bs - 1) // bs + 1
    kv = torch.zeros(cfg.num_hidden_layers, 2, nb, model.n_kv, bs, model.head_dim, dtype=torch.bfloat16, device=dev)
    caches = [(kv[i, 0], kv[i, 1]) for i in range(cfg.num_hidden_layers)]
    bt = torch.arange(1, nb, dtype=torch.int32).view(1, -1)
    pos = torch.arange(T)
    slots = bt[0].long()[pos // bs] * bs + pos % bs
    meta = AttnMeta(True, pos.to(dev), slots.to(dev), bt.to(dev), torch.tensor([T], dtype=torch.int32, device=dev),
                    logits_idx=torch.tensor([T - 1], device=dev),
                    cu_seqlens_q=torch.tensor([0, T], dtype=torch.int32, device=dev))
    return model.compute_logits(model.forward(ids.to(dev), meta, caches)).float().cpu()


def _cos(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()


def test_fp8_model_cpu_tracks_bf16():
    cfg = get_config("small")
    m = LlamaForCausalLM(cfg, device="cpu").random_init(4)
    ids = torch.randint(0, cfg.vocab_size, (40,))
    base = _run(m, ids, "cpu")
    m.quantize_fp8()
    assert m.fp8 and "qkv" not in m.layers[0] and m.layers[0]["qkv_q"].dtype == torch.float8_e4m3fn
    q = _run(m, ids, "cpu")
    assert _cos(base, q) > 0.98


def test_fp8_engine_cpu():
    eng = LLMEngine(EngineConfig(model="small", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64,
                                 max_num_seqs=4, use_cuda_graph=False, quantization="fp8"))
    out = []
    eng.add_request("a", list(range(5, 60)), SamplingParams(max_tokens=4, ignore_eos=True),
                    on_output=lambda r, t, lp, fin: out.extend(t))
    while eng.has_unfinished():
        eng.step()
    assert len(out) == 4
    with pytest.raises(ValueError):
        LLMEngine(EngineConfig(model="small", device="cpu", num_gpu_blocks=8, max_model_len=64, quantization="int3"))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("hidden", [1024, 4096, 1000, 8192])
def test_rmsnorm_quant_gpu(cuda, hidden):
    T = 37
    x = torch.randn(T, hidden, device=cuda, dtype=torch.bfloat16)
    r = torch.randn(T, hidden, device=cuda, dtype=torch.bfloat16)
    w = (torch.rand(hidden, device=cuda) + 0.5).to(torch.bfloat16)
    r_ref = r.clone().cpu()
    q, s = ops.rmsnorm_quant(x, r, w, 1e-5)
    qe, se = ops.rmsnorm_quant(x.cpu(), r_ref, w.cpu(), 1e-5)
    torch.testing.assert_close(r.cpu(), r_ref)  # residual updated in place identically
    torch.testing.assert_close(s.cpu(), se, rtol=1e-2, atol=1e-6)
    d, de = _dequant(q.cpu(), s.cpu()), _dequant(qe, se)
    assert (d - de).abs().max() <= TOL * de.abs().max()
    # no residual (first layer)
    q0, s0 = ops.rmsnorm_quant(x, None, w, 1e-5)
    q0e, s0e = ops.rmsnorm_quant(x.cpu(), None, w.cpu(), 1e-5)
    assert (_dequant(q0.cpu(), s0.cpu()) - _dequant(q0e, s0e)).abs().max() <= TOL * _dequant(q0e, s0e).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("ffn", [14336, 2816, 1000, 28672, 20000])
def test_silu_mul_quant_and_quant_rows_gpu(cuda, ffn):
    T = 19
    gu = torch.randn(T, 2 * ffn, device=cuda, dtype=torch.bfloat16)
    q, s = ops.silu_mul_quant(gu)
    qe, se = ops.silu_mul_quant(gu.cpu())
    de = _dequant(qe, se)
    assert (_dequant(q.cpu(), s.cpu()) - de).abs().max() <= TOL * de.abs().max()
    x = torch.randn(T, ffn, device=cuda, dtype=torch.bfloat16) * 3
    q, s = ops.quant_rows(x)
    assert (_dequant(q.cpu(), s.cpu()) - x.float().cpu()).abs().max() <= TOL * x.float().abs().max().cpu()
    # exact agreement of the encodings with PyTorch's e4m3fn cast away from ties
    qe, se = ref.quant_fp8_rows(x.cpu())
    assert (q.cpu().view(torch.uint8) == qe.view(torch.uint8)).float().mean() > 0.99


@pytest.mark.gpu
def test_fp8_linear_gpu(cuda):
    x = torch.randn(300, 4096, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(6144, 4096, device=cuda, dtype=torch.bfloat16) * 0.02
    x8, sx = ops.quant_rows(x)
    w8, sw = ref.quant_fp8_weight(w)
    sw = sw.view(1, -1).contiguous()
    got = ops.fp8_linear(x8, sx, w8, sw).float()
    exp = ref.fp8_linear(x8.cpu(), sx.cpu(), w8.cpu(), sw.cpu()).float()
    assert (got.cpu() - exp).abs().max() < 0.02 * exp.abs().max()
    assert _cos(got.cpu(), (x.float() @ w.float().t()).cpu()) > 0.995


@pytest.mark.gpu
def test_fp8_model_gpu_matches_cpu_and_bf16(cuda):
    cfg = get_config("small")
    g = LlamaForCausalLM(cfg, device=cuda).random_init(6)
    c = LlamaForCausalLM(cfg, device="cpu")
    c.layers = [{k: v.cpu() for k, v in L.items()} for L in g.layers]
    c.embed, c.norm, c.lm_head = g.embed.cpu(), g.norm.cpu(), g.lm_head.cpu()
    ids = torch.randint(0, cfg.vocab_size, (90,))
    base = _run(g, ids, cuda)
    g.quantize_fp8()
    c.quantize_fp8()
    lg, lc = _run(g, ids, cuda), _run(c, ids, "cpu")
    assert _cos(lg, lc) > 0.995
    assert _cos(lg, base) > 0.98


@pytest.mark.gpu
def test_fp8_engine_gpu_graphs(cuda):
    eng = LLMEngine(EngineConfig(model="small", device="cuda:0", block_size=16, max_model_len=1024, num_gpu_blocks=256,
                                 max_num_seqs=8, graph_sizes=(1, 2, 4, 8), quantization="fp8"))
    eng.warmup()
    outs = {}
    for i in range(5):
        eng.add_request(f"f{i}", list(range(20 + i, 200 + 9 * i)), SamplingParams(max_tokens=10, ignore_eos=True),
                        on_output=lambda r, t, lp, fin: outs.setdefault(r.request_id, []).extend(t))
    while eng.has_unfinished():
        eng.step()
    assert all(len(v) == 10 for v in outs.values())
