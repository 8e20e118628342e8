"""Small-M MFMA GEMM (csrc/kernels/skinny_gemm.hip) against the fp32 PyTorch
reference: every launch configuration (column/row tile, split-K with the
in-launch ticket combine), ragged M, strided x, graph replay, and the model's
tuning pass."""
import pytest
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.ops import reference as ref


def test_skinny_configs_cpu():
    cfgs = ops.skinny_configs(128, 6144, 4096)
    assert (32, 32, 1) in cfgs and (64, 64, 8) in cfgs
    assert all(4096 % (s * 256) == 0 for _, _, s in cfgs)
    assert (128, 128, 8) in cfgs and (128, 64, 1) not in cfgs  # wide kernel: bm = M rounded up to 32
    assert ops.skinny_configs(300, 6144, 4096) == []  # M > 256: library only
    assert {s for _, _, s in ops.skinny_configs(64, 4096, 14336)} == {1, 2, 4, 8}  # 14336 = 256 * 56
    x = torch.randn(5, 256)
    w = torch.randn(64, 256)
    torch.testing.assert_close(ops.skinny_linear(x, w, (32, 32, 1)), x @ w.t())


def _check(M, N, K, cfg, dev, x_stride=None):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    xs = torch.randn(M, x_stride or K, generator=g).to(torch.bfloat16)
    x = xs[:, :K].to(dev)
    if x_stride is None:
        x = x.contiguous()
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    got = ops.skinny_linear(x, w, cfg).float().cpu()
    want = x.float().cpu() @ w.float().cpu().t()
    err = (got - want).abs().max().item()
    assert err <= 0.02 * want.abs().max().item() + 1e-3, (M, N, K, cfg, err)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 7, 32, 33, 64, 100, 128, 200, 256])
def test_skinny_all_configs_gpu(cuda, M):
    for N, K in ((256, 1024), (192, 2048)):
        for cfg in ops.skinny_configs(M, N, K):
            _check(M, N, K, cfg, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 4096), (4096, 14336), (28672, 4096)])
def test_skinny_llama_shapes_gpu(cuda, N, K):
    for M in (16, 128, 256):
        mp = -(-M // 32) * 32
        for cfg in [(32, 32, 1), (32, 64, 2), (64, 32, 4), (64, 64, 8), (32, 32, 8), (128, mp, 1), (128, mp, 4)]:
            if cfg in ops.skinny_configs(M, N, K):
                _check(M, N, K, cfg, cuda)


@pytest.mark.gpu
def test_skinny_strided_x_and_ticket_reset(cuda):
    _check(40, 128, 512, (32, 32, 2), cuda, x_stride=768)
    # every ticket is back to zero after split-K launches (graph replays rely on it)
    for _ in range(3):
        _check(96, 512, 2048, (64, 32, 8), cuda)
        _check(200, 512, 1024, (128, 224, 8), cuda)
    torch.cuda.synchronize()
    assert int(ops._skinny_ws(torch.device(cuda), ops._stream())[1].abs().sum()) == 0


@pytest.mark.gpu
def test_skinny_workspace_per_stream(cuda):
    """Split-K launches on two streams at once get separate slabs/tickets."""
    s1 = torch.cuda.Stream(cuda)
    with torch.cuda.stream(s1):
        ws1 = ops._skinny_ws(torch.device(cuda), ops._stream())
    ws0 = ops._skinny_ws(torch.device(cuda), ops._stream())
    assert ws0[0].data_ptr() != ws1[0].data_ptr() and ws0[1].data_ptr() != ws1[1].data_ptr()
    x = torch.randn(96, 2048, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(1024, 2048, device=cuda, dtype=torch.bfloat16) * 0.02
    ref = (x.float() @ w.float().T)
    s1.wait_stream(torch.cuda.current_stream())
    outs = []
    for i in range(4):
        st = s1 if i % 2 else torch.cuda.current_stream()
        with torch.cuda.stream(st):
            outs.append(ops.skinny_linear(x, w, (64, 32, 8)))
    torch.cuda.current_stream().wait_stream(s1)
    for o in outs:
        assert torch.allclose(o.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
@torch.inference_mode()  # as the engine captures (and the CUDA RNG state may already be an inference tensor)
def test_skinny_graph_replay(cuda):
    x = torch.randn(64, 4096, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(6144, 4096, device=cuda, dtype=torch.bfloat16) * 0.02
    out = torch.empty(64, 6144, device=cuda, dtype=torch.bfloat16)
    ops.skinny_linear(x, w, (32, 32, 4), out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.skinny_linear(x, w, (32, 32, 4), out=out)
    for _ in range(3):
        x.normal_()
        g.replay()
        torch.cuda.synchronize()
        want = ref.linear(x.cpu(), w.cpu()).float()
        assert (out.float().cpu() - want).abs().max() <= 0.02 * want.abs().max()


@pytest.mark.gpu
def test_model_tune_gemms_gpu(cuda):
    from dynamo_exp_amd.models.config import get_config
    from dynamo_exp_amd.models.llama import LlamaForCausalLM
    m = LlamaForCausalLM(get_config("small"), device=cuda).random_init(3)
    report = m.tune_gemms([1, 8, 64, 300])
    assert {r["key"][0] for r in report} == {1, 8, 64}
    for r in report:
        assert r["lib_us"] > 0 and (r["adopted"] == (r["key"] in m.gemm_plan))


@pytest.mark.gpu
def test_model_tune_prefill_gemms_gpu(cuda):
    """Prefill-size buckets routed to gemm256 give the library's result."""
    from dynamo_exp_amd.models.config import get_config
    from dynamo_exp_amd.models.llama import LlamaForCausalLM
    m = LlamaForCausalLM(get_config("small"), device=cuda).random_init(3)
    report = m.tune_prefill_gemms(2048, min_tokens=1024)
    assert {r["bucket"] for r in report} == {4, 5, 6, 7, 8}
    assert all(r["lib_us"] > 0 and r["gemm256_us"] > 0 for r in report)
    assert {(r["bucket"], r["N"], r["K"]) for r in report if r["adopted"]} == m.prefill_plan
    w = m.layers[0]["down"]
    x = torch.randn(1000, w.shape[1], device=cuda, dtype=torch.bfloat16)
    m.prefill_plan = {(4, w.shape[0], w.shape[1])}  # force the gemm256 route for M 769..1024
    got = m._mm(x, w).float()
    want = (x.float() @ w.float().t())
    assert (got - want).abs().max().item() <= 0.02 * want.abs().max().item()


# (round 2's LDS-DMA weight-streaming kernel was removed in round 4: the deep-stream
#  kernel below matches or beats it on every Llama-3-8B decode shape, profiles/r4_gemm_families.txt)

# ---- deep-stream kernel (csrc/kernels/dstream_gemm.hip)

def test_dstream_configs_cpu():
    cfgs = ops.dstream_configs(128, 4096, 4096)
    assert cfgs and all(c[0] == ops.DSTREAM and c[3] == 8 for c in cfgs)  # 128 tokens: one 8 x 16 tile
    assert {c[3] for c in ops.dstream_configs(100, 4096, 4096)} == {8}
    assert {c[3] for c in ops.dstream_configs(20, 4096, 4096)} == {2}
    # weight-ring depth divides the K steps of a slice; grids cover the chip
    for M, N, K in ((128, 4096, 14336), (256, 28672, 4096), (64, 6144, 4096)):
        for c in ops.dstream_configs(M, N, K):
            _, nw, r, t, dw, dx, s = c
            assert (K // 64 // s) % dw == 0 and 128 <= N // (nw * 16 * r) * s <= 2048
            assert dx * 16 * t * 128 + 1040 <= 160 * 1024
    assert ops.dstream_configs(300, 4096, 4096) == []
    x, w = torch.randn(40, 256), torch.randn(128, 256)
    torch.testing.assert_close(ops.skinny_linear(x, w, (ops.DSTREAM, 4, 1, 4, 4, 2, 1)), x @ w.t())
    assert ops.dstream_tune_configs(1, 6144, 4096) == []


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 16, 33, 64, 100, 128, 200, 256])
def test_dstream_all_configs_gpu(cuda, M):
    t = next(tt for tt in (2, 4, 8, 16) if 16 * tt >= M)
    # N 1344 = 7 x 192 = 12 x 112 = 28 x 48: every 3 / 6 / 7-wave row tile divides it
    for N, K in ((256, 1024), (512, 4096), (1344, 1024)):
        for nw, r, tt in sorted(ops.DSTREAM_SHAPES):
            if tt != t:
                continue
            for dw, dx in ops.DSTREAM_DEPTHS:
                for s in (1, 2, 4):
                    if ops._dstream_ok(M, N, K, nw, r, t, dw, dx, s):
                        _check(M, N, K, (ops.DSTREAM, nw, r, t, dw, dx, s), cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 4096), (4096, 14336), (28672, 4096)])
def test_dstream_llama_shapes_gpu(cuda, N, K):
    for M in (64, 128, 256):
        for cfg in ops.dstream_configs(M, N, K)[::3]:
            _check(M, N, K, cfg, cuda)


@pytest.mark.gpu
@torch.inference_mode()
def test_dstream_strided_x_graph_replay_and_ticket_reset(cuda):
    _check(72, 256, 1024, (ops.DSTREAM, 4, 1, 8, 4, 2, 4), cuda, x_stride=1536)
    _check(72, 256, 1024, (ops.DSTREAM, 8, 1, 8, 8, 4, 2), cuda, x_stride=1536)
    x = torch.randn(128, 4096, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(4096, 4096, device=cuda, dtype=torch.bfloat16) * 0.02
    out = torch.empty(128, 4096, device=cuda, dtype=torch.bfloat16)
    cfg = (ops.DSTREAM, 4, 1, 8, 8, 4, 4)
    ops.skinny_linear(x, w, cfg, out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.skinny_linear(x, w, cfg, out=out)
    for _ in range(3):
        x.normal_()
        g.replay()
        torch.cuda.synchronize()
        want = ref.linear(x.cpu(), w.cpu()).float()
        assert (out.float().cpu() - want).abs().max() <= 0.02 * want.abs().max()
    assert int(ops._skinny_ws(torch.device(cuda), ops._stream())[1].abs().sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("hidden,K,splits,t", [(4096, 4096, 4, 8), (4096, 14336, 8, 8), (8192, 8192, 2, 4),
                                               (4096, 4096, 2, 16)])
def test_dstream_partials_into_add_rmsnorm_bit_exact(cuda, hidden, K, splits, t):
    """dstream_linear(partial=True) leaves the split-K slabs; add_rmsnorm on
    them equals reduce-then-add_rmsnorm bit for bit (residual and output), and
    splitk_reduce equals the plain launch's output."""
    M = 16 * t - 5
    cfg = (ops.DSTREAM, 4, 1, t, 4, 2, splits)
    assert ops._dstream_ok(M, hidden, K, 4, 1, t, 4, 2, splits)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    w = (torch.randn(hidden, K, generator=g) * 0.02).to(cuda, torch.bfloat16)
    res = torch.randn(M, hidden, generator=g).to(cuda, torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(hidden, generator=g)).to(cuda, torch.bfloat16)
    y = ops.dstream_linear(x, w, cfg)
    r1 = res.clone()
    o1 = ops.add_rmsnorm(y.clone(), r1, gamma, 1e-5)
    p = ops.dstream_linear(x, w, cfg, partial=True)
    assert isinstance(p, ops.SplitK) and p.splits == splits and p.shape == (M, hidden)
    r2 = res.clone()
    o2 = ops.add_rmsnorm(p, r2, gamma, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(r1, r2) and torch.equal(o1, o2)
    p = ops.dstream_linear(x, w, cfg, partial=True)
    assert torch.equal(ops.splitk_reduce(p), y)


def _silu_ref(x, w_inter):
    """fp32 SwiGLU of a 32-row interleaved gate_up weight, on the CPU."""
    g_u = x.float().cpu() @ w_inter.float().cpu().t()
    return ref.silu_and_mul(g_u, ops.GEMM256_BLK)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 16, 64, 100, 128, 256])
def test_dstream_swiglu_form_gpu(cuda, M):
    """The deep-stream kernel's SwiGLU form (round 6, flags bit 1): gate / up
    rows interleaved in blocks of 32, r = 2, y[M, N / 2] = silu(g) * u --
    split-K included (splitk_reduce_silu_kernel) -- against an fp32 CPU
    reference, on a 5376-row weight (every wave count's tile divides it) and
    the Llama-3-8B gate_up shape."""
    torch.manual_seed(M)
    t = next(tt for tt in (2, 4, 8, 16) if 16 * tt >= M)
    for N, K in ((5376, 1024), (28672, 4096)):
        x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
        w = ref.interleave_gate_up(torch.randn(N, K, device=cuda, dtype=torch.bfloat16) * 0.02,
                                   ops.GEMM256_BLK).contiguous()
        want = _silu_ref(x, w)
        cfgs = [(ops.DSTREAM, nw, 2, t, dw, dx, s) for nw, r, tt in sorted(ops.DSTREAM_SHAPES) if r == 2 and tt == t
                for dw, dx in ops.DSTREAM_DEPTHS for s in (1, 2, 4)
                if ops._dstream_ok(M, N, K, nw, 2, t, dw, dx, s)]
        if N == 28672:
            cfgs = cfgs[::3]
        assert cfgs or M > 16 * 8, (M, N, K)
        for cfg in cfgs:
            got = ops.dstream_linear(x, w, cfg, silu=True).float().cpu()
            err = ((got - want).abs().max() / want.abs().max()).item()
            assert err < 2e-2, (cfg, err)
    with pytest.raises(ValueError):  # one 16-row block per wave cannot pair gate and up
        ops.dstream_linear(x, w, (ops.DSTREAM, 4, 1, t, 4, 2, 1), silu=True)
