import torch, time
print(torch.__version__, torch.cuda.get_device_name(0))
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e)/it*1e3
for M in (8192, 128):
  for (K,N) in ((4096,6144),(4096,28672),(14336,4096),(4096,4096)):
    a = torch.randn(M,K,device='cuda').to(torch.bfloat16)
    w = (torch.randn(N,K,device='cuda')*0.02).to(torch.bfloat16)
    t_bf = bench(lambda: a@w.t())
    res = {"M":M,"K":K,"N":N,"bf16_us":round(t_bf,1),"bf16_TF":round(2*M*N*K/t_bf/1e6)}
    for dt in (torch.float8_e4m3fn, torch.float8_e4m3fnuz):
        try:
            a8 = a.to(dt); w8 = w.to(dt)
            st = torch.tensor(1.0, device='cuda')
            t = bench(lambda: torch._scaled_mm(a8, w8.t(), scale_a=st, scale_b=st, out_dtype=torch.bfloat16))
            res[str(dt)+"_tensor_us"] = round(t,1); res[str(dt)+"_TF"]=round(2*M*N*K/t/1e6)
            sa = torch.ones(M,1,device='cuda'); sb = torch.ones(1,N,device='cuda')
            t = bench(lambda: torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16))
            res[str(dt)+"_rowwise_us"] = round(t,1); res[str(dt)+"_rowTF"]=round(2*M*N*K/t/1e6)
        except Exception as ex:
            res[str(dt)] = repr(ex)[:200]
    print(res, flush=True)
