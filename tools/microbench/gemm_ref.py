import torch, time
def t(fn, it=30):
    for _ in range(3): fn()
    s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e)/it*1e3
for (M,N,K) in [(4200,256,2304),(4200,256,1024),(4200,1024,256),(4200,512,9216),(6272,512,4608),(6272,512,2048),(6272,2048,512),(8192,8192,8192)]:
    a=torch.randn(M,K,device='cuda').bfloat16(); b=torch.randn(N,K,device='cuda').bfloat16()
    us=t(lambda: a@b.t())
    print(M,N,K,'hipblaslt %.1f us  %.0f TF/s'%(us, 2*M*N*K/us/1e6), flush=True)
