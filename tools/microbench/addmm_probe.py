import torch, json, sys
sys.path.insert(0, '/root/repo')
from tools.microbench.conv_tiles import timeit
dev = 'cuda'
for M, K, N in [(33600, 1024, 256), (4200, 1024, 256), (33600, 256, 1024)]:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    r = {'M': M, 'K': K, 'N': N}
    r['linear_us'] = round(timeit(lambda: torch.nn.functional.linear(x, w)), 1)
    r['addmm_act_us'] = round(timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False)), 1)
    r['linear_bias_relu_us'] = round(timeit(lambda: torch.relu(torch.nn.functional.linear(x, w, b))), 1)
    y = torch._addmm_activation(b, x, w.t(), use_gelu=False)
    ref = torch.relu(x.float() @ w.float().t() + b.float())
    r['err'] = float((y.float() - ref).abs().max() / ref.abs().max())
    print(json.dumps(r), flush=True)
