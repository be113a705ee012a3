import torch,time
def t(f,n=20):
    for _ in range(3): f()
    torch.cuda.synchronize();t0=time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize();return (time.perf_counter()-t0)/n*1e6
a=torch.empty(256*1024*1024,device='cuda')  # 1 GB
a.uniform_()
us=t(lambda: a.sum()); print('sum 1GB contiguous: %.1f us %.2f TB/s'%(us,a.numel()*4/us/1e6))
us=t(lambda: torch.amax(a)); print('amax 1GB: %.1f us %.2f TB/s'%(us,a.numel()*4/us/1e6))
b=torch.empty_like(a)
us=t(lambda: b.copy_(a)); print('copy 1GB: %.1f us %.2f TB/s total'%(us,2*a.numel()*4/us/1e6))
us=t(lambda: b.fill_(1.0)); print('fill 1GB: %.1f us %.2f TB/s'%(us,a.numel()*4/us/1e6))
v=a.view(-1,256)
us=t(lambda: v.sum(dim=0)); print('colsum [1M,256]: %.1f us %.2f TB/s'%(us,a.numel()*4/us/1e6))
