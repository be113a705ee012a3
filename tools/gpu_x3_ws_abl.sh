#!/bin/bash
# Ablation of the warp-specialised 1x1 (TCAMD_X3_WS_DBG: 1 no MFMA, 2 no stores, 3 neither).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for K in 64 256; do
  for D in 0 1 2 3; do
    echo -n "k=$K dbg=$D "
    TCAMD_X3_WS_DBG=$D timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw 56 --k $K --imgs 128 --iters 30 2>&1 | grep conv1x1 || exit 1
  done
done
echo -n "torch copy 411MB: "
timeout -k 10 60 python3 -c "
import torch,time
a=torch.empty(401408*256,device='cuda');b=torch.empty_like(a)
for _ in range(3): b.copy_(a)
torch.cuda.synchronize();t=time.perf_counter()
for _ in range(20): b.copy_(a)
torch.cuda.synchronize();us=(time.perf_counter()-t)/20*1e6
print('%.1f us %.2f TB/s'%(us,2*a.numel()*4/us/1e6))
" 2>&1 | grep TB || exit 1
echo -n "torch strided read 128B of 1KB rows: "
timeout -k 10 60 python3 -c "
import torch,time
a=torch.empty(401408,256,device='cuda')
v=a[:,:64]
for _ in range(3): s=v.sum(dim=1)
torch.cuda.synchronize();t=time.perf_counter()
for _ in range(20): s=v.sum(dim=1)
torch.cuda.synchronize();us=(time.perf_counter()-t)/20*1e6
print('%.1f us %.2f TB/s (read 103MB)'%(us,v.numel()*4/us/1e6))
" 2>&1 | grep TB || exit 1
