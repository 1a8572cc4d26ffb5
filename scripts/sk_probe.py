import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from pytorch_distributed_matmul_benchmark_amd.ops import gemm
M=N=K=5120
torch.manual_seed(0)
A,_=gemm.fp8_quantize(torch.randn(M,K,device="cuda"))
B,_=gemm.fp8_quantize(torch.randn(K,N,device="cuda"),colmajor=True)
C=torch.empty(M,N,device="cuda",dtype=torch.bfloat16)
for mode in ("0","1","2"):
    os.environ["PDMB_STREAMK"]=mode
    for _ in range(20): gemm.matmul(A,B,out=C)
    torch.cuda.synchronize()
print("done")
