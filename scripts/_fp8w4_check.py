import torch, sys
sys.path.insert(0, "/root/repo")
from pytorch_distributed_matmul_benchmark_amd.ops import gemm
FP8 = torch.float8_e4m3fn
def cm(x): return x.transpose(-1, -2).contiguous().transpose(-1, -2)
g = torch.Generator(device="cuda").manual_seed(1)
ok = True
for (M, N, K) in [(256, 256, 128), (512, 768, 256), (1000, 1052, 384), (300, 200, 128), (2304, 2048, 1024), (256, 256, 256)]:
    Af = torch.randint(-3, 4, (M, K), device="cuda", generator=g).float()
    Bf = torch.randint(-3, 4, (K, N), device="cuda", generator=g).float()
    C = gemm.matmul(Af.to(FP8), cm(Bf.to(FP8)), kernel="fp8_w4")
    ref = (Af.double() @ Bf.double()).to(torch.bfloat16)
    e = torch.equal(C, ref)
    ok &= e
    print(M, N, K, "exact" if e else f"MISMATCH maxdiff={(C.float()-ref.float()).abs().max().item()}", flush=True)
print("ALL OK" if ok else "FAIL")
