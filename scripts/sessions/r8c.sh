#!/bin/bash
# Round 6 session C (PDMB_EXPERIMENTS=1 build in the tree): does the 16k bf16
# W4S clock follow the L2 / Infinity Cache hit rate? The
# shipping W4S against four tile orders of the same K-loop: XCD sub-blocks
# 8x4 (tall) and 2x16 (wide: 18 panels per K-step instead of 12, a lower L2
# hit), 16x16 rounds in snake order and sweeping M fastest (Infinity Cache
# reuse between rounds). Bitwise check of every arm against W4S, interleaved
# timing at the power cap (power_attrib.py), then PMC passes (GRBM clock,
# MFMA busy, L2 hit / misses) per arm.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8c; mkdir -p $OUT
ARMS=w4s,x_w4s_tall,x_w4s_wide,x_w4s_snake,x_w4s_mcol
echo "== build $(date +%T)"
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== bitwise $(date +%T)"
timeout -k 10 120 python - > $OUT/bitwise.log 2>&1 <<'PY' || exit $?
import torch
from pytorch_distributed_matmul_benchmark_amd.ops import gemm
n = 16384
torch.manual_seed(0)
A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
ref = gemm.matmul(A, B, kernel="w4s")
ok = True
for k in ["x_w4s_tall", "x_w4s_wide", "x_w4s_snake", "x_w4s_mcol"]:
    C = torch.full_like(ref, float("nan"))
    gemm.matmul(A, B, out=C, kernel=k)
    eq = torch.equal(C, ref)
    ok &= eq
    print(k, "bitwise_equal_to_w4s", eq, flush=True)
rows = torch.arange(0, n, 997, device="cuda")
err = (ref[rows].float() - (A[rows].float() @ B.float())).abs().max().item()
print("w4s_vs_fp32_rows_maxabs", err)
assert ok
PY
cat $OUT/bitwise.log
echo "== power $(date +%T)"
timeout -k 10 400 python scripts/power_attrib.py --arms $ARMS --rounds 4 --seconds 2 > $OUT/power.log 2>&1; rc=$?
grep '^{' $OUT/power.log > $OUT/power.jsonl; cut -c1-250 $OUT/power.jsonl; [ $rc -eq 0 ] || exit $rc
echo "== pmc $(date +%T)"
OUT=$OUT/pmc KS=$ARMS REPS=3 timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1; rc=$?
tail -5 $OUT/pmc.log; exit $rc
