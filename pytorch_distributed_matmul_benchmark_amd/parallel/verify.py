"""Self-checks of a multi-rank run: is what a collective delivered the right data?

The reference gates its scaling run on a collective self-test
(matmul_scaling_benchmark.py:26-57, gated at :388-394) and states a result
check's intent in ``validate_result`` (:240-249), but never checks what the
timed collectives of its modes (:150 all_reduce, :221 all_gather) returned.
Here every number a multi-GPU run reports is checked:

* ``check_collective`` — before ``pick_collective`` times a candidate
  implementation (RCCL, the direct P2P exchange, the xGMI peer-memory pull),
  it runs it on RANK-CODED payloads (``payload``: small integers, exact in
  bf16 / fp16 / fp32 and in every partial sum a ring or two-shot reduction
  forms) and compares the output BITWISE with the expected gather / sum. Two
  payloads in a row, so an implementation that hands back the previous call's
  bytes (a pull that reads a peer's buffer before the peer's producer is
  visible) fails the second one. A candidate wrong on any rank is dropped on
  every rank.
* ``digest`` — an exact, position-weighted int64 fingerprint of a tensor's
  bits (each element's bit pattern times a position weight, summed in int64),
  so an all-gather's blocks can be compared with their producers' local
  outputs across ranks bitwise without moving the tensors.
* ``ref_rows`` / ``rows_error`` — sampled rows of a GEMM recomputed in fp32
  (broadcast products of the upcast operands summed over K: no library GEMM)
  against the kernel's output: the GEMM side of bench.py's per-mode check
  (``Workload.verify``).

Nothing here runs inside a timed region.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch

_INT = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
_MASK = {1: 0xFF, 2: 0xFFFF, 4: 0xFFFFFFFF}
_WEIGHT_MOD = 8191          # position weights 1..8191 (a prime modulus)
_CHUNK = 1 << 24            # elements per digest pass (bounded scratch)


def payload_half(ws: int) -> int:
    """Largest |value| of a payload element at world size ``ws``: the sum of
    ws elements (and every partial sum) stays an integer of magnitude <= 255,
    exact in bf16 (8 significant bits), fp16 and fp32."""
    return max(1, min(15, 255 // max(ws, 1)))


def payload(shape: Sequence[int], rank: int, seed: int, ws: int, dtype: torch.dtype,
            device: torch.device) -> torch.Tensor:
    """Rank-coded test data: element [i, j] (the leading dims flattened into
    rows) = ((rank * 7 + seed * 3 + 5 * i + j) mod M) - h with h =
    ``payload_half(ws)``, M = 2h + 1. Distinct ranks give distinct blocks
    (rank * 7 mod M differs for the ranks of one job while ws < M)."""
    shape = tuple(int(s) for s in shape)
    h = payload_half(ws)
    M = 2 * h + 1
    cols = shape[-1] if shape else 1
    rows = 1
    for s in shape[:-1]:
        rows *= s
    r = (torch.arange(rows, device=device, dtype=torch.int64) * 5 + rank * 7 + seed * 3) % M
    c = torch.arange(cols, device=device, dtype=torch.int64) % M
    v = (r.view(-1, 1).to(torch.int32) + c.view(1, -1).to(torch.int32)) % M - h
    return v.to(dtype).view(shape)


def expected_sum(shape: Sequence[int], seed: int, ws: int, dtype: torch.dtype,
                 device: torch.device) -> torch.Tensor:
    """Σ over ranks of ``payload(shape, rank, seed, ws)`` (exact)."""
    acc = None
    for r in range(ws):
        p = payload(shape, r, seed, ws, torch.int32, device)
        acc = p if acc is None else acc.add_(p)
    return acc.to(dtype)


def digest(x: torch.Tensor) -> int:
    """Exact int64 fingerprint of ``x``'s bits in logical (row-major) order:
    Σ_i bits(x_i) * (i mod 8191 + 1), wrapping in int64. Equal tensors give
    equal digests on any device; a changed element changes it unless the
    change is a multiple of 2^64 / weight (never, for one element)."""
    flat = x.reshape(-1)
    es = flat.element_size()
    if es not in _MASK:
        raise ValueError(f"digest: unsupported element size {es}")
    bits = flat.view(_INT[es])
    total = torch.zeros((), dtype=torch.int64, device=x.device)
    n = bits.numel()
    for s in range(0, n, _CHUNK):
        e = min(n, s + _CHUNK)
        w = torch.arange(s, e, device=x.device, dtype=torch.int64) % _WEIGHT_MOD + 1
        total += (bits[s:e].to(torch.int64) & _MASK[es]).mul_(w).sum()
    return int(total.item())


def flip_sign_(x: torch.Tensor) -> torch.Tensor:
    """x <- -x, exactly, for any float dtype (fp8 included: the sign bit is
    flipped through an integer view; a GEMM of -A and B is then exactly the
    negation of A @ B, whatever the accumulation order)."""
    es = x.element_size()
    sign = {1: 0x80, 2: -0x8000, 4: -0x80000000}[es]
    x.view(_INT[es]).bitwise_xor_(sign)
    return x


def sample_rows(m: int, count: int = 24) -> List[int]:
    """``count`` row indices spread over [0, m): first, last and evenly between."""
    if m <= count:
        return list(range(m))
    step = (m - 1) / (count - 1)
    return sorted({int(round(i * step)) for i in range(count)})


def ref_rows(A: torch.Tensor, B: torch.Tensor, rows: Sequence[int], budget_bytes: int = 256 << 20) -> torch.Tensor:
    """fp32 reference of rows ``rows`` of A @ B (A [m, k], B [k, n]; any
    strides, fp8 included) WITHOUT a library GEMM: broadcast products summed
    over k (torch's elementwise and reduction kernels), in column chunks of B
    that keep the [rows, k, chunk] product under ``budget_bytes``. A vendor GEMM
    here would put a hipBLASLt kernel into every bench.py run, which the
    provenance check (tests/test_provenance_gpu.py) forbids."""
    idx = torch.tensor(list(rows), device=A.device, dtype=torch.long)
    if A.element_size() == 1:  # fp8: gather the rows' bytes (index_select has no fp8 kernel)
        a = A.view(torch.uint8).index_select(0, idx).view(A.dtype).float()
    else:
        a = A.index_select(0, idx).float()
    k, n = B.shape[-2], B.shape[-1]
    r = max(len(rows), 1)
    chunk = max(1, min(n, budget_bytes // (4 * r * max(k, 1))))
    out = torch.empty(len(rows), n, device=A.device, dtype=torch.float32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[:, s:e] = (a.unsqueeze(2) * B[:, s:e].float().unsqueeze(0)).sum(dim=1)
    return out


def rows_of(C: torch.Tensor, rows: Sequence[int]) -> torch.Tensor:
    idx = torch.tensor(list(rows), device=C.device, dtype=torch.long)
    return C.index_select(0, idx).float()


# Relative tolerance of a checked GEMM / reduced output against the fp32
# reference, by OUTPUT dtype, as a fraction of the sample's largest magnitude
# (a wrong, stale or sign-flipped block is off by O(1) of it).
REL_TOL = {torch.bfloat16: 2.0 ** -6, torch.float16: 2.0 ** -9, torch.float32: 1e-4}


def rows_error(got: torch.Tensor, ref: torch.Tensor, scale: Optional[torch.Tensor] = None) -> float:
    """max |got - ref| / max(scale) (``scale`` defaults to |ref|); NaN -> inf."""
    if not torch.isfinite(got).all():
        return float("inf")
    den = float((scale if scale is not None else ref.abs()).max().item()) if ref.numel() else 0.0
    err = float((got - ref).abs().max().item()) if ref.numel() else 0.0
    return err / den if den > 0 else err


def check_collective(kind: str, rank: int, ws: int, t: torch.Tensor, out: Optional[torch.Tensor],
                     call: Callable[[], None], sync: Callable[[], None], seeds=(1, 2),
                     corrupt: Optional[Callable[[torch.Tensor], None]] = None) -> Optional[str]:
    """Run ``call`` (one collective of ``t``: all_reduce in place, all_gather
    into ``out``) on rank-coded payloads and compare bitwise. Returns None
    (correct on this rank) or what was wrong. ``corrupt`` (test-only negative
    control) damages the result before the comparison. Not collective by
    itself beyond ``call``: agree on the answer with ``all_ok``."""
    dev = t.device
    wrong = None  # every seed's call runs on every rank (it is a collective), wrong or not
    for seed in seeds:
        t.copy_(payload(t.shape, rank, seed, ws, t.dtype, dev))
        sync()
        call()
        sync()
        res = t if kind == "all_reduce" else out
        if corrupt is not None:
            corrupt(res)
        if wrong is not None:
            continue
        if kind == "all_reduce":
            exp = expected_sum(t.shape, seed, ws, t.dtype, dev)
            if not torch.equal(t, exp):
                bad = int((t != exp).sum().item())
                wrong = f"all_reduce payload {seed}: {bad} of {t.numel()} elements wrong"
        else:
            rows = t.shape[0]
            for j in range(ws):
                exp = payload(t.shape, j, seed, ws, t.dtype, dev)
                if not torch.equal(out[j * rows:(j + 1) * rows], exp):
                    wrong = f"all_gather payload {seed}: block of rank {j} wrong"
                    break
    return wrong
