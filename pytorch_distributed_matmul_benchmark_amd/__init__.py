"""MI355X-native distributed GEMM scaling benchmark.

Layers:
  ops/       hand-written gfx950 MFMA GEMM kernels (HIP), native timing loop, bindings
  parallel/  torchrun bring-up on RCCL, partitioning, event-ordered comm streams
  models/    workloads ("modes"): independent, batch_parallel, matrix_parallel,
             data_parallel, model_parallel, no_overlap / overlap / pipeline
  utils/     metrics, timing, reporting
  runner     the per-size driver behind every CLI entry point
"""
__version__ = "0.1.0"
